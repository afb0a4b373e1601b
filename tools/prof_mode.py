#!/usr/bin/env python3
"""Fixed pipeline workload for rocprofv3 PMC runs, one kernel family."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd")]
from svx import batch as sb  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="resident")
ap.add_argument("--frames", type=int, default=4096)
ap.add_argument("--reps", type=int, default=1)
ap.add_argument("--chunk", type=int, default=0)
a = ap.parse_args()
b = sb.Batch(a.frames, step=1, with_bgr=True, with_points=True)
b.pipeline_mode(a.mode)
b.synth(0)
for _ in range(a.reps):
    b.pipeline(chunk=a.chunk, sync=True)
b.close()
print("done")
