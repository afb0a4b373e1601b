#!/usr/bin/env python3
"""Small fixed workload for rocprofv3 runs: K1 and/or the pipeline on N frames."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd")]
from svx import batch as sb  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--what", default="k1,pipe")
ap.add_argument("--frames", type=int, default=4096)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--chunk", type=int, default=0)
a = ap.parse_args()
b = sb.Batch(a.frames, step=1, with_bgr="pipe" in a.what, with_points="pipe" in a.what)
b.synth(0)
for _ in range(a.reps):
    if "k1" in a.what:
        b.project(sync=True)
    if "pipe" in a.what:
        b.pipeline(chunk=a.chunk, sync=True)
b.close()
print("done")
