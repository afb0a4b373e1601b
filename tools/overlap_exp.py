#!/usr/bin/env python3
"""Experiment: do K1 (pure write stream) and the pipeline overlap when run
concurrently on two streams? Prints wall times of each alone and both."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd")]
from svx import batch as sb

a = sb.Batch(2048, with_bgr=False)
b = sb.Batch(2048, with_bgr=True, with_points=True)
a.synth(0); b.synth(5000)
def wall(fn, reps=10):
    fn(); a.sync(); b.sync()
    t = time.perf_counter()
    for _ in range(reps): fn()
    a.sync(); b.sync()
    return (time.perf_counter() - t) / reps * 1e3
k1 = wall(lambda: a.project(sync=False))
pp = wall(lambda: b.pipeline(sync=False))
both = wall(lambda: (a.project(sync=False), b.pipeline(sync=False)))
print(f"K1 alone {k1:.3f} ms, pipeline alone {pp:.3f} ms, both concurrently {both:.3f} ms (sum {k1+pp:.3f})")
