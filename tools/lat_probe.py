"""DIAGNOSTIC: 1-frame K1 latency per instance (tune nontemporal 0/1/2) and the 4096-frame K1 time."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "stereo.vision_amd")]
from svx import batch as sb
for rep in range(2):
    for nt in (1, 2, 0):
        with sb.Batch(1, 544, 1024, 1, with_bgr=False) as one:
            one.tune(1, nt)
            one.synth(0)
            for _ in range(5):
                one.project(sync=False)
            one.reset_timing()
            for _ in range(50):
                one.project(sync=False)
            ms, n = one.timing("project")
            print("nt", nt, "latency us", round(ms / n * 1e3, 2), flush=True)
b = sb.Batch(4096, 544, 1024, 1, with_bgr=False)
b.synth(0)
for _ in range(3): b.project(sync=True)
b.reset_timing()
for _ in range(10): b.project(sync=False)
ms, n = b.timing("project"); print("K1 4096 ms", round(ms/n, 4))
