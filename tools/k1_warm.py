"""DIAGNOSTIC: K1 4096-frame launch time over ~12 s of continuous load (clock / power ramp)."""
import sys
import time
sys.path[:0] = [sys.argv[1] if len(sys.argv) > 1 else "stereo.vision_amd"]
from svx import batch as sb
b = sb.Batch(4096, 544, 1024, 1, with_bgr=False)
b.synth(0)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 12:
    b.reset_timing()
    for _ in range(20):
        b.project(sync=False)
    ms, n = b.timing("project")
    print(f"t={time.perf_counter() - t0:5.1f}s K1 {ms / n:.4f} ms", flush=True)
