"""Probe: the batched RANSAC alone on 4096 carmask frames (kernel times under rocprofv3 --kernel-trace)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd"), os.path.join(REPO, "tests")]
from svx import batch as sb
from test_prepass_cpu import carmask
F = int(os.environ.get("PROBE_FRAMES", 4096))
with sb.Batch(F, step=1, with_bgr=True, with_points=True) as rb:
    rb.synth(0); rb.set_mask(carmask()); rb.prepass("previous")
    rb.ransac(seed_base=0, trials=600)
    t0 = time.perf_counter()
    for _ in range(5):
        rb.ransac(seed_base=0, trials=600, sync=False)
    rb.sync()
    print(f"ransac: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms", flush=True)
