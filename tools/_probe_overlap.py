"""Scratch probe: do a batch's RANSAC and another batch's pipeline run concurrently on two streams?"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd"), os.path.join(REPO, "tests")]
from svx import batch as sb
from test_prepass_cpu import carmask
F = 4096
a = sb.Batch(F, step=1, with_bgr=True, with_points=True); a.synth(0); a.set_mask(carmask()); a.prepass("previous", sync=True)
b = sb.Batch(F, step=1, with_bgr=True, with_points=True); b.synth(F); b.set_mask(carmask()); b.prepass("previous", sync=True)
for x in (a, b):
    x.ransac(seed_base=0, trials=600, sync=True); x.pipeline_planes(sync=True)
def t(name, fn, reps=5):
    fn(); a.sync(); b.sync()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    a.sync(); b.sync()
    print(f"{name:45s} {(time.perf_counter() - t0) / reps * 1e3:8.3f} ms", flush=True)
t("ransac(a)", lambda: a.ransac(seed_base=0, trials=600, sync=False))
t("pipeline_planes(b)", lambda: b.pipeline_planes(sync=False))
t("ransac(a) + pipeline_planes(b), two streams", lambda: (a.ransac(seed_base=0, trials=600, sync=False), b.pipeline_planes(sync=False)))
t("ransac(a) then pipeline_planes(a), one stream", lambda: (a.ransac(seed_base=0, trials=600, sync=False), a.pipeline_planes(sync=False)))
t("road(b)", lambda: (b.road_raster(sync=False), b.nonzero(sync=False)))
t("ransac(a) + road(b)", lambda: (a.ransac(seed_base=0, trials=600, sync=False), b.road_raster(sync=False), b.nonzero(sync=False)))
a.close(); b.close()
