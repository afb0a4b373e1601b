"""Probe: the road pass from the pipeline's bitmap, ms per 4096 frames (per-frame RANSAC planes, as bench.py's
road_from_bitmap). Diagnostic: run with SVX_LIB=<libsvx_diag.so> to let SVX_* knobs apply."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd"), os.path.join(REPO, "tests")]
from svx import batch as sb
from test_prepass_cpu import carmask
F = int(os.environ.get("PROBE_FRAMES", 4096))
with sb.Batch(F, step=1, with_bgr=True, with_points=True) as b:
    b.synth(0); b.set_mask(carmask()); b.prepass("previous", sync=True)
    b.ransac(seed_base=0, trials=600)
    b.road_bits(True)
    b.pipeline_planes(sync=True)
    for _ in range(3):
        b.road_raster(sync=False)
    b.sync()
    variants = os.environ.get("PROBE_RPW", "1").split(",")   # SVX_ROAD_RPW values, alternated in this process
    res = {v: [] for v in variants}
    for _ in range(5):
        for v in variants:
            os.environ["SVX_ROAD_RPW"] = v
            b.road_raster(sync=False)
            b.sync()
            t0 = time.perf_counter()
            for _ in range(5):
                b.road_raster(sync=False)
            b.sync()
            res[v].append((time.perf_counter() - t0) / 5 * 1e3)
    for v, r in res.items():
        print(f"road from bitmap RPW={v} NT={os.environ.get('SVX_ROAD_NT', '0')} IMG_NT={os.environ.get('SVX_ROAD_IMG_NT', '0')}: "
              f"min {min(r):.3f} median {sorted(r)[2]:.3f} ms per {F} frames", flush=True)
