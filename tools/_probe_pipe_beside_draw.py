"""Probe (diagnostic build): does the config-4 pipeline slow down beside the RANSAC draw for the draw's resources
(LDS, registers, wave slots) or for its work? Batch A runs the pipeline; batch B (another stream) runs the batched
RANSAC launched just before it: the real draw, or (SVX_RANSAC_ABLATE=128) a draw whose waves hold their resources
for 4 ms and draw nothing. The pipeline's own HIP-event time is reported for each case."""
import os, sys, statistics, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd"), os.path.join(REPO, "tests")]
os.environ.setdefault("SVX_LIB", os.path.join(REPO, "stereo.vision_amd/svx/_lib/libsvx_diag.so"))
from svx import batch as sb
from test_prepass_cpu import carmask
F = int(os.environ.get("PROBE_FRAMES", 4096))
A = sb.Batch(F, step=1, with_bgr=True, with_points=True)
A.synth(0)
LOOPVAR = os.environ.get("PROBE_LOOP_PIPE") == "1"   # the frame loop's pipeline: per-frame planes + road bitmap
if LOOPVAR:
    A.set_mask(carmask())
    A.prepass("previous", sync=True)
    A.ransac(seed_base=0, trials=600, sync=True)
    A.road_bits(True)
run_pipe = (lambda: A.pipeline_planes(sync=False)) if LOOPVAR else (lambda: A.pipeline(sync=False))
B = sb.Batch(F, step=1, with_bgr=False)
B.synth(0)
B.set_mask(carmask())
B.prepass("previous", sync=True)
for _ in range(2):
    run_pipe(); A.sync()
    B.ransac(seed_base=0, trials=600, sync=True)
res = {}
for r in range(5):
    for mode in ("alone", "real_draw", "sleeping_draw", "real_draw_counts", "sleeping_draw_counts"):
        os.environ["SVX_RANSAC_ABLATE"] = "128" if mode.startswith("sleeping") else "0"
        # _counts: the draw's LDS sized from the frames' counts read back instead of the mask's bound
        os.environ["SVX_RANSAC_BOUND"] = "0" if mode.endswith("_counts") else "1"
        A.sync(); B.sync()
        A.reset_timing()
        if mode != "alone":
            B.ransac(seed_base=0, trials=600, sync=False)
            time.sleep(0.0015)   # maskpoints (~0.6 ms) done and the draw's waves resident before the pipeline
        run_pipe()
        A.sync(); B.sync()
        ms, n = A.timing("pipeline")
        res.setdefault(mode, []).append(ms / n)
os.environ["SVX_RANSAC_ABLATE"] = "0"
for mode, t in res.items():
    print(f"{mode:14s} pipeline {statistics.median(t):7.3f} ms (min {min(t):.3f}, max {max(t):.3f})", flush=True)
A.close(); B.close()
