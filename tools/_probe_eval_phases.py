"""Probe (diagnostic build, SVX_RANSAC_ABLATE=32): where the batched RANSAC evaluation's time goes, per phase, from
each workgroup's wall-clock stamps at the barriers that end the phases (kernels/ransac_batch.hip g_eval_phase)."""
import ctypes, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd"), os.path.join(REPO, "tests")]
os.environ.setdefault("SVX_LIB", os.path.join(REPO, "stereo.vision_amd/svx/_lib/libsvx_diag.so"))
os.environ["SVX_RANSAC_ABLATE"] = "32"
from svx import _abi, batch as sb
from test_prepass_cpu import carmask
lib = _abi.lib()
F = int(os.environ.get("PROBE_FRAMES", 4096))
buf = (ctypes.c_ulonglong * 8)()
names = ["LDS fill", "plane solves", "screen", "compaction", "candidates fp64", "decision"]
with sb.Batch(F, step=1, with_bgr=True, with_points=True) as rb:
    rb.synth(0); rb.set_mask(carmask()); rb.prepass("previous")
    rb.ransac(seed_base=0, trials=600)
    rb.sync()
    lib.sv_diag_eval_phases(buf, 1)
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        rb.ransac(seed_base=0, trials=600, sync=False)
    rb.sync()
    print(f"ransac (with stamps): {(time.perf_counter() - t0) / reps * 1e3:.3f} ms per call", flush=True)
    lib.sv_diag_eval_phases(buf, 1)
    wgs = buf[6]
    tot = sum(buf[i] for i in range(6))
    print(f"workgroups stamped {wgs} ({wgs / reps:.0f} a call)")
    for i, n in enumerate(names):
        print(f"  {n:18s} {buf[i] * 10 / wgs / 1e3:8.2f} us per workgroup ({100 * buf[i] / tot:5.1f} %)")
    print(f"  {'total':18s} {tot * 10 / wgs / 1e3:8.2f} us per workgroup; x frames / 256 CUs = "
          f"{tot * 10 / wgs / 1e6 * F / 256:.3f} ms at one workgroup a CU")
