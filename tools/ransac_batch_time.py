"""Time sv_batch_ransac (maskpoints + per-frame RANSAC) on synthetic frames with the carmask."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "stereo.vision_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from svx import batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=1024)
ap.add_argument("--trials", type=int, default=600)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--ablate", default="0", help="SVX_RANSAC_ABLATE values to alternate (A/B in one process)")
a = ap.parse_args()
from test_prepass_cpu import carmask  # noqa: E402

mask = carmask()
with batch.Batch(a.frames, H=544, W=1024, step=2, with_bgr=False) as b:
    b.synth(0)
    b.set_mask(mask)
    b.ransac(seed_base=0, trials=2)
    for r in range(a.reps):
        for ab in a.ablate.split(","):
            os.environ["SVX_RANSAC_ABLATE"] = ab
            t0 = time.perf_counter()
            b.ransac(seed_base=r, trials=a.trials, sync=True)
            dt = time.perf_counter() - t0
            res = [b.read_ransac(f) for f in range(min(a.frames, 64))]
            fl = [x["flags"] for x in res]
            tr = [x["trial"] for x in res]
            print(f"ablate={ab} frames={a.frames} trials={a.trials} {dt*1e3:.1f} ms  {dt*1e3/a.frames:.3f} ms/frame "
                  f"flags(first 64)={sorted(set(fl))} trials(first 4)={tr[:4]}", flush=True)
