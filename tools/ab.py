#!/usr/bin/env python3
"""A/B timing of pipeline variants inside ONE process (box-to-box spread is
~10-15 %, so compare only within a run). Variants: SVX_ABLATE values and/or
pipeline modes, alternated round-robin; prints the median ms per variant.
DIAGNOSTIC: ablated runs produce invalid results.

usage: ab.py --ablate 0,128,8320 --modes resident,split:512,split:1024 --rounds 5 --reps 3
(a mode "split:L" runs the split schedule with SVX_SPLIT_LAG=L)
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd")]
from svx import batch as sb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ablate", default="0")
    ap.add_argument("--modes", default="resident")
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--k1", action="store_true", help="time K1 (project) instead of the pipeline")
    ap.add_argument("--with-k1", action="store_true", help="also time K1 (a per-box reference)")
    a = ap.parse_args()
    b = sb.Batch(a.frames, step=1, with_bgr=True, with_points=True)
    b.synth(0)
    variants = [(m, int(x)) for m in a.modes.split(",") for x in a.ablate.split(",")]
    if a.with_k1:   # K1 beside the variants: the box's HBM speed, to compare runs across boxes
        variants.append(("k1", 0))
    res = {v: [] for v in variants}
    for _ in range(a.rounds):
        for mode, abl in variants:
            os.environ["SVX_ABLATE"] = str(abl)
            m, _, lag = mode.partition(":")
            if lag:
                os.environ["SVX_SPLIT_LAG"] = lag
            k1 = a.k1 or m == "k1"
            if not k1:
                b.pipeline_mode(m)
            run = (lambda sync: b.project(sync=sync)) if k1 else (lambda sync: b.pipeline(sync=sync))
            run(True)
            b.reset_timing()
            for _ in range(a.reps):
                run(False)
            ms, n = b.timing("project" if k1 else "pipeline")
            res[(mode, abl)].append(ms / n)
    os.environ["SVX_ABLATE"] = "0"
    for (mode, abl), v in res.items():
        print(json.dumps({"mode": mode, "ablate": abl, "median_ms": round(statistics.median(v), 4),
                          "min_ms": round(min(v), 4), "max_ms": round(max(v), 4)}), flush=True)
    b.close()


if __name__ == "__main__":
    main()
