#!/usr/bin/env python3
"""Tail-quantisation probe: pipeline and K1 ms per frame at several batch sizes
(one workgroup per frame; 256 CUs x 5 workgroups = 1280 slots, so 3840 frames
are exactly 3 rounds and 4096 are 3.2). Prints one JSON line per size."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd")]
from svx import batch as sb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1280,2560,3840,4096,5120")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--mode", default="resident")
    ap.add_argument("--planes", action="store_true", help="also time the per-frame-plane pipeline")
    a = ap.parse_args()
    for n in (int(s) for s in a.sizes.split(",")):
        with sb.Batch(n, step=1, with_bgr=True, with_points=True) as b:
            b.synth(0)
            b.pipeline_mode(a.mode)
            res = {"frames": n}
            for what in ("k1", "pipe") + (("planes",) if a.planes else ()):
                if what == "planes":
                    b.ransac(seed_base=0, trials=600)
                fn = {"k1": lambda: b.project(sync=False), "pipe": lambda: b.pipeline(sync=False),
                      "planes": lambda: b.pipeline_planes(sync=False)}[what]
                for _ in range(2):
                    fn()
                b.sync()
                b.reset_timing()
                for _ in range(a.reps):
                    fn()
                b.sync()
                ms, cnt = b.timing("project" if what == "k1" else "pipeline")
                res[what + "_ms"] = round(ms / cnt, 4)
                res[what + "_us_per_frame"] = round(ms / cnt / n * 1e3, 3)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
