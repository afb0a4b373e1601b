#!/usr/bin/env python3
"""Launch-shape sweep on one GPU: K1 (grid cap, store flavour) and the pipeline
chunk size. Prints one line per variant (kernel ms from HIP events)."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd")]

from svx import batch as sb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--k1", default="1:1,2:1,4:1,1:0")
    ap.add_argument("--chunks", default="8,16,32,64")
    ap.add_argument("--step", type=int, default=1)
    ap.add_argument("--modes", default="tiled,resident")
    ap.add_argument("--rchunks", default="0", help="resident: frames per launch (0 = default)")
    a = ap.parse_args()
    b = sb.Batch(a.frames, step=a.step, with_bgr=True, with_points=True)
    b.synth(0)
    ng = b.Ng * a.frames
    res = []
    for v in a.k1.split(","):
        cap, nt = (int(t) for t in v.split(":"))
        b.tune(cap, nt)
        b.project(sync=True)
        b.reset_timing()
        for _ in range(a.reps):
            b.project(sync=False)
        ms, n = b.timing("project")
        ms /= n
        res.append({"k1_qpl": cap, "nt": nt, "ms": round(ms, 4),
                    "GBps": round(13 * ng / ms / 1e6, 1), "Gpts": round(ng / ms / 1e6, 1)})
        print(json.dumps(res[-1]), flush=True)
    for mode in a.modes.split(","):
        b.pipeline_mode(mode)
        for c in (a.chunks if mode == "tiled" else a.rchunks).split(","):
            c = int(c)
            b.pipeline(chunk=c, sync=True)
            b.reset_timing()
            for _ in range(a.reps):
                b.pipeline(chunk=c, sync=False)
            ms, n = b.timing("pipeline")
            ms /= n
            res.append({"mode": mode, "chunk": c, "pipeline_ms": round(ms, 4), "Gpts": round(ng / ms / 1e6, 1)})
            print(json.dumps(res[-1]), flush=True)
    b.close()


if __name__ == "__main__":
    main()
