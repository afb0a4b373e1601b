#!/usr/bin/env python3
"""A/B of two builds of libsvx on one box: each round runs one process per
library (SVX_LIB, diagnostic override in svx/_abi.py), alternating, and prints
the median kernel ms per library and workload.

usage: ab_lib.py --libs _ab/libsvx_base.so,stereo.vision_amd/svx/_lib/libsvx.so --what pipe,planes --rounds 3
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys
sys.path[:0] = [{repo!r}, {pkg!r}]
from svx import batch as sb
what, frames, reps = {what!r}, {frames}, {reps}
out = {{}}
with sb.Batch(frames, step=1, with_bgr=True, with_points=True) as b:
    b.synth(0)
    for w in what.split(","):
        if w == "planes":
            b.ransac(seed_base=0, trials=600)
        fn = {{"k1": lambda: b.project(sync=False), "pipe": lambda: b.pipeline(sync=False),
               "planes": lambda: b.pipeline_planes(sync=False)}}[w]
        for _ in range(2):
            fn()
        b.sync()
        b.reset_timing()
        for _ in range(reps):
            fn()
        b.sync()
        ms, n = b.timing("project" if w == "k1" else "pipeline")
        out[w] = ms / n
print(json.dumps(out))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--what", default="pipe")
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    libs = [os.path.join(REPO, l) for l in a.libs.split(",")]
    res = {l: [] for l in libs}
    code = CHILD.format(repo=REPO, pkg=os.path.join(REPO, "stereo.vision_amd"), what=a.what, frames=a.frames,
                        reps=a.reps)
    for r in range(a.rounds):
        for l in (libs if r % 2 == 0 else libs[::-1]):
            env = dict(os.environ, SVX_LIB=l)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stderr[-2000:], file=sys.stderr)
                sys.exit(p.returncode)
            res[l].append(json.loads(p.stdout.strip().splitlines()[-1]))
            print(os.path.basename(l), res[l][-1], flush=True)
    for l in libs:
        print(json.dumps({"lib": os.path.relpath(l, REPO),
                          **{w: round(statistics.median(x[w] for x in res[l]), 4) for w in a.what.split(",")}}))


if __name__ == "__main__":
    main()
