#!/usr/bin/env python3
"""Diagnostic (GPU box): the per-frame-plane loop's frames whose device digest differs from
tests/golden/plane_digests.npz, compared point by point with the oracle chain."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "stereo.vision_amd"), os.path.join(REPO, "tests"),
                os.path.join(REPO, "tests", "golden")]
import oracle  # noqa: E402
from svx import batch  # noqa: E402
from test_prepass_cpu import carmask  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 320
z = np.load(os.path.join(REPO, "tests", "golden", "plane_digests.npz"))
want = z["planes"]
m = carmask()
with batch.Batch(N, step=1, with_bgr=True, with_points=True) as b:
    b.synth(0)
    b.set_mask(m)
    b.prepass("previous")
    b.ransac(seed_base=0, trials=600)
    b.pipeline_planes()
    got = b.digest("pipeline")
    names = ("n_valid", "n_kept", "n_kept2", "disp_hash", "hist_hash", "pts_hash")
    bad = {}
    for k, nm in enumerate(names):
        for f in np.nonzero(got[:, k] != want[nm][:N].astype(np.uint64))[0]:
            bad.setdefault(int(f), []).append(nm)
    print("frames", N, "mismatching", len(bad), dict(list(bad.items())[:20]), flush=True)
    nbits = sum(not np.array_equal(b.read_ransac(f)["abc"], want["abc"][f]) for f in range(N))
    print("planes differing in bits:", nbits, flush=True)
    prev, cleaned = None, {}
    pick = sorted(bad)[:4]
    for f in range(max(pick) + 1 if pick else 0):
        d, bgr = oracle.synth_frame(f)
        c = d.copy() if prev is None else oracle.fill_previous(d, prev)
        prev = c
        if f in pick:
            cleaned[f] = (c, bgr)
    for f, (c, bgr) in cleaned.items():
        r = b.read_ransac(f)
        print(f, "gpu abc", r["abc"].tolist(), "trial", r["trial"], "flags", r["flags"], flush=True)
        print("   gold abc", want["abc"][f].tolist(), "trial", int(want["trial"][f]))
        xyz, pts = b.read_points(f)
        cnt = b.read_counts()[f].tolist()
        for name, abc in (("gold-plane", want["abc"][f]), ("gpu-plane", r["abc"])):
            R = oracle.pipeline_frame(c, bgr, 1, abc=abc)
            print("  ", name, "counts", R["counts"], "gpu", cnt, flush=True)
            if len(R["pts"]) == len(pts):
                dif = np.nonzero((R["pts"] != pts).any(axis=1))[0]
                print("     pts differing", len(dif), dif[:5].tolist(), R["pts"][dif[:5]].tolist(),
                      pts[dif[:5]].tolist(), "src", R["src2"][dif[:5]].tolist(), flush=True)
                xd = np.abs(xyz.astype(np.float64) - R["xyz2"]) / np.abs(R["xyz2"])
                print("     xyz max rel", float(np.nanmax(xd)), flush=True)
