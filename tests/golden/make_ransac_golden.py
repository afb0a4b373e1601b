#!/usr/bin/env python3
"""RANSAC fixtures from the REFERENCE's own functions.RANSAC (functions.py:278-298).

CONTAINER ONLY (needs /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_ransac_golden.py

For every case of ransac_inputs.CASES and seed: random.seed(seed), then the
reference's RANSAC(points, trials) runs unmodified on the points as a list of
numpy rows (what projectDisparityTo3d returns). Saved (ransac.json): the
returned plane's float64 bits (or null), whether normal and coefficients are
the same object, and a digest of random.getstate() afterwards — so a
replacement must consume the global random stream exactly as the reference.
"""
import hashlib
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, REPO, os.path.join(REPO, "tests")]
from make_golden import load_reference  # noqa: E402
import ransac_inputs  # noqa: E402
from test_prepass_cpu import carmask  # noqa: E402

import oracle  # noqa: E402


def state_digest():
    return hashlib.sha256(repr(random.getstate()).encode()).hexdigest()[:16]


def main():
    f = load_reference()
    m = carmask()
    out = {}
    for name, (trials, seeds) in ransac_inputs.CASES.items():
        pts = ransac_inputs.case_points(name, oracle, m)
        rows = list(pts)
        for seed in seeds:
            random.seed(seed)
            normal, abc = f.RANSAC(rows, trials)
            rec = {"n": len(rows), "trials": trials, "seed": seed, "state_after": state_digest()}
            if abc is None:
                rec["abc_bits"] = None
            else:
                rec["abc_bits"] = [format(int(v), "016x") for v in np.asarray(abc, np.float64).reshape(3).view(np.uint64)]
                rec["same_object"] = normal is abc
            out[f"{name}/{seed}"] = rec
            print(name, seed, rec)
    with open(os.path.join(HERE, "ransac.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
