"""ORACLE — test infrastructure only: RANSAC restatement (functions.py:240-298).

Draws through the Python `random` module given (CPython's own generator), by
index: random.sample(points, k) picks population[j] for a j sequence that
depends only on len(points) and k, so sample(range(n), k) yields the same
indices; randomNonCollinearPoints' three sample(points, 1) likewise. The
numeric steps are the reference's numpy calls: inv of the 3x3, dot with ones,
sqrt norm, mean of |P.abc - 1| / d. Pinned by tests/golden/ransac.json (the
reference's RANSAC run on the same points and seeds).
"""
import math

import numpy as np


def ransac(points, trials, k=600, rng=None):
    """-> (abc (3,1) float64 or None, per-trial records). points: (N, >=3) array."""
    import random as _random
    rng = rng or _random
    P = np.asarray(points, np.float64)[:, :3]
    n = len(P)
    recs = []
    if n < k:                       # sample() raises before drawing, in every trial
        return None, recs
    best, best_err = None, float("inf")
    for _ in range(trials):
        idx = rng.sample(range(n), k)
        while True:                 # functions.py:240-260
            i1, i2, i3 = (rng.sample(range(n), 1)[0] for _ in range(3))
            c = np.cross(P[i1] - P[i2], P[i2] - P[i3])
            if (c != 0).any():
                break
        rec = {"idx": idx, "tri": (i1, i2, i3)}
        recs.append(rec)
        try:
            abc = np.dot(np.linalg.inv(np.array([P[i1], P[i2], P[i3]])), np.ones([3, 1]))
        except np.linalg.LinAlgError:
            rec["err"] = None
            continue
        d = math.sqrt(abc[0, 0] * abc[0, 0] + abc[1, 0] * abc[1, 0] + abc[2, 0] * abc[2, 0])
        err = np.mean(np.abs((np.dot(P[idx], abc) - 1) / d))
        rec["abc"], rec["err"] = abc, err
        if err < best_err:
            best, best_err = abc, err
    return best, recs
