"""RANSAC plane fit (functions.py:278-298) as a drop-in.

``RANSAC(points, trials)`` consumes Python's global ``random`` stream exactly
as the reference does (libsvx replays CPython's MT19937 / _randbelow /
random.sample from ``random.getstate()`` and the advanced state is put back),
evaluates every trial on the GPU (one workgroup per trial: 3x3 solve, 600
point-plane distances, mean), and then re-decides the winner with the
reference's own numpy calls on the few trials that can matter (flagged
singular / ill-conditioned ones, and those within 1e-6 relative of the best
GPU error) in trial order, so the returned plane is bit-identical and chosen
by the same strict ``error < bestError`` rule (functions.py:289-293). Trials
that raise in the reference (singular matrix) raise in numpy here too and are
skipped the same way; with fewer points than the sample size every trial's
``random.sample`` raises before drawing, so the result is ``(None, None)`` and
the random state is untouched.
"""
import ctypes
import math
import random
from collections.abc import Sequence

import numpy as np

from . import _abi

SAMPLE = 600          # functions.py:286
BAND = 1e-6           # GPU error vs numpy: |dE|/E < 1e-7 for |det| >= 1e-6 |r1||r2||r3|


def _points_array(points):
    from .dropin import as_points_array
    arr = as_points_array(points)
    if arr.ndim != 2 or arr.shape[1] < 3:
        raise ValueError(f"points must be rows of at least [X, Y, Z], got shape {arr.shape}")
    return arr


def trials_gpu(points, trials, state=None, k=SAMPLE):
    """Draw + evaluate. state: random.getstate() tuple (default: the global one).
    Returns dict(sidx, tri, abc, err, flag, state_after) (trial arrays empty if none ran)."""
    arr = _points_array(points)
    st = state if state is not None else random.getstate()
    words = np.array(st[1], dtype=np.uint32)
    n = len(arr)
    # page-locked (pooled): sv_ransac sends each chunk of drawn trials up while it draws the next
    sidx = _abi.pinned_empty((max(trials, 1), k), np.int32)
    tri = _abi.pinned_empty((max(trials, 1), 3), np.int32)
    abc = np.empty((max(trials, 1), 3), np.float64)
    err = np.empty(max(trials, 1), np.float64)
    flag = np.empty(max(trials, 1), np.uint8)
    ran = ctypes.c_int(0)
    _abi.call("sv_ransac", _abi.ptr(words), _abi.ptr(arr), n, arr.shape[1], int(trials), int(k), _abi.ptr(sidx),
              _abi.ptr(tri), _abi.ptr(abc), _abi.ptr(err), _abi.ptr(flag), ctypes.byref(ran))
    r = ran.value
    return dict(arr=arr, sidx=sidx[:r], tri=tri[:r], abc=abc[:r], err=err[:r], flag=flag[:r],
                state_after=(st[0], tuple(int(v) for v in words), st[2]))


def RANSAC(points, trials):  # noqa: N802 (reference signature)
    """functions.py:278-298 on the GPU; returns (normal, coefficients) = (abc, abc) or (None, None)."""
    if not isinstance(points, Sequence) or len(points) < SAMPLE or trials <= 0:
        return (None, None)       # every trial's random.sample raises before drawing
    g = trials_gpu(points, trials)
    random.setstate(g["state_after"])
    arr, err, flag = g["arr"], g["err"], g["flag"]
    ok = flag == 0
    cand = ~ok
    if ok.any():
        cand |= ok & (err <= err[ok].min() * (1 + BAND))
    best, best_err = None, float("inf")
    for t in np.nonzero(cand)[0]:          # trial order; the reference's numpy calls
        try:
            abc = np.dot(np.linalg.inv(arr[g["tri"][t], :3]), np.ones([3, 1]))
        except Exception:                  # functions.py:294-296 swallows per-trial errors
            continue
        d = math.sqrt((abc[0] * abc[0] + abc[1] * abc[1] + abc[2] * abc[2]).item())
        e = np.mean(abs((np.dot(arr[g["sidx"][t], :3], abc) - 1) / d))
        if e < best_err:
            best, best_err = abc, e
    return (best, best) if best is not None else (None, None)
