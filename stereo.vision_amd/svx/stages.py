"""Drop-ins for the stages a2-a6 one by one, as stereovision.py:97-106 calls them:

    dist   = f.calculatePointErrors(abc, points)                  # functions.py:300-312
    points = f.computePlanarThreshold(points, dist, thr)          # functions.py:314-323
    hist   = f.calculateColourHistogram(points)                   # functions.py:215-226
    points = f.filterPointsByHistogram(points, hist, thr2)        # functions.py:228-230

Each is one device call (kernels/stages.hip); host code only moves data and
builds the Python return values. Contract, as the reference:

* calculatePointErrors returns np.dot(P, abc)'s shape ((N, 1) for the (3, 1)
  plane RANSAC returns, (N,) for a flat one), float64 and bit-identical to the
  reference's BLAS result (P.abc = fma(z, c, fma(x, a, y*b))).
  d = math.sqrt(abc[0]*abc[0] + abc[1]*abc[1] + abc[2]*abc[2]) on the host,
  the reference's own expression. No points: ValueError (np.dot's); no plane
  (None): TypeError, both raised before any device work, as the reference's.
* computePlanarThreshold / filterPointsByHistogram return the caller's own row
  objects, in order (a PointList that still knows its array, so the next stage
  skips re-stacking rows).
* calculateColourHistogram returns {str(round(hue, 3)): count} in the order the
  reference inserts keys (first occurrence over the points). Keys are the
  integer bins of the exact hue (all 2^24 colours checked, tests/golden).
* filterPointsByHistogram raises KeyError(key) for the first point whose key is
  not in the histogram, as the reference's lookup does.
* RGB must be integers in [0, 255] (what projectDisparityTo3d produces); other
  values raise ValueError rather than being hashed differently.
"""
import ctypes
import math

import numpy as np

from . import _abi
from .points import PointList, as_points_array, gather_rgb_u8, select_rows

BINS = 1000


def bin_key(k):
    """The reference's key str(round(h, 3)) of hue bin k = rint(h * 1000): round() of a numpy
    float64 is rint(h * 1000) / 1000, and str() of it is Python's shortest repr."""
    return str(k / 1000)


_KEYS = [bin_key(k) for k in range(BINS)]


def _rows_array(points, min_cols, what):
    arr = as_points_array(points)
    if arr.ndim != 2 or arr.shape[1] < min_cols:
        raise ValueError(f"{what}: points must be rows of at least {min_cols} values, got shape {arr.shape}")
    return arr


def _rgb_u8(points):
    u8 = gather_rgb_u8(points)   # a PointList over the projection's array: one C pass over the selected rows
    if u8 is not None:
        return u8
    arr = _rows_array(points, 6, "colour stages")
    rgb = arr[:, 3:6]
    u8 = rgb.astype(np.uint8)
    if not np.array_equal(u8, rgb):
        raise ValueError("colour stages: R, G, B must be integers in [0, 255]")
    return np.ascontiguousarray(u8)


# The last colour stage's result, for the next stage on the same points: the reference's chain
# (stereovision.py:103-106) bins the same selection twice, calculateColourHistogram(points) then
# filterPointsByHistogram(points, hist, thr). Kept only for a PointList (by weak reference) and reused only when the
# colours gathered again are byte-for-byte the ones it was computed from, so a write through a row in between is seen.
_hue_last = {"ref": None, "rgb": None, "out": None}


def _hue(points, bins):
    """(bins int16, hist u32[1000], first i64[1000]) of the points' colours (device)."""
    import weakref
    rgb = _rgb_u8(points)
    last = _hue_last
    ref = last["ref"]
    if ref is not None and ref() is points and last["rgb"].shape == rgb.shape and np.array_equal(last["rgb"], rgb):
        return last["out"]
    n = len(rgb)
    hist = np.empty(BINS, np.uint32)
    first = np.empty(BINS, np.int64)
    out_bins = np.empty(n, np.int16)
    _abi.call("sv_hue_histogram", _abi.ptr(rgb), n, 3, _abi.ptr(out_bins), _abi.ptr(hist), _abi.ptr(first))
    out = (out_bins, hist, first)
    if isinstance(points, PointList):
        last.update(ref=weakref.ref(points), rgb=rgb, out=out)
    else:
        last.update(ref=None, rgb=None, out=None)
    return out


def _select(points, idx):
    if isinstance(points, PointList):
        return PointList.subset(points, idx)
    return select_rows(points, idx)


def calculatePointErrors(abc, points):  # noqa: N802 (reference signature)
    """functions.py:300-312 on the GPU."""
    d = math.sqrt(_scalar(abc[0] * abc[0] + abc[1] * abc[1] + abc[2] * abc[2]))   # :307, TypeError for None
    col = np.asarray(abc, np.float64)
    n = len(points)
    if n == 0:   # the reference's np.dot(np.array([]), abc), numpy's message
        shape = "(" + ",".join(map(str, col.shape)) + ("," if col.ndim == 1 else "") + ")"
        raise ValueError(f"shapes (0,) and {shape} not aligned: 0 (dim 0) != {col.shape[0]} (dim 0)")
    if col.shape[0] != 3 or col.ndim > 2 or (col.ndim == 2 and col.shape[1] != 1):
        raise ValueError(f"calculatePointErrors: plane must have shape (3,) or (3, 1), got {col.shape}")
    arr = _rows_array(points, 3, "calculatePointErrors")
    abcd = np.array([col.reshape(3)[0], col.reshape(3)[1], col.reshape(3)[2], d], np.float64)
    out = np.empty(n, np.float64)
    _abi.call("sv_point_errors", _abi.ptr(arr), n, arr.shape[1], _abi.ptr(abcd), _abi.ptr(out))
    return out.reshape(n, 1) if col.ndim == 2 else out


def _scalar(v):
    a = np.asarray(v, np.float64)
    if a.size != 1:
        raise TypeError("only length-1 arrays can be converted to Python scalars")
    return float(a.reshape(-1)[0])


def computePlanarThreshold(points, differences, threshold=0.01):  # noqa: N802
    """functions.py:314-323 on the GPU: the rows whose distance is < threshold, in order."""
    n = len(points)
    if n == 0:
        return []
    diff = np.asarray(differences, np.float64)
    if diff.ndim > 2 or (diff.ndim == 2 and diff.shape[1] != 1):
        raise ValueError("The truth value of an array with more than one element is ambiguous. "
                         "Use a.any() or a.all()")
    vals = np.ascontiguousarray(diff.reshape(-1))
    if len(vals) < n:
        raise IndexError(f"index {len(vals)} is out of bounds for axis 0 with size {len(vals)}")
    idx = np.empty(n, np.int64)
    k = ctypes.c_int64(0)
    _abi.call("sv_select_less", _abi.ptr(vals), n, float(threshold), _abi.ptr(idx), ctypes.byref(k))
    return _select(points, idx[: k.value])


def calculateColourHistogram(points):  # noqa: N802
    """functions.py:215-226 on the GPU: {key: count}, keys in first-occurrence order."""
    if len(points) == 0:
        return {}
    _, hist, first = _hue(points, bins=False)
    present = np.nonzero(hist)[0]
    order = present[np.argsort(first[present], kind="stable")]
    return {_KEYS[k]: int(hist[k]) for k in order}


def filterPointsByHistogram(points, histogram, threshold=100):  # noqa: N802
    """functions.py:228-230 on the GPU: the rows whose key's count is > threshold, in order."""
    n = len(points)
    if n == 0:
        return []
    bins, hist, first = _hue(points, bins=True)
    ok = np.zeros(BINS, np.uint8)
    missing = []
    for k in np.nonzero(hist)[0]:
        key = _KEYS[k]
        if key in histogram:
            ok[k] = 1 if histogram[key] > threshold else 0
        else:
            missing.append(k)
    if missing:   # the reference raises at the first point whose key is absent
        k = min(missing, key=lambda b: first[b])
        raise KeyError(_KEYS[k])
    idx = np.empty(n, np.int64)
    cnt = ctypes.c_int64(0)
    _abi.call("sv_select_bins", _abi.ptr(bins), n, _abi.ptr(ok), _abi.ptr(idx), ctypes.byref(cnt))
    return _select(points, idx[: cnt.value])
