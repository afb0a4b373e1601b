"""The point sequences the drop-ins pass between stages (functions.py:178-323).

The reference's callers need a Sequence of rows (random.sample, functions.py:252,
286; row[0..5] and row[:3], :205-207,218,252,272,304), not a list as such (SURVEY
§8b). Building 74,200 row views per frame was most of the drop-in chain's host
time (a1 alone 5-8 ms a call), so the sequence is lazy: it holds the (N, 3|6)
float64 array behind it and makes a row view the first time that row is read,
then keeps it, so the same row is the same object every time it is read, through
the sequence and through every selection of it (the selecting stages return the
caller's own row objects, as the reference's list comprehensions do). The GPU
stages take the array itself and never create rows. A mutation turns the
sequence into a plain list of its rows (created then) and it forgets the array.
"""
import collections.abc
import ctypes
import operator

import numpy as np

from . import _abi


def select_rows(seq, idx):
    """[seq[i] for i in idx] with the per-item work in C (operator.itemgetter)."""
    idx = [int(i) for i in idx] if not isinstance(idx, np.ndarray) else idx.tolist()
    if not idx:
        return []
    if len(idx) == 1:
        return [seq[idx[0]]]
    return list(operator.itemgetter(*idx)(seq))


class PointList(collections.abc.MutableSequence):
    """A lazy sequence of the rows of an (N, c) array: projectDisparityTo3d's return
    value and, through PointList.subset, the selections computePlanarThreshold and
    filterPointsByHistogram return. Rows are views of the array (a write through a
    row is a write to the array), made on first read and shared with every
    selection. array() is the (n, c) C-contiguous float64 array of the current
    rows (zero-copy for a whole array; a selection gathers it on every call, so
    writes through rows are seen); None once the sequence was mutated."""

    __slots__ = ("_base", "_cache", "_idx", "_rows", "__weakref__")

    def __init__(self, array):
        self._base = array
        self._cache = [None] * len(array)   # base row index -> its row view, once read
        self._idx = None                    # base row indices of this selection (None: all rows)
        self._rows = None                   # a plain list after a mutation

    @classmethod
    def subset(cls, parent, idx):
        """parent's rows idx (a selection of a selection maps through to the base rows)."""
        if not isinstance(parent, PointList) or parent._rows is not None:
            return select_rows(parent, idx)
        out = cls.__new__(cls)
        out._base, out._cache, out._rows = parent._base, parent._cache, None
        idx = np.asarray(idx, np.int64)
        out._idx = idx if parent._idx is None else parent._idx[idx]
        return out

    # --- Sequence ----------------------------------------------------------
    def __len__(self):
        if self._rows is not None:
            return len(self._rows)
        return len(self._base) if self._idx is None else len(self._idx)

    def _row(self, b):
        r = self._cache[b]
        if r is None:
            r = self._cache[b] = self._base[b]
        return r

    def __getitem__(self, i):
        if self._rows is not None:
            return self._rows[i]
        if isinstance(i, slice):
            sel = np.arange(len(self), dtype=np.int64)[i]
            return PointList.subset(self, sel)
        n = len(self)
        i = operator.index(i)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("list index out of range")
        return self._row(i if self._idx is None else int(self._idx[i]))

    def __iter__(self):
        if self._rows is not None:
            return iter(self._rows)
        ids = range(len(self._base)) if self._idx is None else self._idx.tolist()
        return map(self._row, ids)

    # --- mutation: become a plain list --------------------------------------
    def _materialise(self):
        if self._rows is None:
            self._rows = list(iter(self))
            self._base = self._cache = self._idx = None
        return self._rows

    def __setitem__(self, i, v):
        self._materialise()[i] = v

    def __delitem__(self, i):
        del self._materialise()[i]

    def insert(self, i, v):
        self._materialise().insert(i, v)

    def sort(self, *a, **k):
        self._materialise().sort(*a, **k)

    def copy(self):
        return list(iter(self))

    def __repr__(self):
        return repr(list(iter(self)))

    def __eq__(self, other):   # as a list compares (rows by identity first, then ==)
        if isinstance(other, (list, PointList)):
            return list(iter(self)) == list(iter(other))
        return NotImplemented

    __hash__ = None

    def rows_spec(self):
        """(base, idx or None) when the rows are an index selection of a C-contiguous float64 array (what
        projectDisparityTo3d returns), for the C gathers below; None after a mutation or for another base."""
        if self._rows is not None:
            return None
        b = self._base
        if not (isinstance(b, np.ndarray) and b.dtype == np.float64 and b.ndim == 2 and b.flags.c_contiguous):
            return None
        return b, (None if self._idx is None else np.ascontiguousarray(self._idx, np.int64))

    def array(self):
        if self._rows is not None:
            return None
        if self._idx is None:
            return self._base
        return np.ascontiguousarray(self._base[self._idx])


def as_points_array(points):
    """(N, >=3) float64 C-contiguous array of a point sequence (zero-copy for a whole PointList)."""
    if isinstance(points, PointList) and points.array() is not None:
        return points.array()
    arr = points if isinstance(points, np.ndarray) else np.asarray(list(points) if isinstance(points, PointList)
                                                                   else points)
    return np.ascontiguousarray(arr, dtype=np.float64)


def _spec(points, min_cols):
    if isinstance(points, PointList):
        spec = points.rows_spec()
        if spec is not None and spec[0].shape[1] >= min_cols:
            return spec
    return None


def gather_columns(points, c0, nc, pinned=False):
    """(n, nc) float64 C-contiguous columns c0..c0+nc-1 of a point sequence (n >= 1, rows of >= c0 + nc values).
    A PointList over an array is gathered by libsvx in one pass over the selected rows (sv_gather_f64): reads
    through rows and writes through them are both seen, as with as_points_array, at a fraction of numpy's whole-row
    gather (bench extras.dropin_frame_chain)."""
    spec = _spec(points, c0 + nc)
    if spec is None:
        arr = as_points_array(points)
        if arr.ndim != 2 or arr.shape[1] < c0 + nc:
            return arr   # the caller's shape check reports it
        return np.ascontiguousarray(arr[:, c0:c0 + nc])
    base, idx = spec
    n = len(points)
    # pinned: the result goes to the device next, so gather it into page-locked memory (a direct DMA)
    out = _abi.pinned_empty((n, nc), np.float64) if pinned else np.empty((n, nc), np.float64)
    _abi.call("sv_gather_f64", _abi.ptr(base), base.shape[0], base.shape[1], _abi.ptr(idx), n, c0, nc, _abi.ptr(out))
    return out


def gather_rgb_u8(points):
    """(n, 3) uint8 R, G, B (columns 3..5) of a point sequence of >= 6-value rows, or None when the rows are not a
    PointList over an array (the caller converts them itself). ValueError if a colour is not an integer in
    [0, 255] (sv_gather_rgb_u8)."""
    spec = _spec(points, 6)
    if spec is None:
        return None
    base, idx = spec
    n = len(points)
    out = np.empty((n, 3), np.uint8)
    rc = _abi.lib().sv_gather_rgb_u8(_abi.ptr(base), ctypes.c_int64(base.shape[0]), ctypes.c_int64(base.shape[1]),
                                     _abi.ptr(idx), ctypes.c_int64(n), _abi.ptr(out))
    if rc != 0:
        raise ValueError("colour stages: R, G, B must be integers in [0, 255]")
    return out
