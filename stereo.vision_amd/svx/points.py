"""The point lists the drop-ins pass between stages (functions.py:178-323):
a Python list of row views, as the reference's callers expect, that remembers
the array behind it so the next GPU stage does not re-stack rows."""
import operator

import numpy as np


def select_rows(seq, idx):
    """[seq[i] for i in idx] with the per-item work in C (operator.itemgetter)."""
    idx = [int(i) for i in idx] if not isinstance(idx, np.ndarray) else idx.tolist()
    if not idx:
        return []
    if len(idx) == 1:
        return [seq[idx[0]]]
    return list(operator.itemgetter(*idx)(seq))


class PointList(list):
    """The list of row views projectDisparityTo3d returns, remembering the (N, 3|6)
    array behind it while the list is unmodified, so later GPU stages (RANSAC,
    back-projection, the a2-a6 stage drop-ins) skip re-stacking N Python rows.
    Any list mutation drops it; writes through a row view write the array
    itself, so they stay consistent.

    PointList.subset(parent, idx) is a selection of a PointList (the stages
    that filter, functions.py:314-323, :228-230): its items are the parent's own
    row objects, as the reference returns them, and its array is parent[idx],
    gathered when asked for (so writes through the rows stay visible)."""

    __slots__ = ("_array", "_idx")

    def __init__(self, array):
        super().__init__(array)
        self._array = array
        self._idx = None

    @classmethod
    def subset(cls, parent, idx):
        out = list.__new__(cls)
        list.__init__(out, select_rows(parent, idx))
        base = parent.array() if isinstance(parent, PointList) else None
        out._array = base
        out._idx = np.asarray(idx, np.int64) if base is not None else None
        return out

    def array(self):
        a = self._array
        if a is None:
            return None
        if self._idx is not None:
            return np.ascontiguousarray(a[self._idx]) if len(self._idx) == len(self) else None
        return a if len(a) == len(self) else None

    def _drop(name):  # noqa: N805
        base = getattr(list, name)

        def f(self, *a, **k):
            self._array = None
            return base(self, *a, **k)
        f.__name__ = name
        return f

    for _n in ("append", "extend", "insert", "remove", "pop", "clear", "sort", "reverse", "__setitem__",
               "__delitem__", "__iadd__", "__imul__"):
        locals()[_n] = _drop(_n)
    del _n, _drop


def as_points_array(points):
    """(N, >=3) float64 C-contiguous array of a point sequence (zero-copy for a PointList)."""
    if isinstance(points, PointList) and points.array() is not None:
        return points.array()
    arr = points if isinstance(points, np.ndarray) else np.asarray(points)
    return np.ascontiguousarray(arr, dtype=np.float64)
