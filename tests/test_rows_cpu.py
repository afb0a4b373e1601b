"""The stage drop-ins' host row gathers (sv_gather_rgb_u8, sv_gather_f64; svx/points.py), on the CPU.

The one-by-one drop-ins (stereovision.py:97-113) pass points as index selections of projectDisparityTo3d's
(N, 6) float64 array; each stage gathers the columns it uploads. The gathers must equal numpy's whole-row
selection, see writes made through row views, reject the colours the numpy path rejects, and leave mutated
(materialised) sequences to the numpy path. Host code only: no device work.
"""
import numpy as np
import pytest

from svx import stages
from svx.points import PointList, gather_columns, gather_rgb_u8


def _base(n=5000, seed=0):
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.normal(size=(n, 3)), rng.integers(0, 256, (n, 3)).astype(np.float64)], 1)


def _selections(base):
    rng = np.random.default_rng(1)
    pl = PointList(base)
    idx = np.sort(rng.choice(len(base), 1700, replace=False))
    sel = PointList.subset(pl, idx)
    sel2 = PointList.subset(sel, np.arange(0, len(sel), 3))
    return [(pl, np.arange(len(base))), (sel, idx), (sel2, idx[::3]), (sel[5:900:7], idx[5:900:7])]


def test_gathers_equal_numpy_selection():
    base = _base()
    for seq, rows in _selections(base):
        np.testing.assert_array_equal(gather_rgb_u8(seq), base[rows, 3:6].astype(np.uint8))
        np.testing.assert_array_equal(gather_columns(seq, 0, 3), base[rows, 0:3])
        np.testing.assert_array_equal(gather_columns(seq, 2, 4), base[rows, 2:6])
        np.testing.assert_array_equal(stages._rgb_u8(seq), base[rows, 3:6].astype(np.uint8))


def test_writes_through_rows_are_seen():
    base = _base()
    sel = PointList.subset(PointList(base), np.array([4, 10, 11, 4000]))
    row = sel[2]
    row[0] = 123.25
    row[4] = 7.0
    assert gather_columns(sel, 0, 3)[2, 0] == 123.25
    assert gather_rgb_u8(sel)[2, 1] == 7


@pytest.mark.parametrize("bad", [256.0, -1.0, 1.5, np.nan, np.inf])
def test_bad_colours_raise_like_the_numpy_path(bad):
    base = _base(64)
    base[17, 4] = bad
    sel = PointList.subset(PointList(base), np.arange(10, 40))
    with pytest.raises(ValueError):
        gather_rgb_u8(sel)
    with pytest.raises(ValueError):
        stages._rgb_u8(sel)
    with pytest.raises(ValueError):   # the plain-list path rejects it the same way
        stages._rgb_u8([list(r) for r in base[10:40]])


def test_mutated_and_foreign_sequences_use_the_numpy_path():
    base = _base(100)
    pl = PointList(base)
    pl.append(base[0].copy())   # materialised: a plain list of rows
    assert pl.rows_spec() is None and gather_rgb_u8(pl) is None
    np.testing.assert_array_equal(gather_columns(pl, 0, 3), np.vstack([base, base[:1]])[:, :3])
    rows = [list(r) for r in base[:9]]
    assert gather_rgb_u8(rows) is None
    np.testing.assert_array_equal(gather_columns(rows, 0, 3), base[:9, :3])
    xyz = PointList(np.ascontiguousarray(base[:, :3]))   # rows of 3 values: no colours to gather
    assert gather_rgb_u8(xyz) is None


def test_indices_outside_the_rows_are_refused():
    """the C ABI checks every index against the row count before reading (no out-of-bounds read)"""
    import ctypes
    from svx import _abi
    base = _base(10)
    out8 = np.empty((2, 3), np.uint8)
    out64 = np.empty((2, 3), np.float64)
    for bad in ([0, 10], [-1, 2]):
        idx = np.array(bad, np.int64)
        assert _abi.lib().sv_gather_rgb_u8(_abi.ptr(base), ctypes.c_int64(10), ctypes.c_int64(6), _abi.ptr(idx),
                                           ctypes.c_int64(2), _abi.ptr(out8)) != 0
        assert _abi.lib().sv_gather_f64(_abi.ptr(base), ctypes.c_int64(10), ctypes.c_int64(6), _abi.ptr(idx),
                                        ctypes.c_int64(2), 0, 3, _abi.ptr(out64)) != 0
    assert _abi.lib().sv_gather_f64(_abi.ptr(base), ctypes.c_int64(1), ctypes.c_int64(6), None, ctypes.c_int64(2),
                                    0, 3, _abi.ptr(out64)) != 0   # n > nrows without indices
