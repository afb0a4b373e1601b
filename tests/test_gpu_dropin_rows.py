"""The drop-in projection's rows path (sv_project_rows into pooled page-locked memory, svx/_abi.py pinned_empty):
the same rows, bit for bit, as sv_project_frame's separate XYZ / colour arrays assembled on the host
(functions.py:178-198: X, Y, Z, then the colour bytes as float64), with and without colours, and a chain that
drops each frame's points reuses the same page-locked blocks (no allocation per call)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame_rows(disp, bgr):
    from svx import _abi, dropin
    h, w = disp.shape
    cap = (h // 2) * (w // 2)   # range(0, h - 1, 2) x range(0, w - 1, 2)
    xyz = np.empty((cap, 3)); rgb = np.empty((cap, 3), np.uint8); n = ctypes.c_int64(0)
    cam = dropin._camera()
    _abi.call("sv_project_frame", _abi.ptr(disp), h, w, w, _abi.ptr(bgr), 3 * w if bgr is not None else 0, 2,
              ctypes.byref(cam), _abi.ptr(xyz), _abi.ptr(rgb) if bgr is not None else None, cap, ctypes.byref(n))
    k = n.value
    if bgr is None:
        return xyz[:k]
    out = np.empty((k, 6))
    out[:, :3] = xyz[:k]
    out[:, 3:] = rgb[:k]
    return out


@pytest.mark.parametrize("with_rgb", [True, False])
def test_rows_equal_frame_arrays(with_rgb):
    import oracle
    from svx import dropin
    for f in (0, 7, 4095):
        disp, bgr = oracle.synth_frame(f)
        rows = dropin.project_rows(disp, bgr if with_rgb else None)
        want = _frame_rows(disp, bgr if with_rgb else None)
        assert rows.shape == want.shape
        assert np.array_equal(rows.view(np.uint64), want.view(np.uint64)), f
        pts = dropin.projectDisparityTo3d(disp, 128, bgr if with_rgb else [])
        assert len(pts) == len(want) and np.array_equal(np.asarray(pts[len(pts) // 2]), want[len(want) // 2])


def test_chain_reuses_pinned_blocks():
    import oracle
    from svx import _abi, dropin
    disp, bgr = oracle.synth_frame(3)
    held = None
    counts = []
    for _ in range(6):
        pts = dropin.projectDisparityTo3d(disp, 128, bgr)
        held = pts[::2]   # a selection keeps the previous frame's block alive across the next call, as a chain does
        counts.append(_abi._pool.allocs)
    assert counts[-1] == counts[2], counts
    assert len(held) > 0


def test_colour_stages_reuse_only_unchanged_colours():
    """filterPointsByHistogram reuses calculateColourHistogram's bins for the same points only while their colours
    are unchanged: a write through a row in between is binned afresh (svx/stages.py _hue)."""
    import oracle
    from svx import dropin, stages
    disp, bgr = oracle.synth_frame(11)
    pts = dropin.projectDisparityTo3d(disp, 128, bgr)
    hist = stages.calculateColourHistogram(pts)
    kept = stages.filterPointsByHistogram(pts, hist, 10)                 # reuses the bins
    stages._hue_last["ref"] = None
    fresh = stages.filterPointsByHistogram(pts, hist, 10)                # bins computed again
    assert len(kept) == len(fresh) and all(a is b for a, b in zip(kept, fresh))
    # recolour the first point with the colour of a point whose key is rare (count <= 10): the filter must see it
    bins = stages._hue(pts, True)[0]
    rare = next(i for i, k in enumerate(bins.tolist()) if hist[stages.bin_key(k)] <= 10)
    row0, src = pts[0], pts[rare]
    row0[3], row0[4], row0[5] = src[3], src[4], src[5]
    after = stages.filterPointsByHistogram(pts, hist, 10)
    stages._hue_last["ref"] = None
    want = stages.filterPointsByHistogram(pts, hist, 10)
    assert [id(r) for r in after] == [id(r) for r in want]
    assert all(r is not row0 for r in after)
