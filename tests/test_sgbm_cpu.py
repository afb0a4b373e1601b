"""The disparity-stage oracle (oracle/sgbm_oracle.c, oracle/sgbm.py) on the CPU.

Pinned by the reference's own numpy code (tests/golden/sgbm.json from
make_sgbm_golden.py): the gamma tables and the scaling/crop tail of
functions.disparity. StereoSGBM, filterSpeckles, cvtColor and equalizeHist are
OpenCV (absent): PARITY UNPINNED — checked here against independent
restatements (numpy BFS, numpy colour conversion) and against known-disparity
pairs; tests/test_sgbm_cv2.py compares with cv2 wherever it imports.
"""
import json
import os
from collections import deque

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import digest
from oracle import sgbm as osg

META = json.load(open(os.path.join(GOLDEN, "sgbm.json")))


def test_gamma_tables_match_reference():
    for g, table in META["gamma"].items():
        assert osg.gamma_table(float(g)).tolist() == table


def _scaled_inputs(names):
    out = {}
    for name in names:
        if name == "all_int16":
            out[name] = (np.arange(65536, dtype=np.int64) - 32768).astype(np.int16).reshape(256, 256)
        else:
            L, R = osg.synth_pair(int(name[-1]))
            out[name] = osg.disparity(L, R, with_raw=True)[2]
    return out


@pytest.mark.parametrize("name", ["all_int16", "pair0"])
def test_scale_tail_matches_reference(name):
    arr = _scaled_inputs([name])[name]
    rec = META["scaled"][name]
    assert digest(arr) == rec["in"]
    for md in (128, 64):
        for crop in (0, 1):
            r = osg.scale(arr, md, bool(crop))
            exp = rec[f"md{md}_crop{crop}"]
            assert list(r.shape) == exp["shape"] and digest(r) == exp["digest"], (md, crop)


def test_grey_equalize_matches_numpy_restatement():
    rng = np.random.default_rng(5)
    for shape in [(37, 53), (64, 64), (3, 7)]:
        bgr = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
        bgr[0, 0] = 0
        b, g, r = (bgr[..., i].astype(np.int64) for i in range(3))
        y = (b * 1868 + g * 9617 + r * 4899 + 8192) >> 14
        hist = np.bincount(y.ravel(), minlength=256)
        i0 = int(np.nonzero(hist)[0][0])
        scale = np.float32(255.0) / np.float32(y.size - hist[i0])
        lut = np.zeros(256, np.uint8)
        cum = np.cumsum(hist)
        for i in range(i0 + 1, 256):
            lut[i] = np.clip(np.rint(np.float32(cum[i] - cum[i0]) * scale), 0, 255)
        assert np.array_equal(osg.grey_equalize(bgr), lut[y])
    const = np.full((5, 9, 3), 77, np.uint8)
    g = (77 * 1868 + 77 * 9617 + 77 * 4899 + 8192) >> 14
    assert (osg.grey_equalize(const) == g).all()


def speckles_bfs(img, new_val, max_size, max_diff):
    out = img.copy()
    H, W = img.shape
    seen = np.zeros((H, W), bool)
    for i in range(H):
        for j in range(W):
            if seen[i, j] or img[i, j] == new_val:
                continue
            comp, q = [], deque([(i, j)])
            seen[i, j] = True
            while q:
                y, x = q.popleft()
                comp.append((y, x))
                for yy, xx in ((y + 1, x), (y - 1, x), (y, x + 1), (y, x - 1)):
                    if 0 <= yy < H and 0 <= xx < W and not seen[yy, xx] and img[yy, xx] != new_val and \
                            abs(int(img[y, x]) - int(img[yy, xx])) <= max_diff:
                        seen[yy, xx] = True
                        q.append((yy, xx))
            if len(comp) <= max_size:
                for y, x in comp:
                    out[y, x] = new_val
    return out


def test_filter_speckles_matches_bfs():
    rng = np.random.default_rng(7)
    for trial in range(6):
        H, W = rng.integers(5, 40), rng.integers(5, 40)
        img = (rng.integers(-2, 6, (H, W)) * rng.integers(1, 40)).astype(np.int16)
        for new_val, max_size, max_diff in ((0, 5, 30), (0, 40, 0), (-16, 12, 64)):
            assert np.array_equal(osg.filter_speckles(img, new_val, max_size, max_diff),
                                  speckles_bfs(img, new_val, max_size, max_diff)), trial


def test_sgbm_recovers_a_constant_shift():
    rng = np.random.default_rng(0)
    T = rng.integers(0, 256, (120, 640)).astype(np.uint8)
    for shift in (0, 1, 37, 100):
        L = T[:, :500].copy()
        R = T[:, shift:shift + 500].copy()
        d = osg.sgbm(L, R)
        inner = d[15:105, 150:480]
        assert (inner == 16 * shift).mean() > 0.99, shift
        assert (d[:, :128] == -16).all()


def test_sgbm_synthetic_pair_rows():
    L, R = osg.synth_pair(3, 288, 512)
    d = osg.sgbm(L, R)
    D = osg.pair_true_disparity(288)
    valid = d >= 0
    assert valid.mean() > 0.7
    err = np.abs(d.astype(int) - 16 * D[:, None])
    assert ((err <= 32) & valid).sum() / valid.sum() > 0.8


def test_sgbm_geometry_limits():
    z = np.zeros((10, 128), np.uint8)
    assert (osg.sgbm(z, z) == -16).all()              # no cost columns: all invalid, like OpenCV
    with pytest.raises(ValueError):
        osg.sgbm(np.zeros((10, 135), np.uint8), np.zeros((10, 135), np.uint8))   # width1 <= SW2


@pytest.mark.parametrize("kw,H,W", [(dict(), 40, 300), (dict(block=35), 80, 400), (dict(block=5, P1=8, P2=32), 30, 260),
                                    (dict(uniqueness=10, disp12_max_diff=3), 36, 300), (dict(block=1), 9, 200)])
def test_oracle_loop_matches_numpy_paths(kw, H, W):
    """The C oracle's OpenCV-shaped row loop and tests/sgbm_numpy.py's per-direction
    recurrences (the GPU's organisation) agree, including all-saturated pixels
    (bestDisp stays -1: INVALID) in a textureless patch with a 35 x 35 block."""
    import sgbm_numpy
    L, R = osg.synth_pair(7, H, W)
    L = L.copy()
    L[H // 4:H // 2, W // 2:W // 2 + 60] = 90
    raw = sgbm_numpy.sgbm(L, R, **kw)
    assert np.array_equal(osg.sgbm_raw(L, R, **kw), raw)
    assert np.array_equal(osg.sgbm(L, R, **kw), median3_numpy(raw))


def median3_numpy(a):
    """cv2.medianBlur(a, 3) for a 2-D int16 image: the 5th of the 9 replicated-border
    neighbours (OpenCV's 1-D median of 3 for a single row or column is the same thing)."""
    H, W = a.shape
    p = np.pad(a, 1, mode="edge")
    return np.sort(np.stack([p[i:i + H, j:j + W] for i in range(3) for j in range(3)]), axis=0)[4]


def test_median3_matches_numpy():
    """compute()'s medianBlur(disp, disp, 3) (OpenCV StereoSGBMImpl::compute): the C
    oracle against a numpy restatement, degenerate shapes included."""
    rng = np.random.default_rng(11)
    for H, W in [(1, 1), (1, 9), (9, 1), (2, 2), (3, 5), (40, 57), (544, 1024)]:
        a = rng.integers(-16, 2048, (H, W)).astype(np.int16)
        a[rng.random((H, W)) < 0.3] = -16
        assert np.array_equal(osg.median3(a), median3_numpy(a)), (H, W)
    L, R = osg.synth_pair(0)
    raw = osg.sgbm_raw(L, R)
    out = osg.sgbm(L, R)
    assert np.array_equal(out, median3_numpy(raw))
    assert (out != raw).mean() > 0.05   # the median changes a large share of a real frame


@pytest.mark.parametrize("P1,P2,block", [(2, 5, 21), (8, 15, 9), (1, 15, 3), (4, 32, 5)])
def test_path_minus_cost_in_p2_band(P1, P2, block):
    """The identity behind the GPU's 4-bit direction volumes (kernels/sgbm.hip q_byte): every
    path value OpenCV's recurrence produces is L = C + min(Lp(d), Lp(d +- 1) + P1, min Lp + P2) - (min Lp + P2),
    so q = C - L is in [0, P2] in every direction, on random and textureless pairs alike, and the row walk's
    P = sat16(L0 + L1 + L2 + L3) is sat16(4 C - (q0 + q1 + q2 + q3)) from 4-bit q's whenever P2 <= 15."""
    import sgbm_numpy as sn
    rng = np.random.default_rng(P2 * 100 + block)
    H, W = 24, 200
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = np.roll(L, 7, axis=1) if P2 != 15 else rng.integers(0, 256, (H, W), dtype=np.uint8)
    L[5:12, 40:90] = 77   # a textureless patch: flat path costs
    C = sn.cost_volume(L, R, 128, 15, block // 2, block // 2)
    w1 = W - 128
    qs = []
    for sh in (1, 0, -1):   # the three row-to-row directions
        prev = np.zeros((w1, 128), np.int64)
        pmin = np.zeros(w1, np.int64)
        q = np.zeros((H, w1, 128), np.int64)
        for y in range(H):
            if y == 0:
                p, pm = np.zeros_like(prev), np.zeros_like(pmin)
            elif sh == 1:
                p, pm = np.vstack([np.zeros((1, 128), np.int64), prev[:-1]]), np.concatenate([[0], pmin[:-1]])
            elif sh == -1:
                p, pm = np.vstack([prev[1:], np.zeros((1, 128), np.int64)]), np.concatenate([pmin[1:], [0]])
            else:
                p, pm = prev, pmin
            Lv, prev, pmin = sn._step(C[y], p, pm, P1, P2)
            q[y] = C[y] - Lv
        qs.append(q)
    prev = np.zeros((H, 128), np.int64)   # the row walk's own forward direction
    pmin = np.zeros(H, np.int64)
    q0 = np.zeros((H, w1, 128), np.int64)
    for x in range(w1):
        Lv, prev, pmin = sn._step(C[:, x], prev, pmin, P1, P2)
        q0[:, x] = C[:, x] - Lv
    qs.append(q0)
    for q in qs:
        assert q.min() >= 0 and q.max() <= P2, (q.min(), q.max())
