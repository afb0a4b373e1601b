"""RANSAC (functions.py:240-298): the oracle restatement against the
reference-run fixtures, and libsvx's host replay of CPython's random draws
against CPython itself. CPU only (sv_ransac_draw never touches the GPU)."""
import ctypes
import hashlib
import json
import os
import random
import sys

import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from oracle import ransac as oransac
from test_prepass_cpu import carmask

sys.path.insert(0, GOLDEN)
import ransac_inputs  # noqa: E402

FIX = json.load(open(os.path.join(GOLDEN, "ransac.json")))


def state_digest():
    return hashlib.sha256(repr(random.getstate()).encode()).hexdigest()[:16]


def bits(abc):
    return [format(int(v), "016x") for v in np.asarray(abc, np.float64).reshape(3).view(np.uint64)]


@pytest.fixture(scope="module")
def cases():
    m = carmask()
    return {name: ransac_inputs.case_points(name, oracle, m) for name in ransac_inputs.CASES}


def test_oracle_matches_reference(cases):
    saved = random.getstate()
    try:
        for key, ref in FIX.items():
            name, seed = key.split("/")
            random.seed(int(seed))
            abc, _ = oransac.ransac(cases[name], ref["trials"])
            assert (None if abc is None else bits(abc)) == ref["abc_bits"], key
            assert state_digest() == ref["state_after"], key
    finally:
        random.setstate(saved)


def _draw(state, pts, trials, k):
    from svx import _abi
    words = np.array(state[1], dtype=np.uint32)
    pts = np.ascontiguousarray(pts, np.float64)
    sidx = np.empty((max(trials, 1), k), np.int32)
    tri = np.empty((max(trials, 1), 3), np.int32)
    ran = ctypes.c_int(0)
    _abi.call("sv_ransac_draw", _abi.ptr(words), _abi.ptr(pts), len(pts), pts.shape[1], trials, k,
              _abi.ptr(sidx), _abi.ptr(tri), ctypes.byref(ran))
    return ran.value, sidx[: ran.value], tri[: ran.value], (state[0], tuple(int(v) for v in words), state[2])


@pytest.mark.parametrize("n,k,trials,seed", [(26287, 600, 40, 0), (2000, 600, 30, 1), (4117, 600, 5, 2),
                                             (4118, 600, 5, 3), (700, 600, 10, 4), (64, 5, 50, 5),
                                             (22, 1, 20, 6), (599, 600, 3, 7), (1 << 20, 600, 3, 8)])
def test_host_draw_replay_matches_cpython(cases, n, k, trials, seed):
    """Both random.sample branches (n <= setsize: pool; else set), n a power of
    two (rejection at half rate), n < k (no draws), and the collinear retries."""
    rng = np.random.default_rng(seed)
    pts = rng.normal(0, 10, (n, 3))
    if n == 700:
        pts = cases["collinear"]
    r = random.Random(seed)
    st0 = r.getstate()
    ran, sidx, tri, st1 = _draw(st0, pts, trials, k)
    _, recs = oransac.ransac(pts, trials, k, rng=r)
    assert ran == len(recs)
    for t, rec in enumerate(recs):
        assert list(sidx[t]) == rec["idx"]
        assert tuple(tri[t]) == rec["tri"]
    assert st1 == r.getstate()


@pytest.mark.parametrize("pre,trials", [(0, 0), (3, 4), (623, 2), (624 * 3 + 100, 3)])
def test_host_draw_from_any_stream_position(pre, trials):
    """The caller's stream at any position (words already drawn from the current twist block, or exactly at its
    end) and zero trials (the state must stay untouched: no twist without a draw)."""
    n, k = 26287, 600
    pts = np.random.default_rng(pre).normal(0, 10, (n, 3))
    r = random.Random(11)
    for _ in range(pre):
        r.getrandbits(32)
    st0 = r.getstate()
    ran, sidx, tri, st1 = _draw(st0, pts, trials, k)
    _, recs = oransac.ransac(pts, trials, k, rng=r)
    assert ran == len(recs) == trials
    for t, rec in enumerate(recs):
        assert list(sidx[t]) == rec["idx"] and tuple(tri[t]) == rec["tri"]
    assert st1 == r.getstate()
    if trials == 0:
        assert st1 == st0


def test_host_draw_rejects_bad_state():
    from svx import _abi
    st = list(random.Random(1).getstate()[1])
    st[624] = 700
    with pytest.raises(_abi.SvxError):
        _draw((3, tuple(st), None), np.zeros((10, 3)), 1, 1)


def _systems(rng, n):
    """3 x 3 systems as RANSAC meets them: maskpoint-like triples, scaled normals, near-collinear triples."""
    out = []
    for kind in range(3):
        P = np.empty((n, 3, 3))
        if kind == 0:
            P[:, :, 0] = rng.uniform(-20, 20, (n, 3))
            P[:, :, 1] = rng.uniform(-3, 3, (n, 3))
            P[:, :, 2] = rng.uniform(2, 80, (n, 3))
        elif kind == 1:
            P = rng.standard_normal((n, 3, 3)) * 10 ** rng.uniform(-3, 3, (n, 1, 1))
        else:
            a, b = rng.uniform(-10, 10, (n, 3)), rng.uniform(-10, 10, (n, 3))
            t = rng.uniform(0, 1, (n, 1))
            P[:, 0], P[:, 1] = a, b
            P[:, 2] = a + t * (b - a) + rng.standard_normal((n, 3)) * 1e-4
        out.append(P)
    return np.concatenate(out)


def test_plane_lapack_matches_numpy():
    """functions.py:267, abc = np.dot(np.linalg.inv(P), np.ones([3, 1])): the restated
    dgesv + dot (oracle svo_plane_lapack, the sequence the device's rb_solve_record
    runs) equals numpy's bits on every system, maskpoint triples included, and is
    singular exactly where numpy raises LinAlgError."""
    rng = np.random.default_rng(2024)
    P = _systems(rng, 4000)
    m = carmask()
    pts = ransac_inputs.case_points(next(iter(ransac_inputs.CASES)), oracle, m)
    tri = pts[rng.integers(0, len(pts), (4000, 3))][:, :, :3]
    P = np.concatenate([P, tri, np.round(P[:200]), P[:50, [0, 0, 1]]])   # integer and repeated-row systems
    bad = []
    for i, p in enumerate(P):
        got, sing = oracle.plane_lapack(*p)
        try:
            want = np.dot(np.linalg.inv(p), np.ones([3, 1]))[:, 0]
        except np.linalg.LinAlgError:
            if not sing:
                bad.append((i, "numpy singular"))
            continue
        if sing or not np.array_equal(got.view(np.uint64), want.view(np.uint64)):
            bad.append((i, got, want))
    assert bad == [], (len(bad), bad[:3])


@pytest.mark.parametrize("k", [1, 5, 7, 8, 9, 100, 128, 129, 600, 1000, 1023, 1024])
def test_ransac_err_matches_numpy(k):
    """functions.py:269-275, :289 — error = np.mean(abs((np.dot(T, abc) - 1) / d)):
    the restated gemv fmas and numpy's pairwise sum (oracle svo_ransac_err, the
    order the device's rb_np_pairwise uses) equal numpy's bits, for every sample
    size the batch accepts up to 1024."""
    import math
    rng = np.random.default_rng(k)
    m = carmask()
    pts = ransac_inputs.case_points(next(iter(ransac_inputs.CASES)), oracle, m)
    for _ in range(20):
        T = pts[rng.choice(len(pts), k, replace=False)]
        abc = np.dot(np.linalg.inv(pts[rng.integers(0, len(pts), 3)][:, :3]), np.ones([3, 1]))
        d = math.sqrt(abc[0, 0] * abc[0, 0] + abc[1, 0] * abc[1, 0] + abc[2, 0] * abc[2, 0])
        rp = [[x[0], x[1], x[2]] for x in T]
        want = np.mean(abs((np.dot(rp, abc) - 1) / d))
        assert oracle.ransac_err(T, abc) == float(want)


def test_numpy_blas_build_is_the_goldens():
    """The bit-exact plane / error restatement follows ONE numpy + OpenBLAS build; the golden
    planes were made with the build recorded in tests/golden/blas_env.json. Another build may round the 3x3
    solve or the gemv differently in the last bit: say so here, by name. (The OpenBLAS kernel architecture
    picked at run time is recorded for information; the pins above are checked on every host they run on.)"""
    sys.path.insert(0, GOLDEN)
    import make_blas_env
    want = json.load(open(os.path.join(GOLDEN, "blas_env.json")))
    got = make_blas_env.env()
    for key in ("numpy", "blas_name", "blas_version", "openblas_configuration"):
        assert got[key] == want[key], f"{key}: running {got[key]!r}, goldens made with {want[key]!r}"
