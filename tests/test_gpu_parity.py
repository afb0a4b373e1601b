"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden
fixtures. Bit-exact for integer/index/byte outputs and for the fp64 drop-in;
fp32 XYZ within 1e-5 relative (BASELINE.json north_star tolerance)."""
import collections.abc
import os
import random
import types

import numpy as np
import pytest

import oracle
from conftest import sparse_frame

pytestmark = pytest.mark.gpu

RTOL = 1e-5  # north_star: fp32 XYZ within 1e-5 relative


@pytest.fixture(scope="module")
def svx_mod():
    import svx
    from svx import batch, dropin
    assert svx.device_count() >= 1
    return types.SimpleNamespace(svx=svx, batch=batch, dropin=dropin)


def _bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


# ---------------------------------------------------------------------------
# exhaustive tables
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("variant", [0, 1])
def test_hue_lut_exhaustive(svx_mod, golden, variant):
    """every colour's bin: the exact device function (0) and the resident pipeline's fp32 path with its tie-band
    fallback (1, hue_bin_sel) both equal the reference-run LUT digest (functions.py:73-78, 215-226)"""
    lut = svx_mod.batch.hue_lut(variant=variant)
    ref = oracle.hue_lut()
    bad = np.flatnonzero(lut != ref)
    assert bad.size == 0, f"{bad.size} colours differ, first {bad[:5]}"
    assert oracle.digest(lut) == golden.meta["hue_lut"]["digest"]


def test_delta_tables(svx_mod):
    dx, dy = svx_mod.batch.delta_tables()
    rdx, rdy = oracle.delta_tables()
    assert np.array_equal(dx, rdx) and np.array_equal(dy, rdy)
    cam = (401.25, 0.21, 500.3, 250.7)   # a non-default camera too
    from svx import _abi
    dx, dy = svx_mod.batch.delta_tables(400, 640, camera=_abi.Camera(*cam))
    rdx, rdy = oracle.delta_tables(400, 640, camera=cam)
    assert np.array_equal(dx, rdx) and np.array_equal(dy, rdy)


@pytest.mark.parametrize("fid", [0, 1, 4095, 32767])
def test_device_generator(svx_mod, fid):
    d, b = svx_mod.batch.synth_frame(fid)
    rd, rb = oracle.synth_frame(fid)
    assert np.array_equal(d, rd) and np.array_equal(b, rb)


# ---------------------------------------------------------------------------
# drop-in projection / back-projection (fp64, bit-exact)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("k", [0, 1, 2])
def test_dropin_project_sparse(svx_mod, golden, k):
    disp, bgr = sparse_frame(golden, k)
    xyz, rgb = svx_mod.dropin.project_frame(disp, bgr)
    assert np.array_equal(_bits(xyz), _bits(golden.sparse[f"f{k}_xyz"]))
    assert np.array_equal(rgb, golden.sparse[f"f{k}_rgb"])
    xyz2, none = svx_mod.dropin.project_frame(disp, None)
    assert none is None and np.array_equal(_bits(xyz2), _bits(golden.sparse[f"f{k}_mask_xyz"]))


@pytest.mark.parametrize("fid", ["0", "1", "4095"])
def test_dropin_project_full_frames(svx_mod, golden, fid):
    m = golden.meta["full_frames_step2"][fid]
    disp, bgr = oracle.synth_frame(int(fid))
    xyz, rgb = svx_mod.dropin.project_frame(disp, bgr)
    assert oracle.digest(xyz) == m["xyz"] and oracle.digest(rgb) == m["rgb"]


@pytest.mark.parametrize("step", [1, 3])
def test_dropin_project_other_steps(svx_mod, step):
    disp, bgr = oracle.synth_frame(5)
    xyz, rgb = svx_mod.dropin.project_frame(disp, bgr, step=step)
    rxyz, rrgb = oracle.project(disp, bgr, step)
    assert np.array_equal(_bits(xyz), _bits(rxyz)) and np.array_equal(rgb, rrgb)


@pytest.mark.parametrize("shape", [(1, 1), (2, 2), (3, 7), (17, 33), (544, 1023), (100, 1)])
def test_dropin_project_ragged_shapes(svx_mod, shape):
    rng = np.random.default_rng(sum(shape))
    disp = rng.integers(0, 256, shape).astype(np.uint8)
    disp[rng.random(shape) < 0.3] = 0
    bgr = rng.integers(0, 256, shape + (3,)).astype(np.uint8)
    xyz, rgb = svx_mod.dropin.project_frame(disp, bgr)
    rxyz, rrgb = oracle.project(disp, bgr, 2)
    assert np.array_equal(_bits(xyz), _bits(rxyz)) and np.array_equal(rgb, rrgb)


def test_dropin_project_empty_and_strided(svx_mod):
    z = np.zeros((544, 1024), np.uint8)
    assert svx_mod.dropin.projectDisparityTo3d(z, 128) == []
    full = np.full((544, 1024), 255, np.uint8)
    assert len(svx_mod.dropin.projectDisparityTo3d(full, 128)) == 272 * 512
    disp, bgr = oracle.synth_frame(9)
    big = np.zeros((600, 1100), np.uint8)
    big[:544, :1024] = disp
    view = big[:544, :1024]                      # non-contiguous rows
    xyz, _ = svx_mod.dropin.project_frame(view, None)
    assert np.array_equal(_bits(xyz), _bits(oracle.project(disp, None, 2)[0]))


def test_dropin_backproject_exact(svx_mod, golden):
    for k in range(3):
        s = golden.sparse
        rows = s[f"f{k}_xyz"][s[f"f{k}_keep2_idx"]]
        xy = svx_mod.dropin.project3DPointsTo2DImagePoints(list(rows))
        assert np.array_equal(_bits(xy), _bits(oracle.backproject(rows)))
        pp = np.array(xy, np.int32).reshape((-1, 1, 2))
        assert np.array_equal(pp, s[f"f{k}_plane_points"])
    empty = svx_mod.dropin.project3DPointsTo2DImagePoints([])
    assert np.array(empty, np.int32).reshape((-1, 1, 2)).shape == (0, 1, 2)


def test_dropin_sequence_protocol(svx_mod):
    """What the unchanged downstream reference functions need."""
    disp, bgr = oracle.synth_frame(0)
    pts = svx_mod.dropin.projectDisparityTo3d(disp, 128, bgr)
    assert isinstance(pts, collections.abc.Sequence)                 # a Sequence of rows
    assert len(random.sample(pts, 600)) == 600                     # functions.py:286
    p = pts[0]
    assert len(p[:3]) == 3 and type(p[0]) is np.float64 and isinstance(p[3], np.generic)
    from oracle import cpu_loop
    assert cpu_loop.hue_key(p[3], p[4], p[5]) == cpu_loop.hue_key(*(np.uint8(v) for v in p[3:6]))


def test_dropin_installed_chain_matches_reference(svx_mod, golden):
    """stereovision.py:84-113 with the drop-in installed into a functions-like module
    (the rest of the chain is the nested-loop port standing in for the reference)."""
    from oracle import cpu_loop
    f = types.SimpleNamespace(
        camera_focal_length_px=oracle.F_PX, stereo_camera_baseline_m=oracle.BASELINE_M,
        image_centre_w=oracle.CW, image_centre_h=oracle.CH,
        projectDisparityTo3d=lambda d, m, rgb=[]: cpu_loop.project(d, rgb if len(rgb) else None),
        project3DPointsTo2DImagePoints=cpu_loop.backproject,
        calculatePointErrors=cpu_loop.point_errors, computePlanarThreshold=cpu_loop.plane_keep,
        calculateColourHistogram=cpu_loop.colour_hist, filterPointsByHistogram=cpu_loop.hist_keep)
    svx_mod.dropin.install(f)
    try:
        assert f.projectDisparityTo3d is svx_mod.dropin.projectDisparityTo3d
        m = golden.meta["full_frames_step2"]["0"]
        disp, bgr = oracle.synth_frame(0)
        abc = np.array(m["abc"]).reshape(3, 1)
        points = f.projectDisparityTo3d(disp, 128, bgr)
        diffs = f.calculatePointErrors(abc, points)
        points = f.computePlanarThreshold(points, diffs, 0.05)
        assert len(points) == m["n_kept"]
        hist = f.calculateColourHistogram(points)
        points = f.filterPointsByHistogram(points, hist, 10)
        assert len(points) == m["n_kept2"]
        pp = np.array(f.project3DPointsTo2DImagePoints(points), np.int32).reshape((-1, 1, 2))
        assert oracle.digest(pp) == m["plane_points"]
    finally:
        svx_mod.dropin.uninstall()


# ---------------------------------------------------------------------------
# fused pipeline (one host frame)
# ---------------------------------------------------------------------------
def _check_pipe(got, ref, xyz_ref=None):
    assert got["counts"] == ref["counts"], (got["counts"], ref["counts"])
    assert np.array_equal(got["hist"], ref["hist"])
    assert np.array_equal(got["pts"], ref["pts"])
    xr = ref["xyz2"] if xyz_ref is None else xyz_ref
    np.testing.assert_allclose(got["xyz2"], xr, rtol=RTOL, atol=0)


@pytest.mark.parametrize("k", [0, 1, 2])
def test_pipeline_sparse(svx_mod, golden, k):
    disp, bgr = sparse_frame(golden, k)
    s = golden.sparse
    got = svx_mod.batch.pipeline_frame(disp, bgr, 2, plane=tuple(golden.meta["plane_abc"]))
    ref = dict(counts=(len(s[f"f{k}_xyz"]), len(s[f"f{k}_keep_idx"]), len(s[f"f{k}_keep2_idx"])),
               hist=s[f"f{k}_hist"], pts=s[f"f{k}_plane_points"].reshape(-1, 2),
               xyz2=s[f"f{k}_xyz"][s[f"f{k}_keep2_idx"]])
    _check_pipe(got, ref)


@pytest.mark.parametrize("k", [0, 1, 2])
def test_pipeline_crops(svx_mod, golden, k):
    c = golden.crops
    got = svx_mod.batch.pipeline_frame(c[f"c{k}_disp"], c[f"c{k}_bgr"], 2, plane=tuple(c[f"c{k}_abc"]))
    ref = dict(counts=(len(c[f"c{k}_xyz"]), len(c[f"c{k}_keep_idx"]), len(c[f"c{k}_keep2_idx"])),
               hist=c[f"c{k}_hist"], pts=c[f"c{k}_plane_points"].reshape(-1, 2),
               xyz2=c[f"c{k}_xyz"][c[f"c{k}_keep2_idx"]])
    _check_pipe(got, ref)


@pytest.mark.parametrize("fid", ["0", "1", "4095", "0r"])
def test_pipeline_full_frames_step2(svx_mod, golden, fid):
    m = golden.meta["full_frames_step2"][fid]
    disp, bgr = oracle.synth_frame(0 if fid == "0r" else int(fid))
    got = svx_mod.batch.pipeline_frame(disp, bgr, 2, plane=tuple(m["abc"]))
    assert got["counts"] == (m["n"], m["n_kept"], m["n_kept2"])
    assert oracle.digest(got["hist"]) == m["hist"]
    assert oracle.digest(got["pts"].reshape(-1, 1, 2)) == m["plane_points"]


def _pipe(svx_mod, kind, disp, bgr, step, **kw):
    """One host frame through the fused chain: "frame" = sv_pipeline_frame (tiled
    kernels), "resident" = a 1-frame batch forced onto the frame-resident kernel."""
    if kind == "frame":
        return svx_mod.batch.pipeline_frame(disp, bgr, step, **kw)
    H, W = disp.shape
    with svx_mod.batch.Batch(1, H=H, W=W, step=step, with_bgr=True, with_points=True) as b:
        b.pipeline_mode(kind)
        b.upload(0, disp, bgr)
        b.pipeline(**kw)
        xyz, pts = b.read_points(0)
        return dict(counts=tuple(int(v) for v in b.read_counts()[0]), hist=b.read_hist(0), pts=pts, xyz2=xyz)


KINDS = ["frame", "resident", "resident_nopf", "resident_pf2"]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("fid", [0, 1, 4095])
def test_pipeline_full_frames_step1(svx_mod, fid, kind):
    disp, bgr = oracle.synth_frame(fid)
    got = _pipe(svx_mod, kind, disp, bgr, 1)
    _check_pipe(got, oracle.pipeline_frame(disp, bgr, 1))


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("plane", [(-0.007, 2.79, 0.457), (0.01, 2.5, 0.6), (0.0, 1e-3, 1e-3)])
@pytest.mark.parametrize("thr", [0.05, 0.01, 0.2])
def test_pipeline_planes_and_thresholds(svx_mod, plane, thr, kind):
    disp, bgr = oracle.synth_frame(17)
    got = _pipe(svx_mod, kind, disp, bgr, 2, plane=plane, point_thr=thr, hist_thr=3)
    _check_pipe(got, oracle.pipeline_frame(disp, bgr, 2, abc=np.array(plane), point_thr=thr, hist_thr=3))


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("hist_thr", [-1, 0, 40, 10 ** 9])
def test_pipeline_hist_thresholds(svx_mod, hist_thr, kind):
    """Every tile clean (-1), most tiles dirty (40), everything filtered (1e9)."""
    disp, bgr = oracle.synth_frame(23)
    for step in (1, 2):
        got = _pipe(svx_mod, kind, disp, bgr, step, hist_thr=hist_thr)
        _check_pipe(got, oracle.pipeline_frame(disp, bgr, step, hist_thr=hist_thr))


@pytest.mark.parametrize("kind", KINDS)
def test_pipeline_edge_frames(svx_mod, kind):
    z = np.zeros((544, 1024), np.uint8)
    bgr = np.zeros((544, 1024, 3), np.uint8)
    got = _pipe(svx_mod, kind, z, bgr, 2)
    assert got["counts"] == (0, 0, 0) and got["pts"].shape == (0, 2)
    full = np.full((544, 1024), 255, np.uint8)
    _check_pipe(_pipe(svx_mod, kind, full, bgr, 1), oracle.pipeline_frame(full, bgr, 1))
    rng = np.random.default_rng(3)
    for H, W in ((2, 8), (9, 16), (33, 64)):
        d = rng.integers(0, 256, (H, W)).astype(np.uint8)
        c = rng.integers(0, 4, (H, W, 3)).astype(np.uint8)
        for step in (1, 2):
            got = _pipe(svx_mod, kind, d, c, step, plane=(0.0, 0.0, 0.01), point_thr=1e9, hist_thr=0)
            _check_pipe(got, oracle.pipeline_frame(d, c, step, abc=np.array([0.0, 0.0, 0.01]),
                                                    point_thr=1e9, hist_thr=0))


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("plane", [(0.0, -3.0, -0.5), (0.0, 2.87, 0.44), (0.02, 2.9, -0.3)])
def test_pipeline_chunk_skipping(svx_mod, kind, plane):
    """Planes under which the keep table rules out none, some or all of the
    resident kernel's chunks (those chunks are skipped): the valid count still
    covers every grid point and the outputs equal the oracle's."""
    disp, bgr = oracle.synth_frame(5)
    for step in (1, 2):
        got = _pipe(svx_mod, kind, disp, bgr, step, plane=plane)
        _check_pipe(got, oracle.pipeline_frame(disp, bgr, step, abc=np.array(plane)))


@pytest.mark.parametrize("kind", KINDS)
def test_pipeline_random_colours_and_planes(svx_mod, kind):
    """Uniformly random BGR (every hue bin, exact ties included) and random
    disparity, under planes that put many points near the keep1 boundary."""
    rng = np.random.default_rng(11)
    for trial in range(3):
        d = rng.integers(0, 256, (544, 1024)).astype(np.uint8)
        c = rng.integers(0, 256, (544, 1024, 3)).astype(np.uint8)
        plane = (float(rng.normal(0, 0.01)), float(rng.uniform(1, 3)), float(rng.uniform(0.2, 0.6)))
        for step in (1, 2):
            got = _pipe(svx_mod, kind, d, c, step, plane=plane, point_thr=0.3, hist_thr=50)
            _check_pipe(got, oracle.pipeline_frame(d, c, step, abc=np.array(plane), point_thr=0.3,
                                                    hist_thr=50))


# ---------------------------------------------------------------------------
# batched device-resident API
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("step", [1, 2])
@pytest.mark.parametrize("tune", [(1, 0), (1, 1), (2, 1), (4, 1), (1, 2)])
def test_batch_dense_projection(svx_mod, step, tune):
    first = 40
    with svx_mod.batch.Batch(6, step=step, with_bgr=False) as b:
        b.tune(*tune)
        b.synth(first)
        b.project()
        for f in range(6):
            X, Y, Z = b.read_dense(f)
            disp, _ = oracle.synth_frame(first + f)
            RX, RY, RZ = oracle.project_dense(disp, step)
            assert np.array_equal(Z == 0, RZ == 0)
            for a, r in ((X, RX), (Y, RY), (Z, RZ)):
                np.testing.assert_allclose(a, r, rtol=RTOL, atol=0)


@pytest.mark.parametrize("step,chunk,mode", [(1, 16, "tiled"), (1, 3, "tiled"), (2, 1, "tiled"),
                                             (2, 5, "tiled"), (1, 0, "resident"), (2, 0, "resident"),
                                             (1, 0, "resident_nopf"), (1, 3, "resident_nopf"), (2, 2, "resident_nopf"),
                                             (1, 0, "resident_pf2"), (2, 0, "resident_pf2")])
def test_batch_pipeline(svx_mod, step, chunk, mode):
    frames, first = 7, 1000
    with svx_mod.batch.Batch(frames, step=step, with_bgr=True, with_points=True) as b:
        b.pipeline_mode(mode)
        b.synth(first)
        b.pipeline(chunk=chunk)
        counts = b.read_counts()
        for f in range(frames):
            disp, bgr = oracle.synth_frame(first + f)
            ref = oracle.pipeline_frame(disp, bgr, step)
            xyz, pts = b.read_points(f)
            got = dict(counts=tuple(int(v) for v in counts[f]), hist=b.read_hist(f), pts=pts, xyz2=xyz)
            _check_pipe(got, ref)


def test_batch_baseline_size_properties(svx_mod):
    """BASELINE configs 3/4 at full size (4096 frames, step 1): EVERY frame's
    digest (counts, disparity, histogram and point hashes, fp32 tolerance) equals
    the oracle's (tests/golden/frame_digests.npz) for K1 and for every pipeline
    kernel family; sampled frames are also compared point by point, and the
    tiled results do not depend on the chunking."""
    import os

    from conftest import GOLDEN
    want = np.load(os.path.join(GOLDEN, "frame_digests.npz"))["step1"][:4096]
    cols = ("n_valid", "n_kept", "n_kept2", "disp_hash", "hist_hash", "pts_hash")

    def check(got, which):
        names = cols if which == "pipeline" else ("n_valid", "disp_hash")
        for k, name in enumerate(cols):
            if name in names:
                diff = np.flatnonzero(got[:, k] != want[name].astype(np.uint64))
                assert diff.size == 0, (which, name, diff[:5])
        assert (got[:, 6] == 0).all(), (which, np.flatnonzero(got[:, 6])[:5])

    frames = 4096
    with svx_mod.batch.Batch(frames, step=1, with_bgr=True, with_points=True) as b:
        b.synth(0)
        b.project()
        check(b.digest("dense"), "dense")
        for f in (0, 2047, 4095):
            disp, bgr = oracle.synth_frame(f)
            X, Y, Z = b.read_dense(f)
            RX, RY, RZ = oracle.project_dense(disp, 1)
            assert np.array_equal(Z == 0, RZ == 0)
            np.testing.assert_allclose(Z, RZ, rtol=RTOL, atol=0)
        b.pipeline_mode("tiled")
        for chunk in (16, 29):
            b.pipeline(chunk=chunk)
            check(b.digest("pipeline"), "pipeline")
        for f in (0, 1234, 4095):
            disp, bgr = oracle.synth_frame(f)
            ref = oracle.pipeline_frame(disp, bgr, 1)
            xyz, pts = b.read_points(f)
            assert tuple(b.read_counts()[f]) == ref["counts"]
            assert np.array_equal(pts, ref["pts"])
        for mode in ("resident", "resident_nopf", "resident_pf2"):
            b.pipeline_mode(mode)
            b.pipeline()
            check(b.digest("pipeline"), "pipeline")
            for f in (0, 777, 4095):
                disp, bgr = oracle.synth_frame(f)
                ref = oracle.pipeline_frame(disp, bgr, 1)
                xr, pr = b.read_points(f)
                assert np.array_equal(pr, ref["pts"])
                np.testing.assert_allclose(xr, ref["xyz2"], rtol=RTOL, atol=0)


def test_errors_are_raised(svx_mod):
    from svx import SvxError
    with pytest.raises(SvxError):
        svx_mod.batch.Batch(1, H=544, W=1)          # no grid column (any W >= 2 is accepted)
    with pytest.raises(SvxError):
        svx_mod.batch.Batch(1, H=544, W=1024, step=3)
    with pytest.raises(TypeError):
        svx_mod.dropin.projectDisparityTo3d(np.zeros((4, 4), np.float32), 128)


def test_k1_xyz_against_oracle_every_frame(svx_mod):
    """K1 at the headline size (4096 frames, step 1): X, Y and Z of EVERY frame (2.28 G points) against the C
    oracle's fp64 values (oracle.check_dense_f32, which generates the frame and projects it as
    functions.py:191-193 do), within north_star's 1e-5 relative, with the same zero pattern. The checker is the
    oracle, not the product library's digest kernel; frames are read back one by one and checked on host threads."""
    from concurrent.futures import ThreadPoolExecutor
    frames = 4096
    with svx_mod.batch.Batch(frames, step=1, with_bgr=False) as b:
        b.synth(0)
        b.project()
        res = []
        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as pool:
            for f0 in range(0, frames, 64):   # 64 frames' planes held at a time
                futs = [pool.submit(oracle.check_dense_f32, f, *b.read_dense(f), 1, RTOL) for f in range(f0, f0 + 64)]
                res += [fu.result() for fu in futs]
    bad = [(f, r[0]) for f, r in enumerate(res) if r[0] != 0]
    worst = max(r[1] for r in res)
    assert bad == [], bad[:10]
    assert worst <= RTOL
    print(f"K1 vs oracle, {frames} frames: max relative error {worst:.3g}")
