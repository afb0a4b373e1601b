"""Frames of any width through the fused and batched paths.

functions.py:122-124 (crop_disparity=True) hands the hot path 390 x 889
disparity maps: disparity_scaled[0:390, 135:W]. The batch stores rows at a
stride rounded up to 8 bytes (aligned quad loads); the grid, the pre-pass row
means, numpy's negative-index wrap and every read-back use the frame's own
width. Compared with the oracle at steps 1 and 2 (integers bit-exact, fp32 XYZ
within rtol 1e-5).
"""
import types

import numpy as np
import pytest

import oracle
from test_prepass_cpu import carmask

pytestmark = pytest.mark.gpu
RTOL = 1e-5
CROP = (slice(0, 390), slice(135, 1024))


@pytest.fixture(scope="module")
def sv():
    import svx
    from svx import batch, dropin
    assert svx.device_count() >= 1
    return types.SimpleNamespace(svx=svx, batch=batch, dropin=dropin)


def cropped(fid):
    d, bgr = oracle.synth_frame(fid)
    return np.ascontiguousarray(d[CROP]), np.ascontiguousarray(bgr[CROP])


def check(got, ref):
    assert got["counts"] == ref["counts"], (got["counts"], ref["counts"])
    assert np.array_equal(got["hist"], ref["hist"])
    assert np.array_equal(got["pts"], ref["pts"])
    np.testing.assert_allclose(got["xyz2"], ref["xyz2"], rtol=RTOL, atol=0)


@pytest.mark.parametrize("step", [1, 2])
def test_pipeline_frame_cropped(sv, step):
    d, bgr = cropped(3)
    plane = (0.0, 2.87, 0.44)
    got = sv.batch.pipeline_frame(d, bgr, step, plane=plane)
    check(got, oracle.pipeline_frame(d, bgr, step, abc=np.array(plane)))


@pytest.mark.parametrize("mode", ["tiled", "resident"])
@pytest.mark.parametrize("step", [1, 2])
@pytest.mark.parametrize("shape", [(390, 889), (37, 61), (2, 3)])
def test_batch_pipeline_any_width(sv, mode, step, shape):
    H, W = shape
    rng = np.random.default_rng(H * W + step)
    frames = 3
    if shape == (390, 889):
        data = [cropped(50 + f) for f in range(frames)]
    else:
        data = [(rng.integers(0, 256, (H, W)).astype(np.uint8), rng.integers(0, 256, (H, W, 3)).astype(np.uint8))
                for _ in range(frames)]
    plane = (0.0, 2.87, 0.44) if H > 100 else (0.0, 0.0, 0.01)
    thr = 0.05 if H > 100 else 1e9
    with sv.batch.Batch(frames, H, W, step=step, with_bgr=True, with_points=True) as b:
        b.pipeline_mode(mode)
        for f, (d, c) in enumerate(data):
            b.upload(f, d, c)
        b.pipeline(plane=plane, point_thr=thr, hist_thr=2)
        counts = b.read_counts()
        for f, (d, c) in enumerate(data):
            ref = oracle.pipeline_frame(d, c, step, abc=np.array(plane), point_thr=thr, hist_thr=2)
            xyz, pts = b.read_points(f)
            check(dict(counts=tuple(int(v) for v in counts[f]), hist=b.read_hist(f), pts=pts, xyz2=xyz), ref)
            assert np.array_equal(b.read_disp(f), d)


@pytest.mark.parametrize("step", [1, 2])
def test_batch_dense_any_width(sv, step):
    data = [cropped(60 + f)[0] for f in range(3)]
    with sv.batch.Batch(3, 390, 889, step=step, with_bgr=False) as b:
        for f, d in enumerate(data):
            b.upload(f, d)
        b.project()
        for f, d in enumerate(data):
            X, Y, Z = b.read_dense(f)
            RX, RY, RZ = oracle.project_dense(d, step, pitch=b.pitch)
            assert np.array_equal(Z == 0, RZ == 0)
            for a, r in ((X, RX), (Y, RY), (Z, RZ)):
                np.testing.assert_allclose(a, r, rtol=RTOL, atol=0)


@pytest.mark.parametrize("option", ["previous", "mean"])
def test_batch_prepass_raster_ransac_any_width(sv, option):
    frames = 4
    rng = np.random.default_rng(8)
    raw = []
    for f in range(frames):
        d = cropped(70 + f)[0].copy()
        d[rng.random(d.shape) < 0.2] = rng.integers(0, 3)
        raw.append(d)
    mask = np.ascontiguousarray(carmask()[CROP])
    prev0 = rng.integers(0, 256, (390, 889)).astype(np.uint8)
    bgrs = [cropped(70 + f)[1] for f in range(frames)]
    with sv.batch.Batch(frames, 390, 889, step=1, with_bgr=True, with_points=True) as b:
        for f in range(frames):
            b.upload(f, raw[f], bgrs[f])
        b.set_mask(mask)
        b.prepass(option, prev0=prev0 if option == "previous" else None)
        ref = oracle.fill_previous_chain(raw, prev0) if option == "previous" else [oracle.fill_mean(d) for d in raw]
        for f in range(frames):
            dc, dm = b.read_disp(f, masked=True)
            assert np.array_equal(dc, ref[f]), f
            assert np.array_equal(dm, oracle.mask_disparity(ref[f], mask)), f
        # maskpoints (the batched RANSAC's input): the masked step-2 grid of the cleaned frames
        b.ransac(seed_base=0, trials=50, k=60)
        for f in range(frames):
            mp = b.read_maskpoints(f)
            exp, _ = oracle.project(oracle.mask_disparity(ref[f], mask), None, 2)
            assert np.array_equal(mp.view(np.uint64), exp.view(np.uint64)), f
        plane = (0.0, 2.87, 0.44)
        b.pipeline(plane=plane)
        b.road_raster()
        b.nonzero()
        for f in range(frames):
            r = oracle.pipeline_frame(ref[f], bgrs[f], 1, abc=np.array(plane))
            rimg = oracle.road_raster(r["pts"], 390, 889)
            img, walk = b.read_road(f, walk=True)
            assert np.array_equal(img, rimg)
            assert np.array_equal(walk, oracle.nonzero_points(rimg))


def test_negative_wrap_uses_frame_width(sv):
    """numpy wraps img[y, -1] to column W-1 of the frame's own width, not the padded stride."""
    img = sv.dropin.road_raster(np.array([[[-1, 0]]], np.int32), (4, 13))
    assert img[0, 12] == 255 and int(img.sum()) == 255


def test_synth_and_sgbm_batch_need_aligned_width(sv):
    with sv.batch.Batch(1, 390, 889, with_bgr=False) as b:
        with pytest.raises(sv.svx.SvxError):
            b.synth(0)
        with pytest.raises(sv.svx.SvxError):
            b.synth_pair(0)


@pytest.mark.parametrize("shape", [(300, 512), (300, 784), (291, 1024), (270, 16), (280, 1280)])
def test_resident_lane_contiguous_widths(sv, shape):
    """Widths that take the resident kernel's lane-contiguous layout (W % 16 == 0) and its transposed delta
    stage (dx_words <= 32; 1280 columns read the tables in memory): synthetic frames of that size, whose road
    rows keep chunks of a narrow disparity range under the synthetic plane, against the oracle point for point
    (functions.py:178-230, :201-209)."""
    H, W = shape
    frames = 3
    data = [oracle.synth_frame(40 + f, H, W) for f in range(frames)]
    plane = (0.0, 2.8699791779470996, 0.444875113548583)
    with sv.batch.Batch(frames, H, W, step=1, with_bgr=True, with_points=True) as b:
        b.pipeline_mode("resident")
        for f, (d, c) in enumerate(data):
            b.upload(f, d, c)
        b.pipeline(plane=plane, point_thr=0.05, hist_thr=10)
        counts = b.read_counts()
        for f, (d, c) in enumerate(data):
            ref = oracle.pipeline_frame(d, c, 1, abc=np.array(plane), point_thr=0.05, hist_thr=10)
            assert ref["counts"][1] > 0   # keep1 points (at 16 columns the histogram may drop them all)
            xyz, pts = b.read_points(f)
            check(dict(counts=tuple(int(v) for v in counts[f]), hist=b.read_hist(f), pts=pts, xyz2=xyz), ref)
