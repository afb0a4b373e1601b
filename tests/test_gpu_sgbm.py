"""Disparity stage on the GPU (functions.py:61-128) against
the oracle (oracle/sgbm_oracle.c, bit-exact: every output is integer) and the
reference-run fixtures of tests/golden/sgbm.json.

PARITY UNPINNED for the OpenCV calls themselves (StereoSGBM, filterSpeckles,
cvtColor, equalizeHist): cv2 is absent, so the oracle restates OpenCV's
published algorithm (tests/test_sgbm_cv2.py pins it wherever cv2 imports).
"""
import json
import os
import types

import numpy as np
import pytest

import oracle
from conftest import GOLDEN
from oracle import sgbm as osg

pytestmark = pytest.mark.gpu
META = json.load(open(os.path.join(GOLDEN, "sgbm.json")))


@pytest.fixture(scope="module")
def sv():
    import svx
    from svx import batch, disparity, dropin
    assert svx.device_count() >= 1
    return types.SimpleNamespace(svx=svx, batch=batch, disp=disparity, dropin=dropin)


def test_gamma_lut_matches_reference_tables(sv):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (61, 77, 3), dtype=np.uint8)
    for g, table in META["gamma"].items():
        assert np.array_equal(sv.disp.gammaChange(img, float(g)), np.asarray(table, np.uint8)[img])
    a, b = sv.disp.preProcessImages(img, img[::-1])
    t14 = np.asarray(META["gamma"]["1.4"], np.uint8)
    assert np.array_equal(a, t14[img]) and np.array_equal(b, t14[img[::-1]])


def test_grey_equalize_matches_oracle(sv):
    rng = np.random.default_rng(1)
    _, bgr0 = oracle.synth_frame(0)
    cases = [bgr0, rng.integers(0, 256, (37, 53, 3), dtype=np.uint8),
             rng.integers(100, 104, (544, 1024, 3), dtype=np.uint8), np.full((9, 5, 3), 77, np.uint8),
             np.zeros((1, 1, 3), np.uint8)]
    for bgr in cases:
        assert np.array_equal(sv.disp.grey_equalize(bgr), osg.grey_equalize(bgr)), bgr.shape
    gl, gr = sv.disp.greyscale(bgr0, bgr0[:, ::-1])
    assert np.array_equal(gl, osg.grey_equalize(bgr0)) and np.array_equal(gr, osg.grey_equalize(bgr0[:, ::-1]))


# (42, 296): two whole 21-step blocks of the unrolled rings in both the vertical walk (H = 2 x 21) and each
# wave's quarter of the horizontal sums (296 - 128 = 168 cost columns = 4 x 42); the others cut the blocks short
SMALL = [(96, 320, "pair"), (3, 139, "rand"), (5, 256, "rand"), (21, 200, "rand"), (64, 512, "pair"),
         (33, 300, "rand"), (1, 200, "rand"), (2, 160, "rand"), (42, 296, "rand")]


def _pair(H, W, kind, seed):
    if kind == "pair":
        return osg.synth_pair(seed, H, W)
    rng = np.random.default_rng(seed)
    return (rng.integers(0, 256, (H, W), dtype=np.uint8), rng.integers(0, 256, (H, W), dtype=np.uint8))


@pytest.mark.parametrize("H,W,kind", SMALL)
def test_sgbm_compute_small(sv, H, W, kind):
    L, R = _pair(H, W, kind, H + W)
    assert np.array_equal(sv.disp.sgbm_compute(L, R), osg.sgbm(L, R))


# P2 <= 15 runs the q-nibble walks (C - L stored in 4 bits, kernels/sgbm.hip q_byte), larger P2 the int16
# L volumes: P2 = 15 is the largest nibble, 16 the first int16 case
@pytest.mark.parametrize("kw", [dict(block=5), dict(block=9, P1=8, P2=32), dict(uniqueness=10),
                                dict(disp12_max_diff=3, prefilter_cap=31), dict(block=1), dict(block=35),
                                dict(P1=2, P2=15), dict(P1=1, P2=15, uniqueness=0), dict(P1=8, P2=16),
                                dict(block=7, P1=14, P2=15)])
def test_sgbm_parameters(sv, kw):
    L, R = osg.synth_pair(7, 80, 400)
    L = L.copy()
    L[20:40, 200:260] = 90   # a textureless patch: ambiguous matches, uniqueness and LR rejections
    prm = sv.disp.sgbm_params(**kw)
    assert np.array_equal(sv.disp.sgbm_compute(L, R, prm), osg.sgbm(L, R, **kw)), kw


def test_sgbm_full_frame_whole_stage(sv):
    L, R = osg.synth_pair(0)
    out, raw, filt = sv.disp.stereo_disparity(L, R, 128, False, with_raw=True)
    ro, rr, rf = osg.disparity(L, R, with_raw=True)
    assert np.array_equal(raw, rr)
    assert np.array_equal(filt, rf)
    assert np.array_equal(out, ro)
    assert (raw != filt).sum() > 0            # speckles were removed
    crop = sv.disp.disparity(L, R, 128, True)
    assert crop.shape == (390, 889) and np.array_equal(crop, osg.scale(rf, 128, True))
    rec = META["scaled"]["pair0"]
    assert oracle.digest(filt) == rec["in"] and oracle.digest(out) == rec["md128_crop0"]["digest"]
    assert oracle.digest(crop) == rec["md128_crop1"]["digest"]


def test_filter_speckles_matches_oracle(sv):
    rng = np.random.default_rng(3)
    for H, W in [(1, 1), (7, 3), (40, 57), (544, 1024)]:
        img = (rng.integers(-2, 6, (H, W)) * rng.integers(1, 40)).astype(np.int16)
        for nv, ms, md in ((0, 5, 30), (0, 4000, 123), (-16, 12, 0)):
            got = img.copy()
            ret, _ = sv.disp.filterSpeckles(got, nv, ms, md)
            assert ret is got
            assert np.array_equal(got, osg.filter_speckles(img, nv, ms, md)), (H, W, nv, ms, md)


def test_int16_cost_wrap_and_range(sv):
    """A flat black left image against a white right one: every BT cost is 63,
    so a 23 x 23 block sums to 33,327 and the int16 C wraps (as in OpenCV's
    CostType buffers): the GPU reproduces the wrap. With P2 = 1000 a path
    start's L = C - P2 leaves int16: SV_E_RANGE instead of a silent mismatch."""
    L = np.zeros((40, 300), np.uint8)
    R = np.full((40, 300), 255, np.uint8)
    prm = sv.disp.sgbm_params(block=23)
    assert np.array_equal(sv.disp.sgbm_compute(L, R, prm), osg.sgbm(L, R, block=23))
    with pytest.raises(sv.svx.SvxError, match="int16"):
        sv.disp.sgbm_compute(L, R, sv.disp.sgbm_params(block=23, P2=1000))


def test_sgbm_rejects_unsupported(sv):
    z = np.zeros((10, 300), np.uint8)
    for kw in (dict(num_disp=64), dict(min_disp=1), dict(block=4)):
        with pytest.raises(sv.svx.SvxError):
            sv.disp.sgbm_compute(z, z, sv.disp.sgbm_params(**kw))
    with pytest.raises(sv.svx.SvxError):
        sv.disp.sgbm_compute(np.zeros((10, 128), np.uint8), np.zeros((10, 128), np.uint8))
    with pytest.raises(ValueError):
        sv.disp.sgbm_compute(z, z[:, :200])


def test_batch_sgbm_matches_oracle(sv):
    H, W, n, first = 544, 1024, 5, 11
    with sv.batch.Batch(n, H, W, step=1, with_bgr=False) as b:
        b.synth_pair(first)
        b.sgbm(chunk=2)                       # 3 chunks, the last partial
        for f in range(n):
            L, R = osg.synth_pair(first + f, H, W)
            assert np.array_equal(b.read_disp(f), osg.disparity(L, R)), f
        ms, cnt = b.timing("sgbm")
        assert cnt == 1 and ms > 0
        rng = np.random.default_rng(9)
        L = rng.integers(0, 256, (H, W), dtype=np.uint8)
        R = np.roll(L, -20, axis=1)
        b.upload_pair(3, L, R)
        b.sgbm()
        assert np.array_equal(b.read_disp(3), osg.disparity(L, R))


def test_batch_sgbm_crop(sv):
    """crop_disparity=True (functions.py:122-124) in the batch: 544 x 1024 pairs,
    a 390 x 889 batch (rows stored at a stride of 896) receiving
    disparity_scaled[0:390, 135:1024]; then the pre-pass and the pipeline of
    the cropped frames run fused (tests/test_gpu_anywidth.py)."""
    Hp, Wp, n, first = 544, 1024, 3, 40
    with sv.batch.Batch(n, 390, 889, step=1, with_bgr=False) as b:
        b.pair_shape(Hp, Wp)
        b.synth_pair(first)
        b.sgbm(chunk=2)
        for f in range(n):
            L, R = osg.synth_pair(first + f, Hp, Wp)
            assert np.array_equal(b.read_disp(f), osg.disparity(L, R, crop=True)), f
        rng = np.random.default_rng(4)
        L = rng.integers(0, 256, (Hp, Wp), dtype=np.uint8)
        R = np.roll(L, -30, axis=1)
        b.upload_pair(1, L, R)
        b.sgbm()
        assert np.array_equal(b.read_disp(1), osg.disparity(L, R, crop=True))
        with pytest.raises(ValueError):
            b.upload_pair(0, L[:390, :889], R[:390, :889])
        with pytest.raises(sv.svx.SvxError):
            b.pair_shape(544, 1000)            # 1000 - 135 != 889
        b.pair_shape(390, 889)                 # back to the batch's own shape: 889 % 8 != 0 for SGBM
        with pytest.raises(sv.svx.SvxError):
            b.synth_pair(0)


def _front_end(L, R):
    """oracle chain of stereovision.py:44-46: gamma 1.4 (functions.py:61-87), greyscale (:89-97)."""
    t = osg.gamma_table(1.4)
    gl, gr = t[L], t[R]
    return gl, osg.grey_equalize(gl), osg.grey_equalize(gr)


@pytest.mark.parametrize("crop", [False, True])
def test_batch_bgr_front_end(sv, crop):
    """The batch from BGR stereo pairs: preprocess() (gamma on both images,
    grey + equalizeHist -> the SGBM pairs, the corrected left image's colours
    into the batch), sgbm(), then the pipeline, whose hue histogram reads those
    colours at the disparity's own (y, x) — the top-left of the uncropped image
    when the disparity is cropped (functions.py:178-196)."""
    Hp, Wp, n = (544, 1024, 1) if crop else (96, 320, 3)
    H, W = (390, 889) if crop else (Hp, Wp)
    rng = np.random.default_rng(31 + crop)
    pairs = []
    for f in range(n):
        L = rng.integers(0, 256, (Hp, Wp, 3), dtype=np.uint8)
        pairs.append((L, np.roll(L, -(12 + 5 * f), axis=1)))
    plane = (0.0, 0.0, 0.01)
    with sv.batch.Batch(n, H, W, step=1, with_bgr=True, with_points=True) as b:
        if crop:
            b.pair_shape(Hp, Wp)
        for f, (L, R) in enumerate(pairs):
            b.upload_bgr_pair(f, L, R)
        b.preprocess(1.4)
        b.sgbm()
        b.pipeline(plane=plane, point_thr=1e9, hist_thr=2)
        counts = b.read_counts()
        for f, (L, R) in enumerate(pairs):
            gl, grey_l, grey_r = _front_end(L, R)
            d = osg.disparity(grey_l, grey_r, crop=crop)
            assert np.array_equal(b.read_disp(f), d), f
            ref = oracle.pipeline_frame(d, np.ascontiguousarray(gl[:H, :W]), 1, abc=np.array(plane), point_thr=1e9,
                                        hist_thr=2)
            assert tuple(int(v) for v in counts[f]) == ref["counts"], f
            assert np.array_equal(b.read_hist(f), ref["hist"]), f
            assert np.array_equal(b.read_points(f)[1], ref["pts"]), f
    with sv.batch.Batch(1, 544, 320, with_bgr=False) as b:
        with pytest.raises(sv.svx.SvxError):
            b.preprocess()                         # no BGR pairs
        b.synth_bgr_pair(5)                        # rows below 200 see the synthetic road's disparity
        b.preprocess()
        b.sgbm()
        assert b.read_disp(0)[300:].any()


def test_batch_preprocess_leaves_pairs_raw(sv):
    """preprocess() corrects the stored pairs as it reads them: a second call
    gives the same SGBM pairs, disparity and colours as the first (the
    reference corrects each pair once, stereovision.py:44)."""
    with sv.batch.Batch(2, 96, 320, step=1, with_bgr=True, with_points=True) as b:
        b.synth_bgr_pair(3)
        plane = (0.0, 0.0, 0.01)
        runs = []
        for _ in range(3):
            b.preprocess(1.4)
            b.sgbm()
            b.pipeline(plane=plane, point_thr=1e9, hist_thr=2)
            runs.append((b.read_disp(0), b.read_disp(1), b.read_counts(), b.read_hist(0), b.read_points(1)[1]))
        for r in runs[1:]:
            for a, c in zip(runs[0], r):
                assert np.array_equal(a, c)


def test_dropin_installed_module(sv):
    """functions.disparity / greyscale / preProcessImages patched into a module
    object; a stereoProcessor with OpenCV's getters is honoured."""
    mod = types.SimpleNamespace(camera_focal_length_px=399.9745178222656, stereo_camera_baseline_m=0.2090607502,
                                image_centre_w=474.5, image_centre_h=262.0)
    sv.dropin.install(mod, unpinned=True)   # disparity / greyscale restate cv2 (opt-in)
    try:
        L, R = osg.synth_pair(2, 128, 384)
        assert np.array_equal(mod.disparity(L, R, 128, False), osg.disparity(L, R))

        class Proc:
            def __getattr__(self, name):
                vals = dict(getMinDisparity=0, getNumDisparities=128, getBlockSize=7, getP1=4, getP2=40,
                            getDisp12MaxDiff=2, getPreFilterCap=20, getUniquenessRatio=5, getSpeckleWindowSize=0,
                            getMode=0)
                return lambda: vals[name]
        mod.stereoProcessor = Proc()
        exp = osg.scale(osg.filter_speckles(osg.sgbm(L, R, block=7, P1=4, P2=40, disp12_max_diff=2, prefilter_cap=20,
                                                     uniqueness=5)), 128, False)
        assert np.array_equal(mod.disparity(L, R, 128, False), exp)
        gl, gr = mod.greyscale(*mod.preProcessImages(np.dstack([L] * 3), np.dstack([R] * 3)))
        assert gl.shape == L.shape and gl.dtype == np.uint8
    finally:
        sv.dropin.uninstall()


def test_front_end_from_png_files(sv, tmp_path):
    """loop.py:70-76 then stereovision.py:44-56 from files, through the installed drop-ins: getImagePaths ->
    loadImages (svx.io, PNG ingest) -> preProcessImages -> greyscale -> disparity, against the oracle on the pixels
    the files hold (the PNG round trip is lossless; one file interlaced, the other not)."""
    from test_io_cpu import write_png
    L, R = osg.synth_pair(4)   # a whole 544 x 1024 frame: its regions outlast filterSpeckles' 4000 pixels
    rng = np.random.default_rng(4)
    bgr_l = np.clip(np.dstack([L] * 3).astype(np.int32) + rng.integers(0, 40, 3), 0, 255).astype(np.uint8)
    bgr_r = np.clip(np.dstack([R] * 3).astype(np.int32) + rng.integers(0, 40, 3), 0, 255).astype(np.uint8)
    dl, dr = tmp_path / "left", tmp_path / "right"
    dl.mkdir()
    dr.mkdir()
    write_png(str(dl / "1506942473.484027_L.png"), bgr_l[..., ::-1], 2, filters=(4, 1, 2, 3, 0), interlace=1)
    write_png(str(dr / "1506942473.484027_R.png"), bgr_r[..., ::-1], 2)
    mod = types.SimpleNamespace(camera_focal_length_px=399.9745178222656, stereo_camera_baseline_m=0.2090607502,
                                image_centre_w=474.5, image_centre_h=262.0)
    sv.dropin.install(mod, unpinned=True)   # the PNG readers and the cv2 restatements are opt-in
    try:
        paths = mod.getImagePaths("1506942473.484027_L.png", str(dl), str(dr))
        img_l, img_r = mod.loadImages(paths)
        assert np.array_equal(img_l, bgr_l) and np.array_equal(img_r, bgr_r)
        img_l, img_r = mod.preProcessImages(img_l, img_r)
        gray_l, gray_r = mod.greyscale(img_l, img_r)
        disp = mod.disparity(gray_l, gray_r, 128, False)
        t = np.asarray(META["gamma"]["1.4"], np.uint8)
        exp = osg.disparity(osg.grey_equalize(t[bgr_l]), osg.grey_equalize(t[bgr_r]))
        assert np.array_equal(disp, exp)
        assert disp.any()
    finally:
        sv.dropin.uninstall()
