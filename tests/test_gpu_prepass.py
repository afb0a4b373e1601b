"""Pre-pass (functions.py:131-172) and road raster / non-zero walk
(functions.py:339-365) on the GPU against the oracle restatements and the
reference-run fixtures (tests/golden/prepass.json)."""
import json
import os
import sys
import types

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
import prepass_inputs  # noqa: E402
from test_prepass_cpu import carmask  # noqa: E402

pytestmark = pytest.mark.gpu
META = json.load(open(os.path.join(GOLDEN, "prepass.json")))


@pytest.fixture(scope="module")
def svx_mod():
    import svx
    from svx import batch, dropin
    assert svx.device_count() >= 1
    return types.SimpleNamespace(svx=svx, batch=batch, dropin=dropin)


def test_fill_mean_reference_fixture(svx_mod):
    for d, ref in zip(prepass_inputs.fill_mean_inputs(oracle.synth_frame), META["fill_mean"]):
        work = d.copy()
        out = svx_mod.dropin.fillAltDisparity(work)
        assert out is work                                   # in place, like the reference
        assert oracle.digest(out) == ref["out"]
    strided = prepass_inputs.fill_mean_inputs(oracle.synth_frame)[0][:, ::2].copy()[:, :500]
    view = np.zeros((544, 1000), np.uint8)[:, ::2]
    view[...] = strided
    svx_mod.dropin.fillAltDisparity(view)
    assert np.array_equal(view, oracle.fill_mean(strided))


def test_fill_previous(svx_mod):
    for d, p in prepass_inputs.fill_prev_inputs():
        assert np.array_equal(svx_mod.dropin.fillDisparity(d, p), oracle.fill_previous(d, p))
        assert svx_mod.dropin.fillDisparity(d, None) is d


def test_mask_and_cap(svx_mod):
    m = carmask()
    d, _ = oracle.synth_frame(9)
    f = types.SimpleNamespace(carmask=m)
    svx_mod.dropin.install(f, unpinned=True)   # maskDisparity restates cv2 (not in the default set)
    try:
        assert np.array_equal(f.maskDisparity(d), oracle.mask_disparity(d, m))
        assert f.capDisparity(d) is d
    finally:
        svx_mod.dropin.uninstall()
    odd = np.arange(7 * 13, dtype=np.uint8).reshape(7, 13)
    mo = (np.arange(7 * 13).reshape(7, 13) % 3).astype(np.uint8)
    assert np.array_equal(svx_mod.dropin.mask_disparity(odd, mo), oracle.mask_disparity(odd, mo))


@pytest.mark.parametrize("option", ["previous", "mean", "none"])
def test_batch_prepass(svx_mod, option):
    frames, first = 6, 200
    m = carmask()
    rng = np.random.default_rng(5)
    raw = []
    for f in range(frames):
        d, _ = oracle.synth_frame(first + f)
        d = d.copy()
        d[rng.random(d.shape) < 0.2] = rng.integers(0, 3)
        raw.append(d)
    prev0 = rng.integers(0, 256, (544, 1024)).astype(np.uint8)
    with svx_mod.batch.Batch(frames, with_bgr=False) as b:
        for f, d in enumerate(raw):
            b.upload(f, d)
        b.set_mask(m)
        b.prepass(option, prev0=prev0 if option == "previous" else None)
        if option == "previous":
            ref = oracle.fill_previous_chain(raw, prev0)
        elif option == "mean":
            ref = [oracle.fill_mean(d) for d in raw]
        else:
            ref = raw
        for f in range(frames):
            dc, dm = b.read_disp(f, masked=True)
            assert np.array_equal(dc, ref[f]), f
            assert np.array_equal(dm, oracle.mask_disparity(ref[f], m)), f
    with svx_mod.batch.Batch(3, with_bgr=False) as b:   # no prev0: frame 0 is left as is
        for f in range(3):
            b.upload(f, raw[f])
        b.prepass("previous")
        ref = oracle.fill_previous_chain(raw[:3])
        for f in range(3):
            assert np.array_equal(b.read_disp(f), ref[f])


@pytest.mark.parametrize("frames", [130, 300, 520])
@pytest.mark.parametrize("with_prev0", [False, True])
def test_batch_fill_previous_long(svx_mod, frames, with_prev0):
    """fillDisparity's frame recurrence (functions.py:141-148, stereovision.py:56-60) over hundreds of frames:
    columns that stay 0 throughout (each frame takes prev0 or 0), columns of 1s and 2s whose sums saturate at
    255, columns mostly <= 2, columns that switch from 0 to 7 mid-batch, and synthetic frames, against the
    oracle chain, twice on one batch."""
    H, W = 32, 256
    rng = np.random.default_rng(frames + with_prev0)
    raw = rng.integers(3, 256, (frames, H, W)).astype(np.uint8)
    raw[:, :, :16] = 0                                                    # open in every group
    raw[:, :, 16:32] = rng.integers(1, 3, (frames, H, 16))                # accumulate and saturate
    low = rng.random((frames, H, 64)) < 0.97
    raw[:, :, 32:96] = np.where(low, rng.integers(0, 3, (frames, H, 64)), raw[:, :, 32:96])
    raw[:, :, 96:100] = 0
    raw[frames // 2:, :, 96:100] = 7                                      # opens, then closes mid-batch
    for f in range(frames):
        raw[f, :, 128:] = oracle.synth_frame(f, H=H, W=W)[0][:, 128:]
    prev0 = rng.integers(0, 256, (H, W)).astype(np.uint8) if with_prev0 else None
    with svx_mod.batch.Batch(frames, H=H, W=W, with_bgr=False) as b:
        for f in range(frames):
            b.upload(f, raw[f])
        for rep in range(2):   # the second run re-uses the batch's scratch (flags reset per launch)
            if rep:
                for f in range(frames):
                    b.upload(f, raw[f])
            b.prepass("previous", prev0=prev0)
            ref = oracle.fill_previous_chain(list(raw), prev0)
            for f in range(frames):
                assert np.array_equal(b.read_disp(f), ref[f]), (rep, f)


def test_road_raster_reference_fixture(svx_mod, golden):
    for fid, ref in META["road_raster_step2"].items():
        m = golden.meta["full_frames_step2"][fid]
        disp, bgr = oracle.synth_frame(0 if fid == "0r" else int(fid))
        pp = oracle.pipeline_frame(disp, bgr, 2, abc=np.array(m["abc"]))["pts"].reshape(-1, 1, 2)
        img = svx_mod.dropin.generatePointsAsImage(pp)
        assert oracle.digest(img) == ref["image"]
        nzp = svx_mod.dropin.nonzero_points(img)
        assert np.array_equal(nzp, oracle.nonzero_points(img))
    assert svx_mod.dropin.road_raster(np.zeros((0, 1, 2), np.int32)).sum() == 0
    img = svx_mod.dropin.road_raster(np.array([[[-1, -1]], [[3, 0]]], np.int32), (4, 8))   # numpy wraps negatives
    assert img[3, 7] == 255 and img[0, 3] == 255 and int((img != 0).sum()) == 2
    with pytest.raises(IndexError):
        svx_mod.dropin.road_raster(np.array([[8, 0]], np.int32), (4, 8))
    odd = (np.random.default_rng(1).random((9, 13)) < 0.3).astype(np.uint8) * 7
    assert np.array_equal(svx_mod.dropin.nonzero_points(odd), oracle.nonzero_points(odd))


@pytest.mark.parametrize("step", [1, 2])
@pytest.mark.parametrize("bits", [False, True])
def test_batch_road_raster_and_walk(svx_mod, step, bits):
    """bits: the resident pipeline writes the road bitmap and the road pass reads it (sv_batch_road_bits; step 1,
    1024-wide frames; at step 2 the points path runs either way)."""
    frames, first = 5, 321
    with svx_mod.batch.Batch(frames, step=step, with_bgr=True, with_points=True) as b:
        b.synth(first)
        if bits:
            b.pipeline_mode("resident")
            b.road_bits(True)
        b.pipeline()
        b.road_raster()
        b.nonzero()
        for f in range(frames):
            disp, bgr = oracle.synth_frame(first + f)
            ref = oracle.pipeline_frame(disp, bgr, step)
            rimg = oracle.road_raster(ref["pts"])
            img, walk = b.read_road(f, walk=True)
            assert np.array_equal(img, rimg)
            assert np.array_equal(walk, oracle.nonzero_points(rimg))


@pytest.mark.parametrize("step", [1, 2])
@pytest.mark.parametrize("bits", [False, True])
def test_batch_road_edge_frames(svx_mod, step, bits):
    """The fused road pass (bands of rows in LDS, a cursor over the raster-ordered points) on frames with no
    point, every grid point, points on a few scattered rows only, and random disparity: image and walk equal
    the oracle's generatePointsAsImage and its raster-order walk."""
    rng = np.random.default_rng(7)
    H, W = 544, 1024
    frames = []
    frames.append(np.zeros((H, W), np.uint8))
    frames.append(np.full((H, W), 255, np.uint8))
    sparse = np.zeros((H, W), np.uint8)
    for r in (0, 1, 37, 38, 200, 411, 542, 543):
        sparse[r, rng.integers(0, W, 40)] = rng.integers(1, 256, 40)
    frames.append(sparse)
    frames.append(rng.integers(0, 256, (H, W)).astype(np.uint8))
    bgr = rng.integers(0, 256, (H, W, 3)).astype(np.uint8)
    kw = dict(plane=(0.0, 0.0, 0.01), point_thr=1e9, hist_thr=0)
    with svx_mod.batch.Batch(len(frames), H=H, W=W, step=step, with_bgr=True, with_points=True) as b:
        for f, d in enumerate(frames):
            b.upload(f, d, bgr)
        if bits:
            b.pipeline_mode("resident")
            b.road_bits(True)
        b.pipeline(**kw)
        b.road_map(True)
        b.road_raster()
        b.nonzero()
        for f, d in enumerate(frames):
            ref = oracle.pipeline_frame(d, bgr, step, abc=np.array(kw["plane"]), point_thr=1e9, hist_thr=0)
            rimg = oracle.road_raster(ref["pts"])
            img, walk = b.read_road(f, walk=True)
            assert np.array_equal(img, rimg), f
            assert np.array_equal(walk, oracle.nonzero_points(rimg)), f
            assert np.array_equal(b.read_road_map(f), oracle.road_map(bgr, ref["pts"])), f


def test_batch_road_map_reference_fixture(svx_mod, golden):
    """stereovision.py:131-133 (imageRoadMap) from the batch's road pass against the
    reference's own statements run on the same planePoints (tests/golden/roadmap.json),
    for the golden step-2 chains (each with its plane) and frame 0 at step 1; then a
    crop-width batch (390 x 889 frames at a row stride of 896)."""
    meta = json.load(open(os.path.join(GOLDEN, "roadmap.json")))["cases"]
    for fid, m in golden.meta["full_frames_step2"].items():
        disp, bgr = oracle.synth_frame(0 if fid == "0r" else int(fid))
        with svx_mod.batch.Batch(1, step=2, with_bgr=True, with_points=True) as b:
            b.upload(0, disp, bgr)
            b.pipeline(plane=tuple(m["abc"]))
            b.road_map(True)
            b.road_raster()
            out = b.read_road_map(0)
            assert oracle.digest(out) == meta[f"step2_{fid}"]["image"], fid
    with svx_mod.batch.Batch(3, step=1, with_bgr=True, with_points=True) as b:
        b.synth(0)
        b.pipeline()
        with pytest.raises(svx_mod.svx.SvxError):
            b.read_road_map(0)                   # not requested yet
        b.road_map(True)
        b.road_raster(sync=False)
        b.nonzero()
        assert oracle.digest(b.read_road_map(0)) == meta["step1_0"]["image"]
        for f in (1, 2):
            disp, bgr = oracle.synth_frame(f)
            assert np.array_equal(b.read_road_map(f), oracle.road_map(bgr, oracle.pipeline_frame(disp, bgr, 1)["pts"]))
    with svx_mod.batch.Batch(2, 390, 889, step=1, with_bgr=True, with_points=True) as b:
        frames = []
        for f in range(2):
            d, bgr = oracle.synth_frame(60 + f)
            d, bgr = np.ascontiguousarray(d[:390, :889]), np.ascontiguousarray(bgr[:390, :889])
            frames.append((d, bgr))
            b.upload(f, d, bgr)
        b.pipeline()
        b.road_map(True)
        b.road_raster()
        for f, (d, bgr) in enumerate(frames):
            ref = oracle.pipeline_frame(d, bgr, 1)
            assert np.array_equal(b.read_road_map(f), oracle.road_map(bgr, ref["pts"])), f
    with svx_mod.batch.Batch(1, step=1, with_bgr=False) as b:
        with pytest.raises(svx_mod.svx.SvxError):
            b.road_map(True)                     # needs the batch's BGR
