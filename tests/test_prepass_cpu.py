"""Pre-pass and road-raster restatements (oracle) against the reference-run
fixtures of tests/golden/make_prepass_golden.py. CPU only."""
import json
import os

import numpy as np

import oracle
from conftest import GOLDEN

import sys
sys.path.insert(0, GOLDEN)
import prepass_inputs  # noqa: E402
import roadmap_inputs  # noqa: E402

META = json.load(open(os.path.join(GOLDEN, "prepass.json")))


def carmask():
    z = np.load(os.path.join(GOLDEN, "carmask.npz"))
    shape = tuple(int(v) for v in z["shape"])
    return np.unpackbits(z["bits"])[: shape[0] * shape[1]].reshape(shape).astype(np.uint8) * 255


def test_carmask_fixture():
    m = carmask()
    assert m.shape == (544, 1024)
    assert int((m != 0).sum()) == META["carmask_nonzero"]
    assert oracle.digest((m != 0).astype(np.uint8)) == META["carmask_digest"]


def test_fill_mean_matches_reference():
    for d, ref in zip(prepass_inputs.fill_mean_inputs(oracle.synth_frame), META["fill_mean"]):
        assert oracle.digest(d) == ref["in"]
        assert oracle.digest(oracle.fill_mean(d)) == ref["out"]


def test_road_raster_matches_reference(golden):
    for fid, ref in META["road_raster_step2"].items():
        m = golden.meta["full_frames_step2"][fid]
        disp, bgr = oracle.synth_frame(0 if fid == "0r" else int(fid))
        pp = oracle.pipeline_frame(disp, bgr, 2, abc=np.array(m["abc"]))["pts"].reshape(-1, 1, 2)
        img = oracle.road_raster(pp)
        assert oracle.digest(img) == ref["image"] and int((img != 0).sum()) == ref["nonzero"]
        nzp = oracle.nonzero_points(img)
        assert len(nzp) == ref["nonzero"]
        assert (np.diff(nzp[:, 1] * 1024 + nzp[:, 0]) > 0).all()   # raster order


def test_road_map_matches_reference():
    """stereovision.py:131-133 (imageRoadMap) restated by oracle.road_map, against the
    reference's own statements run on the same planePoints (tests/golden/roadmap.json)."""
    meta = json.load(open(os.path.join(GOLDEN, "roadmap.json")))
    seen = set()
    for name, bgr, pp in roadmap_inputs.cases(oracle.digest):
        ref = meta["cases"][name]
        assert oracle.digest(pp) == ref["points_digest"]
        img = oracle.road_map(bgr, pp)
        green = int(((img[..., 0] == 0) & (img[..., 1] == 255) & (img[..., 2] == 0)).sum())
        assert oracle.digest(img) == ref["image"] and green == ref["green"], name
        seen.add(name)
    assert seen == set(meta["cases"])
    import pytest
    with pytest.raises(IndexError):
        oracle.road_map(bgr, np.array([[[1024, 0]]], np.int32))


def test_fill_previous_semantics():
    for d, p in prepass_inputs.fill_prev_inputs():
        out = oracle.fill_previous(d, p)
        low = d <= 2
        assert np.array_equal(out[~low], d[~low])
        assert np.array_equal(out[low], np.minimum(d[low].astype(int) + p[low], 255))
    chain = oracle.fill_previous_chain([np.full((2, 4), v, np.uint8) for v in (0, 1, 3, 0)])
    assert [int(c[0, 0]) for c in chain] == [0, 1, 3, 3]
