"""The per-frame golden digests (tests/golden/frame_digests.npz) against the
pinned oracle: the file's rows are what the oracle computes for those frames,
and at step 2 its counts are the reference's own (tests/golden/digests.json,
produced by running functions.py). CPU only; the GPU side of the comparison is
tests/test_gpu_digests.py."""
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN


@pytest.fixture(scope="module")
def fd():
    return np.load(os.path.join(GOLDEN, "frame_digests.npz"))


def test_shapes(fd):
    assert fd["step1"].shape == (32768,) and fd["step2"].shape == (4096,)
    assert fd["step1"].dtype.names == oracle.DIGEST_FIELDS


@pytest.mark.parametrize("frame", [0, 1, 2047, 4095, 4096, 12345, 28672, 32767])
def test_step1_rows_recompute(fd, frame):
    assert oracle.frame_digest(frame, 1) == tuple(int(v) for v in fd["step1"][frame])


@pytest.mark.parametrize("frame", [0, 1, 777, 4095])
def test_step2_rows_recompute(fd, frame):
    assert oracle.frame_digest(frame, 2) == tuple(int(v) for v in fd["step2"][frame])


@pytest.mark.parametrize("fid", ["0", "1", "4095"])
def test_step2_counts_are_the_references(fd, golden, fid):
    m = golden.meta["full_frames_step2"][fid]
    row = fd["step2"][int(fid)]
    assert (int(row["n_valid"]), int(row["n_kept"]), int(row["n_kept2"])) == (m["n"], m["n_kept"], m["n_kept2"])


def test_every_frame_is_non_trivial(fd):
    for key in ("step1", "step2"):
        a = fd[key]
        assert (a["n_kept2"] > 0).all() and (a["n_kept2"] <= a["n_kept"]).all() and (a["n_kept"] <= a["n_valid"]).all()
        assert len(np.unique(a["disp_hash"])) == len(a)      # every frame distinct


def test_plane_digests_rows_recompute():
    """tests/golden/plane_digests.npz (the per-frame-plane loop through the oracle:
    fill pre-pass chain + carmask -> maskpoints -> RANSAC(600), random.seed(F) ->
    the step-1 pipeline with that plane) recomputed for frames 0..2 and for a
    block starting at frame 640 from its predecessor's cleaned frame."""
    import sys
    sys.path.insert(0, GOLDEN)
    import make_plane_digests as mpd
    z = np.load(os.path.join(GOLDEN, "plane_digests.npz"))
    gold = z["planes"]
    assert gold.shape == (8192,) and int(z["trials"]) == 600 and int(z["seed_base"]) == 0
    assert (gold["trial"] >= 0).all() and (gold["n_kept2"] > 0).all()
    prev = None
    for f in range(640):
        d, _ = oracle.synth_frame(f)
        prev = d.copy() if prev is None else oracle.fill_previous(d, prev)
    rows = mpd._block((0, 3, None, 0)) + mpd._block((640, 1, prev, 0))
    for r in rows:
        g = gold[r[0]]
        assert r[1] == g["n_maskpoints"] and r[2] == g["trial"], r[0]
        assert np.array_equal(np.asarray(r[5]).view(np.uint64), g["abc"].view(np.uint64)), r[0]
        assert tuple(r[6:]) == tuple(int(g[n]) for n in oracle.DIGEST_FIELDS), r[0]
