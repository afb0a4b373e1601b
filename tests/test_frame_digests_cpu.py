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
