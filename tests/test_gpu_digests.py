"""Every frame at BASELINE.json's full sizes against the oracle.

The device summarises its own outputs per frame (sv_batch_digest,
kernels/digest.hip): the counts, hashes of the disparity, of the hue histogram
and of the surviving points in order (source pixel, disparity, int32
back-projection) and a count of outputs whose fp32 X, Y, Z are not within 1e-5
relative of the fp64 reference values. Those rows must equal
tests/golden/frame_digests.npz, written by the pinned C oracle
(tests/golden/make_frame_digests.py), for EVERY frame:
  * configs[2]: K1 dense projection of 4096 frames (counts, disparity, tolerance)
  * configs[3]: the pipeline over 4096 frames, resident and tiled kernels, steps 1 and 2
  * configs[4]: all 32,768 frames, generated and processed shard by shard as
    the 8 ranks would (4096 frames each, global frame ids), on one GPU.
  * the per-frame-plane loop (stereovision.py:53-113 for every frame of the
    batch: fill pre-pass + carmask -> maskpoints -> RANSAC(600) with
    random.seed(F) -> the pipeline with that frame's plane) against
    tests/golden/plane_digests.npz, the oracle's chain (make_plane_digests.py)."""
import os
import types

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FIELDS = ("n_valid", "n_kept", "n_kept2", "disp_hash", "hist_hash", "pts_hash")


@pytest.fixture(scope="module")
def env():
    import svx
    from svx import batch
    assert svx.device_count() >= 1
    return types.SimpleNamespace(batch=batch, fd=np.load(os.path.join(GOLDEN, "frame_digests.npz")))


def _mismatches(got, want, fields):
    """frames whose digest row differs (field names), plus frames with bad outputs"""
    bad = []
    for k, name in enumerate(FIELDS):
        if name in fields:
            diff = np.flatnonzero(got[:, k] != want[name].astype(np.uint64))
            bad += [(int(i), name) for i in diff[:5]]
    nb = np.flatnonzero(got[:, 6] != 0)
    bad += [(int(i), f"bad={int(got[i, 6])}") for i in nb[:5]]
    return bad


def test_dense_every_frame_step1(env):
    frames = 4096
    want = env.fd["step1"][:frames]
    with env.batch.Batch(frames, step=1, with_bgr=False) as b:
        b.synth(0)
        b.project()
        got = b.digest("dense")
    assert _mismatches(got, want, ("n_valid", "disp_hash")) == []


@pytest.mark.parametrize("step", [1, 2])
def test_pipeline_every_frame(env, step):
    frames = 4096
    want = env.fd[f"step{step}"][:frames]
    with env.batch.Batch(frames, step=step, with_bgr=True, with_points=True) as b:
        b.synth(0)
        for mode in ("resident", "tiled"):
            b.pipeline_mode(mode)
            b.pipeline()
            got = b.digest("pipeline")
            assert _mismatches(got, want, FIELDS) == [], mode


def test_config5_every_shard(env):
    """32,768 frames = 8 shards of 4096 global frame ids (svx.dist.shard), each
    generated on the device from its global ids and run through the pipeline."""
    from svx import dist
    want_all = env.fd["step1"]
    with env.batch.Batch(4096, step=1, with_bgr=True, with_points=True) as b:
        for rank in range(8):
            first, count = dist.shard(32768, 8, rank)
            assert count == 4096
            b.synth(first)
            b.pipeline()
            got = b.digest("pipeline")
            assert _mismatches(got, want_all[first:first + count], FIELDS) == [], f"shard {rank}"


def test_frame_planes_every_frame(env):
    """bench.py's pipeline_frame_planes workload, all 4096 frames end to end: every
    frame's RANSAC picks the oracle's winning trial, with the oracle's error and plane
    bit for bit (np.dot(np.linalg.inv(P), ones) and np.mean of functions.py:267-289:
    the device restates numpy's LAPACK solve and summation order), and every frame's
    pipeline digest — counts, histogram, the surviving points and their int32
    back-projection — equals the oracle chain's."""
    import sys
    sys.path.insert(0, GOLDEN)
    from test_prepass_cpu import carmask
    z = np.load(os.path.join(GOLDEN, "plane_digests.npz"))
    want = z["planes"][:4096]   # the file holds 8192 frames (the frame loop's sequence tests use them all)
    frames = len(want)
    with env.batch.Batch(frames, step=1, with_bgr=True, with_points=True) as b:
        b.synth(0)
        b.set_mask(carmask())
        b.prepass("previous")
        b.ransac(seed_base=int(z["seed_base"]), trials=int(z["trials"]))
        b.pipeline_planes()
        got = b.digest("pipeline")
        bad_planes, bad_trials, bad_errs = [], [], []
        for f in range(frames):
            r = b.read_ransac(f)
            if r["trial"] != int(want["trial"][f]):
                bad_trials.append(f)
            if not np.array_equal(np.asarray(r["abc"], np.float64).view(np.uint64), want["abc"][f].view(np.uint64)):
                bad_planes.append(f)
            if r["err"] != want["err"][f]:
                bad_errs.append(f)
    assert bad_trials == [], bad_trials[:10]
    assert bad_planes == [] and bad_errs == [], (len(bad_planes), bad_planes[:10], len(bad_errs), bad_errs[:10])
    mism = _mismatches(got, want, FIELDS)
    assert mism == [], mism


@pytest.mark.parametrize("hist_thr", [10, 30, 0])
def test_resident_edge_frames(env, hist_thr):
    """The frame-resident kernel (forced, 6 frames) on frames that take its rare paths, against the oracle:
    every grid point valid and kept (a chunk's 4096 outputs wrap onto the carried tail: the early flush),
    ~300 valid points of random colour (every bin ends <= hist_thr: pass 1's drop list), ~3000 such points
    (more drops than the list holds: the candidate-chunk re-read), and two synthetic frames."""
    import oracle
    rng = np.random.default_rng(hist_thr + 1)
    H, W = 544, 1024
    frames = []
    full = rng.integers(1, 256, (H, W)).astype(np.uint8)
    frames.append((full, rng.integers(100, 104, (H, W, 3)).astype(np.uint8)))
    for n in (300, 3000):
        d = np.zeros((H, W), np.uint8)
        d[rng.integers(0, H - 1, n), rng.integers(0, W - 1, n)] = rng.integers(1, 256, n)
        frames.append((d, rng.integers(0, 256, (H, W, 3)).astype(np.uint8)))
    frames.append((full, rng.integers(0, 256, (H, W, 3)).astype(np.uint8)))
    frames += [oracle.synth_frame(f) for f in (5, 6)]
    kw = dict(plane=(0.0, 0.0, 0.01), point_thr=1e9, hist_thr=hist_thr)
    with env.batch.Batch(len(frames), step=1, with_bgr=True, with_points=True) as b:
        b.pipeline_mode("resident")
        for f, (d, bgr) in enumerate(frames):
            b.upload(f, d, bgr)
        for rep in range(2):
            b.pipeline(**kw)
            counts = b.read_counts()
            for f, (d, bgr) in enumerate(frames):
                ref = oracle.pipeline_frame(d, bgr, 1, abc=np.array(kw["plane"]), point_thr=1e9, hist_thr=hist_thr)
                assert tuple(int(v) for v in counts[f]) == ref["counts"], (rep, f)
                assert np.array_equal(b.read_hist(f)[:1000], ref["hist"][:1000]), (rep, f)
                assert np.array_equal(b.read_points(f)[1], ref["pts"]), (rep, f)
