"""Batched on-device RANSAC (sv_batch_ransac): per frame, maskpoints =
projectDisparityTo3d(maskDisparity(d), 128) (stereovision.py:85) and
RANSAC(maskpoints, trials) (functions.py:278-298) with the draws CPython makes
after random.seed(seed_base + frame). Checked against the reference-run
fixtures (tests/golden/ransac.json: the reference's RANSAC on synthetic frame
0/1's maskpoints under seeds 0, 1, 12345, 7) and against the oracle
restatement driven by random.Random(seed) for many frames, both branches of
random.sample, two-word seeds, k != 600 and n < k.

Tolerance: none. The device solves each trial's 3 x 3 system with numpy's
rounding (the dgesv + dot of functions.py:267 restated, oracle svo_plane_lapack,
pinned to numpy in tests/test_ransac_cpu.py) and sums each candidate's error in
numpy's order (the gemv fmas, np.mean's pairwise sum), so the winning trial, its
error and the plane must equal the reference's bit for bit on every frame."""
import random

import numpy as np
import pytest

import oracle
from oracle import ransac as oransac
from test_prepass_cpu import carmask
from test_ransac_cpu import FIX

pytestmark = pytest.mark.gpu

H, W = 544, 1024


@pytest.fixture(scope="module")
def svb():
    import svx
    from svx import batch
    assert svx.device_count() >= 1
    return batch


def _abc_from_bits(b):
    return np.array([int(x, 16) for x in b], np.uint64).view(np.float64)


def _oracle_frame(pts, trials, seed, k=600):
    r = random.Random(seed)
    best, recs = oransac.ransac(pts, trials, k=k, rng=r)
    errs = [rec.get("err") for rec in recs]
    if best is None:
        return None, -1, None
    cand = [(e, t) for t, e in enumerate(errs) if e is not None]
    e, t = min(cand)   # first strict minimum == min over (err, index)
    return best.reshape(3), t, e


def _bits(a):
    return np.ascontiguousarray(np.asarray(a, np.float64)).view(np.uint64)


def _check(res, ref_abc, ref_t, ref_e, what):
    if ref_abc is None:
        assert res["trial"] == -1, what
        return
    assert res["trial"] == ref_t, (what, res["trial"], ref_t)
    assert res["err"] == ref_e, (what, res["err"], ref_e)
    assert np.array_equal(_bits(res["abc"]), _bits(ref_abc)), (what, res["abc"], ref_abc)


def _check_draws(b, frame, pts, seed, trials, k=600):
    tr = b.read_ransac_trace(frame)
    assert tr.shape == (trials, k + 3)
    _, recs = oransac.ransac(pts, trials, k=k, rng=random.Random(seed))
    for t, rec in enumerate(recs[: len(tr)]):
        got = list(tr[t, :k])
        if got != rec["idx"]:
            j = next(i for i in range(k) if got[i] != rec["idx"][i])
            raise AssertionError(f"frame {frame} trial {t}: sample differs first at {j}: "
                                 f"{got[max(0, j - 2):j + 3]} vs {rec['idx'][max(0, j - 2):j + 3]}")
        assert tuple(tr[t, k:]) == rec["tri"], (frame, t, tuple(tr[t, k:]), rec["tri"])


def test_batch_draws_match_cpython(svb):
    """The drawn indices themselves (trial samples and triples) equal CPython's."""
    m = carmask()
    with svb.Batch(2, H=H, W=W, step=2, with_bgr=False) as b:
        b.synth(0)
        b.set_mask(m)
        b.ransac_trace(4)
        b.ransac(seed_base=0, trials=4)
        for f in range(2):
            _check_draws(b, f, b.read_maskpoints(f), f, 4)


def test_batch_matches_reference_fixtures(svb):
    m = carmask()
    with svb.Batch(2, H=H, W=W, step=2, with_bgr=False) as b:
        b.synth(0)
        b.set_mask(m)
        for key, ref in FIX.items():
            name, seed = key.split("/")
            if name not in ("frame0", "frame1"):
                continue
            frame = int(name[-1])
            b.ransac(seed_base=int(seed) - frame, trials=ref["trials"])
            res = b.read_ransac(frame)
            assert res["trial"] >= 0, (key, res)
            assert np.array_equal(_bits(res["abc"]), _bits(_abc_from_bits(ref["abc_bits"]))), (key, res)


def test_batch_maskpoints_bit_exact(svb):
    m = carmask()
    with svb.Batch(3, H=H, W=W, step=1, with_bgr=False) as b:
        b.synth(5)
        b.set_mask(m)
        b.ransac(seed_base=0, trials=1)
        for f in range(3):
            d, _ = oracle.synth_frame(5 + f)
            ref, _ = oracle.project(oracle.mask_disparity(d, m), None, 2)
            got = b.read_maskpoints(f)
            assert got.shape == ref.shape and np.array_equal(got.view(np.uint64), ref.view(np.uint64)), f


def test_batch_many_frames_vs_oracle(svb):
    m = carmask()
    frames, trials, base = 6, 40, 1000
    with svb.Batch(frames, H=H, W=W, step=2, with_bgr=False) as b:
        b.synth(20)
        b.set_mask(m)
        b.ransac(seed_base=base, trials=trials, first_frame=20)
        for f in range(frames):
            pts = b.read_maskpoints(f)
            ref = _oracle_frame(pts, trials, base + 20 + f)
            _check(b.read_ransac(f), *ref, what=f"frame {f}")


def _sparse_frame(n, seed):
    """A disparity whose step-2 grid holds exactly n non-zero points at random places."""
    rng = np.random.default_rng(seed)
    hg, wg = H // 2, W // 2
    cells = rng.choice(hg * wg, n, replace=False)
    d = np.zeros((H, W), np.uint8)
    d[2 * (cells // wg), 2 * (cells % wg)] = rng.integers(1, 256, n)
    return d


@pytest.mark.parametrize("ns,k,seed_base", [
    ((3000, 4117, 4118, 4500), 600, 7),      # pool branch (n <= 4117), set branch with many repeats
    ((599, 600, 601, 20000), 600, 2**32 + 3),   # n < k (no trial), n == k, two-word seeds
    ((20, 21, 22, 300), 5, 11),             # k <= 5: setsize 21
    ((50, 3, 4, 9), 1, 2**40),              # k = 1 (n = 3: collinear redraws of repeated points)
    ((70000, 66000), 600, 21),              # n > 65535: 32-bit sample indices; points past the LDS (from memory)
    ((70000, 1000), 598, 5),                # 32-bit indices with k x 4 B not a multiple of 16 (element loads)
])
def test_batch_sample_branches(svb, ns, k, seed_base):
    trials = 25
    with svb.Batch(len(ns), H=H, W=W, step=2, with_bgr=False) as b:
        for f, n in enumerate(ns):
            b.upload(f, _sparse_frame(n, 100 + n + f))
        b.set_mask(None)
        b.ransac(seed_base=seed_base, trials=trials, k=k)
        for f, n in enumerate(ns):
            pts = b.read_maskpoints(f)
            assert len(pts) == n
            ref = _oracle_frame(pts, trials, seed_base + f, k=k)
            _check(b.read_ransac(f), *ref, what=f"n={n} k={k}")


@pytest.mark.parametrize("ns,k,seed_base", [
    ((3000, 4117, 4118, 20000), 600, 9),     # pool branch (virtual pool), set branch
    ((599, 600, 601, 4500), 600, 2**33 + 1),
    ((20, 21, 22, 300), 5, 13),
])
def test_batch_sample_branches_mask_bound(svb, ns, k, seed_base):
    """With a mask set, the launches are sized from the mask's step-2 points (an upper bound of every frame's
    count) instead of the counts read back; both random.sample branches must still replay CPython exactly. The
    mask keeps grid rows < 120 (61,440 step-2 points: 1,920 bitmap words, 16-bit sample indices) and every
    point of these frames lies there."""
    trials = 25
    mask = np.zeros((H, W), np.uint8)
    mask[:240, :] = 255
    with svb.Batch(len(ns), H=H, W=W, step=2, with_bgr=False) as b:
        for f, n in enumerate(ns):
            d = _sparse_frame(n, 300 + n + f)
            hit = d[240:] != 0
            if hit.any():   # move the points below the masked rows up into them (same count, distinct cells)
                rng = np.random.default_rng(n + f)
                free = np.flatnonzero(d[0:240:2, 0:1023:2] == 0)
                cells = rng.choice(free, int(hit.sum()), replace=False)
                vals = d[240:][hit]
                d[240:] = 0
                d[2 * (cells // 512), 2 * (cells % 512)] = vals
            assert (d[0:543:2, 0:1023:2] != 0).sum() == n
            b.upload(f, d)
        b.set_mask(mask)
        b.ransac(seed_base=seed_base, trials=trials, k=k)
        for f, n in enumerate(ns):
            pts = b.read_maskpoints(f)
            assert len(pts) == n
            ref = _oracle_frame(pts, trials, seed_base + f, k=k)
            _check(b.read_ransac(f), *ref, what=f"mask bound n={n} k={k}")


def _lines_frame(rows, n_per_row, n_rest, seed):
    """n_rest random step-2 points plus n_per_row points on each given grid row at one disparity (50): every
    triple drawn from one row is collinear (same Y and Z)."""
    rng = np.random.default_rng(seed)
    d = _sparse_frame(n_rest, seed + 1)
    for r in rows:
        d[r, :] = 0
        d[r, 2 * rng.choice(W // 2, n_per_row, replace=False)] = 50
    return d


def test_batch_collinear_redraws(svb):
    """Frames whose points lie largely on a few lines: many triples are collinear, so
    randomNonCollinearPoints redraws often (set branch with nine full rows, pool branch with one and two
    rows). The draw kernel checks each triple on a second wave while the next sample is drawn and rewinds
    the stream when it was collinear; every trial's sample and triple, the winner and the plane must still
    be CPython's and the reference's."""
    trials = 300
    frames = [_lines_frame(range(100, 118, 2), 512, 400, 70), _lines_frame([100], 500, 500, 71),
              _lines_frame([100, 300], 300, 150, 72)]
    with svb.Batch(len(frames), H=H, W=W, step=2, with_bgr=False) as b:
        for f, d in enumerate(frames):
            b.upload(f, d)
        b.set_mask(None)
        b.ransac_trace(trials)
        b.ransac(seed_base=33, trials=trials)
        redraws = 0
        for f in range(len(frames)):
            pts = b.read_maskpoints(f)
            _check_draws(b, f, pts, 33 + f, trials)
            _check(b.read_ransac(f), *_oracle_frame(pts, trials, 33 + f), what=f"frame {f}")
            r = random.Random(33 + f)
            P = np.asarray(pts)
            for _ in range(trials):   # how many redraws the frame exercised
                r.sample(range(len(P)), 600)
                while True:
                    i1, i2, i3 = (r.sample(range(len(P)), 1)[0] for _ in range(3))
                    if np.cross(P[i1] - P[i2], P[i2] - P[i3]).any():
                        break
                    redraws += 1
        assert redraws >= 20, redraws


def test_batch_degenerate_frame_gives_up(svb):
    """All maskpoints on one line: the reference loops for ever in
    randomNonCollinearPoints; the kernel stops, flags the frame (8) and the
    other frames of the batch are unaffected."""
    line = np.zeros((H, W), np.uint8)
    line[100, 0:1000:2] = 50                 # one grid row, one disparity: collinear
    good = _sparse_frame(5000, 3)
    with svb.Batch(2, H=H, W=W, step=2, with_bgr=False) as b:
        b.upload(0, line)
        b.upload(1, good)
        b.set_mask(None)
        b.ransac(seed_base=0, trials=3, k=100)
        r0 = b.read_ransac(0)
        assert r0["trial"] == -1 and r0["flags"] & 8
        ref = _oracle_frame(b.read_maskpoints(1), 3, 1, k=100)
        _check(b.read_ransac(1), *ref, what="good frame")


@pytest.mark.parametrize("mode", ["tiled", "resident"])
@pytest.mark.parametrize("step", [2, 1])
def test_pipeline_with_frame_planes(svb, mode, step):
    """stereovision.py:84-113 per frame on the device: RANSAC's plane of each
    frame drives that frame's threshold / histogram / compaction. Each frame's
    output equals the oracle chain run with the ORACLE's plane for that frame
    (oracle/ransac.py on the oracle's maskpoints with random.Random(seed_base +
    F): the reference's np.dot(np.linalg.inv(P), ones) of the same draws); a
    frame with no plane keeps nothing (the reference's plane step raises). Both
    kernel families (the frame-resident one reads each frame's plane from
    memory). tests/test_gpu_digests.py checks the same at 4096 frames."""
    m = carmask()
    frames = 4
    sparse = _sparse_frame(300, 9)   # 300 points: fewer than 600 -> no plane
    with svb.Batch(frames, H=H, W=W, step=step, with_bgr=True, with_points=True) as b:
        b.pipeline_mode(mode)
        b.synth(30)
        _, bgr3 = oracle.synth_frame(33)
        b.upload(3, sparse, bgr3)
        b.set_mask(m)
        b.ransac(seed_base=5, trials=60)
        b.pipeline_planes()
        counts = b.read_counts()
        for f in range(frames):
            res = b.read_ransac(f)
            fp = b.read_frame_plane(f)
            disp, bgr = (sparse, bgr3) if f == 3 else oracle.synth_frame(30 + f)
            if f == 3:
                assert res["trial"] == -1 and fp[3] == -1.0
                assert tuple(counts[f][1:3]) == (0, 0)
                continue
            a, bb, c = res["abc"]
            assert np.array_equal(fp[:3], res["abc"])
            assert fp[3] == np.sqrt(a * a + bb * bb + c * c)       # device sqrt == the reference's math.sqrt
            mpts = oracle.project(oracle.mask_disparity(disp, m), None, 2)[0]
            abc_ref, recs = oransac.ransac(mpts, 60, rng=random.Random(5 + f))
            win = next(i for i, r in enumerate(recs) if r.get("err") is not None and r["err"] == min(
                x["err"] for x in recs if x.get("err") is not None and not np.isnan(x["err"])))
            assert res["trial"] == win, f
            assert np.array_equal(_bits(res["abc"]), _bits(abc_ref.reshape(3))), f
            ref = oracle.pipeline_frame(disp, bgr, step, abc=abc_ref.reshape(3))
            xyz, pts = b.read_points(f)
            assert tuple(int(v) for v in counts[f][:3]) == ref["counts"], f
            assert np.array_equal(b.read_hist(f)[:1000], ref["hist"][:1000]), f
            assert np.array_equal(pts, ref["pts"]), f
            np.testing.assert_allclose(xyz, ref["xyz2"], rtol=1e-5, atol=0)


def test_batch_shard_invariance(svb):
    """Frames sharded across ranks (contiguous global ids, seeds by global id, as
    svx.dist.shard lays them out) give each frame the result of the whole batch."""
    m = carmask()
    full = []
    with svb.Batch(6, H=H, W=W, step=2, with_bgr=False) as b:
        b.synth(40)
        b.set_mask(m)
        b.ransac(seed_base=77, trials=30, first_frame=40)
        full = [b.read_ransac(f) for f in range(6)]
    for first, count in ((40, 2), (42, 4)):
        with svb.Batch(count, H=H, W=W, step=2, with_bgr=False) as b:
            b.synth(first)
            b.set_mask(m)
            b.ransac(seed_base=77, trials=30, first_frame=first)
            for f in range(count):
                r, ref = b.read_ransac(f), full[first - 40 + f]
                assert r["trial"] == ref["trial"] and r["flags"] == ref["flags"]
                assert r["err"] == ref["err"] and np.array_equal(r["abc"], ref["abc"])
