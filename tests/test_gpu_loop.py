"""The software-pipelined frame loop (svx.loop.FrameLoop / sv_loop_*, stereovision.py:53-136 over a sequence of
device batches) against the oracle chain: every frame of every batch in flight equals
tests/golden/plane_digests.npz (make_plane_digests.py: the oracle's fillDisparity chain over the global frame
sequence -> maskpoints -> RANSAC with random.seed(g) -> the pipeline with that plane): the winning trial, its
error and plane bit for bit, and the six pipeline digests. The pre-pass carry between batches is what makes a
sequence of batches equal one long batch; these tests cross 1, 7 and 3 batch boundaries."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FIELDS = ("n_valid", "n_kept", "n_kept2", "disp_hash", "hist_hash", "pts_hash")


@pytest.fixture(scope="module")
def gold():
    import svx
    assert svx.device_count() >= 1
    z = np.load(os.path.join(GOLDEN, "plane_digests.npz"))
    assert int(z["seed_base"]) == 0 and int(z["trials"]) == 600
    return z["planes"]


@pytest.fixture(scope="module")
def mask():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_prepass_cpu import carmask
    return carmask()


def check_batch(b, first, want):
    """mismatching frames of batch b (global ids first..) against the golden rows `want`"""
    n = b.frames
    got = b.digest("pipeline")
    bad = [int(f) for f in np.flatnonzero(got[:, 6] != 0)]
    for k, name in enumerate(FIELDS):
        bad += [int(f) for f in np.flatnonzero(got[:, k] != want[name].astype(np.uint64))]
    for f in range(n):
        r = b.read_ransac(f)
        if not (r["trial"] == want["trial"][f] and r["err"] == want["err"][f] and
                np.array_equal(np.asarray(r["abc"]).view(np.uint64), want["abc"][f].view(np.uint64))):
            bad.append(f)
    return sorted(set(first + f for f in bad))


@pytest.mark.parametrize("slots", [2, 1])
def test_two_batches_in_flight_every_frame(gold, mask, slots):
    """frames 0..4095 as two batches of 2048; with slots = 2 both are in flight at once (the second's RANSAC
    beside the first's pipeline and road), and both are still held when they are checked."""
    from svx.loop import FrameLoop
    with FrameLoop(2048, slots=slots, carmask=mask) as loop:
        seqs = [loop.submit(0), loop.submit(2048)]
        held = seqs if slots == 2 else seqs[1:]
        if slots == 1:   # one slot: the first batch's results are gone once the second is submitted
            with pytest.raises(Exception):
                loop.batch(seqs[0])
        import oracle
        for seq in held:
            loop.wait(seq)
            b, first = loop.batch(seq)
            assert check_batch(b, first, gold[first:first + 2048]) == [], (slots, seq)
            for f in (0, 1, 1000, 2047):   # the road pass (from the pipeline's bitmap) against the pinned points
                _, pts = b.read_points(f)
                rimg = oracle.road_raster(pts)
                img, walk = b.read_road(f, walk=True)
                assert np.array_equal(img, rimg) and np.array_equal(walk, oracle.nonzero_points(rimg)), (seq, f)
        tl = loop.timeline(seqs[-1])
        prev_end = 0.0
        for name in ("input", "prepass", "maskpoints", "draw", "eval", "pipeline", "road"):
            a, z = tl[name]
            assert prev_end - 1e-3 <= a <= z, (name, tl)
            prev_end = z


def test_eight_batches_every_frame(gold, mask):
    """8192 frames as eight batches of 1024 through two slots (seven carries); each batch is checked after the
    next one is submitted, while both are in flight."""
    from svx.loop import FrameLoop
    if len(gold) < 8192:
        pytest.skip("plane_digests.npz holds fewer than 8192 frames")
    frames = 1024
    with FrameLoop(frames, slots=2, carmask=mask) as loop:
        prev = None
        for i in range(8):
            seq = loop.submit(i * frames)
            if prev is not None:
                loop.wait(prev)
                b, first = loop.batch(prev)
                assert check_batch(b, first, gold[first:first + frames]) == [], prev
            prev = seq
        loop.wait(prev)
        b, first = loop.batch(prev)
        assert check_batch(b, first, gold[first:first + frames]) == [], prev


@pytest.mark.parametrize("H,W,step", [(544, 1024, 1), (544, 1024, 2), (390, 889, 1)])
def test_caller_filled_batches_equal_one_batch(mask, H, W, step):
    """source="caller": frames uploaded into the acquired slot (svx.loop.FrameLoop.acquire). Three batches of 4
    frames give, frame for frame, what one 12-frame batch gives with the same pre-pass, RANSAC and pipeline
    (the carry is the previous batch's last cleaned frame), and the imageRoadMap / road walk are produced; at
    the reference's step 2 and on the cropped 390 x 889 frames too (the tiled pipeline and the road from the
    points)."""
    import oracle
    from svx import batch
    from svx.loop import FrameLoop
    ids = list(range(300, 312))
    frames = [tuple(np.ascontiguousarray(a[:H, :W]) for a in oracle.synth_frame(g)) for g in ids]
    mask = np.ascontiguousarray(mask[:H, :W])
    with batch.Batch(12, H=H, W=W, step=step, with_bgr=True, with_points=True) as one:
        for f, (d, c) in enumerate(frames):
            one.upload(f, d, c)
        one.set_mask(mask)
        one.prepass("previous")
        one.ransac(seed_base=7, trials=600, first_frame=ids[0])
        one.pipeline_planes()
        one.road_map()
        one.road_raster()
        want = one.digest("pipeline")
        want_r = [one.read_ransac(f) for f in range(12)]
        want_road = [one.read_road(f, walk=True) for f in range(12)]
        want_map = [one.read_road_map(f) for f in (0, 11)]
    with FrameLoop(4, H=H, W=W, step=step, slots=2, source="caller", seed_base=7, road="map", carmask=mask) as loop:
        for i in range(3):
            b = loop.acquire()
            for f in range(4):
                b.upload(f, *frames[4 * i + f])
            seq = loop.submit(ids[4 * i])
            if i >= 1:
                pb, first = loop.batch(seq - 1)
                loop.wait(seq - 1)
                base = first - ids[0]
                assert np.array_equal(pb.digest("pipeline"), want[base:base + 4])
                for f in range(4):
                    r = pb.read_ransac(f)
                    assert r["trial"] == want_r[base + f]["trial"] and r["err"] == want_r[base + f]["err"]
                    img, walk = pb.read_road(f, walk=True)
                    assert np.array_equal(img, want_road[base + f][0]) and np.array_equal(walk, want_road[base + f][1])
        loop.wait(seq)
        b, first = loop.batch(seq)
        assert np.array_equal(b.digest("pipeline"), want[8:12])
        assert np.array_equal(b.read_road_map(3), want_map[1])


@pytest.mark.parametrize("prepass", ["mean", "none"])
def test_caller_slot_keeps_its_raw_frames(mask, prepass):
    """A caller-fed slot keeps the frames the caller wrote: the pre-pass reads them there and writes the cleaned
    frames elsewhere, so submitting the slot again without refilling it processes the same raw frames (with a
    per-frame pre-pass, fillAltDisparity or none, the results are identical), and the raw frames are never
    overwritten by a clean. The first submit must also equal a plain batch given the same uploads (with
    prepass="none" the stages read frames the loop copied from the raw buffer, not a buffer never written)."""
    import oracle
    from svx import batch
    from svx.loop import FrameLoop
    frames = [oracle.synth_frame(g) for g in range(40, 44)]
    with batch.Batch(4, with_bgr=True, with_points=True) as one:
        for f, (d, c) in enumerate(frames):
            one.upload(f, d, c)
        one.set_mask(mask)
        if prepass != "none":
            one.prepass(prepass)
        one.ransac(seed_base=3, trials=600, first_frame=40)
        one.pipeline_planes()
        ref = one.digest("pipeline")
        ref_r = [one.read_ransac(f)["trial"] for f in range(4)]
    assert np.all(ref[:, 2] > 0)   # the frames keep points: a batch of zeros would not
    with FrameLoop(4, slots=1, source="caller", prepass=prepass, seed_base=3, carmask=mask) as loop:
        b = loop.acquire()
        for f, (d, c) in enumerate(frames):
            b.upload(f, d, c)
        s0 = loop.submit(40)
        loop.wait(s0)
        b0, _ = loop.batch(s0)
        want = b0.digest("pipeline")
        want_r = [b0.read_ransac(f)["trial"] for f in range(4)]
        assert np.array_equal(want, ref) and want_r == ref_r
        for rep in range(2):
            loop.acquire()   # not refilled
            s1 = loop.submit(40)
            b1, _ = loop.batch(s1)
            assert np.array_equal(b1.digest("pipeline"), want), rep
            assert [b1.read_ransac(f)["trial"] for f in range(4)] == want_r, rep


def test_step2_resident_batches_equal_one_batch(mask):
    """Two 1024-frame batches at the reference's step 2 (the resident pipeline, road from its points: the
    bitmap is step-1 only) equal one 2048-frame batch frame for frame: RANSAC, pipeline digests, road."""
    from svx import batch
    from svx.loop import FrameLoop
    n = 1024
    with batch.Batch(2 * n, step=2, with_bgr=True, with_points=True) as one:
        one.synth(0)
        one.set_mask(mask)
        one.prepass("previous")
        one.ransac(seed_base=0, trials=600)
        one.pipeline_planes()
        one.road_raster()
        want = one.digest("pipeline")
        probe = (0, 1, n - 1, n, n + 1, 2 * n - 1)
        want_r = {f: one.read_ransac(f) for f in probe}
        want_road = {f: one.read_road(f, walk=True) for f in probe}
    with FrameLoop(n, step=2, slots=2, carmask=mask) as loop:
        seqs = [loop.submit(0), loop.submit(n)]
        for seq in seqs:
            loop.wait(seq)
            b, first = loop.batch(seq)
            assert np.array_equal(b.digest("pipeline"), want[first:first + n]), seq
            for f in probe:
                if first <= f < first + n:
                    r = b.read_ransac(f - first)
                    assert r["trial"] == want_r[f]["trial"] and r["err"] == want_r[f]["err"], f
                    img, walk = b.read_road(f - first, walk=True)
                    assert np.array_equal(img, want_road[f][0]) and np.array_equal(walk, want_road[f][1]), f
