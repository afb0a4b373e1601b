"""RCCL plumbing on the GPU box (world size 1: the box has one GPU; the N>1
path is exercised by the driver's 8-GPU scaling run and by the gloo tests)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_world1_broadcast_and_allreduce():
    from svx import dist
    ctrl = dist.Control(rank=0, world=1)
    comm = dist.RcclComm(ctrl, device=0)
    try:
        plane = (0.0, 2.8699791779470996, 0.444875113548583)
        assert comm.broadcast_plane(plane, root=0) == plane       # bit-exact round trip
        assert list(comm.allreduce_i64(np.array([1, -2, 3 << 40]))) == [1, -2, 3 << 40]
    finally:
        comm.close()


def test_sharded_batches_equal_one_batch():
    """Frames are pure functions of their global id: two 'ranks' (shards) give
    exactly the per-frame results of one unsharded batch."""
    from svx import batch as sb
    from svx import dist
    total = 6
    with sb.Batch(total, step=2, with_bgr=True, with_points=True) as full:
        full.synth(100)
        full.pipeline(chunk=4)
        ref_counts = full.read_counts()
        ref_pts = [full.read_points(i)[1] for i in range(total)]
    for rank in range(2):
        first, count = dist.shard(total, 2, rank)
        with sb.Batch(count, step=2, with_bgr=True, with_points=True) as b:
            b.synth(100 + first)
            b.pipeline(chunk=2)
            c = b.read_counts()
            for j in range(count):
                assert tuple(c[j]) == tuple(ref_counts[first + j])
                assert np.array_equal(b.read_points(j)[1], ref_pts[first + j])


@pytest.mark.parametrize("mode", ["resident", "tiled"])
def test_device_plane_broadcast_drives_the_pipeline(mode):
    """The plane broadcast into device memory (RCCL, world 1) and read there by
    the pipeline gives exactly the host-plane pipeline's outputs; so does the
    one-process driver (ncclCommInitAll + grouped broadcast, sv_multi_pipeline)."""
    from svx import batch as sb
    from svx import dist
    plane = sb.synthetic_plane()
    frames = 6
    with sb.Batch(frames, step=1, with_bgr=True, with_points=True) as ref:
        ref.pipeline_mode(mode)
        ref.synth(300)
        ref.pipeline(plane=plane)
        want = ref.digest("pipeline")
    ctrl = dist.Control(rank=0, world=1)
    comm = dist.RcclComm(ctrl, device=0)
    mcomm = dist.MultiComm([0])
    try:
        with sb.Batch(frames, step=1, with_bgr=True, with_points=True) as b:
            b.pipeline_mode(mode)
            b.synth(300)
            for _ in range(2):   # the second call reuses the broadcast buffer
                dp = comm.broadcast_plane_dev(b, plane, root=0)
                assert dp
                b.pipeline_dev(dp, sync=True)
                assert np.array_equal(b.digest("pipeline"), want)
            b.pipeline(plane=(0.0, 1.0, 0.0))          # something else in between
            mcomm.pipeline([b], plane, root=0, sync=True)
            assert np.array_equal(b.digest("pipeline"), want)
    finally:
        mcomm.close()
        comm.close()
