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
