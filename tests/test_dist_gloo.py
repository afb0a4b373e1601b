"""Multi-process (world_size 2, CPU) tests of the sharded driver's host
logic over both control planes — svx.control's TCP star (the default, no
PyTorch) and a torch.distributed gloo group (SVX_CONTROL=gloo): frame
sharding, max-over-ranks timing, the RCCL unique-id hand-off path (bytes
broadcast), bench.py's whole-job aggregation and the per-frame independence
the sharding relies on (checked with the oracle standing in for the device)."""
import os
import socket
import sys

import numpy as np
import pytest
import multiprocessing as mp

from conftest import PKG, REPO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_partitions_exactly():
    from svx.dist import shard
    for total in (1, 7, 4096, 32768, 32769):
        for world in (1, 2, 3, 8):
            spans = [shard(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (f0, c0), (f1, _) in zip(spans, spans[1:]):
                assert f0 + c0 == f1
            assert sum(c for _, c in spans) == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _worker(rank, world, port, control, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SVX_CONTROL=control)
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import oracle
    from svx import dist
    ctrl = dist.Control()
    try:
        assert (ctrl.rank, ctrl.world) == (rank, world)
        # unique-id style hand-off: 128 bytes from rank 0
        payload = bytes(range(128)) if rank == 0 else bytes(128)
        got = ctrl.broadcast_bytes(payload, src=0)
        assert got == bytes(range(128))
        mx = ctrl.max([float(rank + 1), -float(rank)])
        sm = ctrl.sum([1.0, float(rank)])
        # weak scaling: 2 frames per rank, global ids; per-frame results are independent
        first, count = dist.shard(2 * world, world, rank)
        counts = []
        for f in range(first, first + count):
            d, c = oracle.synth_frame(f)
            crop = (np.ascontiguousarray(d[180:260]), np.ascontiguousarray(c[180:260]))
            counts.append(oracle.pipeline_frame(*crop, 2, abc=oracle.synthetic_plane())["counts"])
        tot = ctrl.sum(np.array(counts, np.float64).sum(axis=0))
        # bench.py's whole-job figure: all ranks' points over the slowest rank's time
        import bench
        agg = bench.aggregate(ctrl, world, 1000.0 * (rank + 1), 4, 0.5 + rank)
        ctrl.barrier()
        q.put((rank, list(mx), list(sm), first, count, counts, list(tot), agg))
    finally:
        ctrl.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("control", ["tcp", "gloo"])
def test_two_rank_control_plane_and_sharding(control):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, control, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    import oracle
    ref = []
    for f in range(2 * world):
        d, c = oracle.synth_frame(f)
        crop = (np.ascontiguousarray(d[180:260]), np.ascontiguousarray(c[180:260]))
        ref.append(oracle.pipeline_frame(*crop, 2, abc=oracle.synthetic_plane())["counts"])
    for rank, mx, sm, first, count, counts, tot, agg in res:
        assert agg["n_gpus"] == 2 and agg["points"] == 3000.0 * 4
        assert abs(agg["value"] - 3000.0 * 4 / 1.5 / 1e6) < 1e-12 and abs(agg["ms_per_step"] - 1.5 / 4 * 1e3) < 1e-9
        assert mx == [2.0, 0.0] and sm == [2.0, 1.0]
        assert (first, count) == (2 * rank, 2)
        assert [tuple(c) for c in counts] == ref[first:first + count]
        assert tot == list(np.array(ref, np.float64).sum(axis=0))


def _ramp_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SVX_CONTROL="tcp")
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import time

    import bench
    from svx import dist
    ctrl = dist.Control()
    calls = []
    try:
        def step():   # a collective in every call, like bench.py's RCCL broadcast: ranks run at different speeds
            time.sleep(0.002 * (1 + 3 * rank))
            calls.append(ctrl.sum([1.0])[0])
        n = bench.ramp_agreed(step, (), 60.0, ctrl)
        ctrl.barrier()
        q.put((rank, n, len(calls), set(calls)))
    finally:
        ctrl.close()


@pytest.mark.timeout(120)
def test_two_rank_ramp_with_a_collective_agrees_on_the_call_count():
    """bench.py's warm-up of a step holding a collective: both ranks run the same number of calls although one
    is 4x slower (a per-rank wall-clock ramp would not; its extra collective would hang)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ramp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1] == res[0][2] == res[1][2] >= 2   # the larger of the two ranks' counts, ceil(60 ms / one call)
    assert all(r[3] == {2.0} for r in res)


def _rccl_agree_worker(rank, world, port, fail_step, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SVX_CONTROL="tcp")
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from svx import _abi, dist
    calls = []

    def fake_call(name, *args):   # the RCCL steps without a GPU: `fail_step` fails on the last rank only
        calls.append(name)
        if name == fail_step and rank == world - 1:
            raise _abi.SvxError(f"simulated {name} failure")
        if name == "sv_comm_init":
            args[-1]._obj.value = 0x1000   # the communicator handle (byref's target)
        return 0
    _abi.call = fake_call
    ctrl = dist.Control()
    try:
        try:
            dist.RcclComm(ctrl, rank)
            q.put((rank, "ok", calls))
        except _abi.SvxError as e:
            q.put((rank, str(e), calls))
        ctrl.barrier()   # the control plane is still in step after the failure
    finally:
        ctrl.close()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("fail_step", ["sv_init", "sv_comm_init"])
def test_two_rank_rccl_setup_failure_on_one_rank_fails_every_rank(fail_step):
    """svx.dist.RcclComm: a setup step failing on ONE rank raises on every rank (agreed over the control plane)
    instead of leaving the others in the next collective; a communicator made on the other rank is destroyed."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rccl_agree_worker, args=(r, world, port, fail_step, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for rank, msg, calls in res:
        assert "failed on 1 of 2" in msg, (rank, msg)
        if fail_step == "sv_init":
            assert "sv_comm_init" not in calls           # nobody entered the collective init
        elif rank == 0:
            assert calls[-1] == "sv_comm_destroy"        # its communicator is released
