"""bench.py's N-GPU drivers on the one-GPU box (the driver's 8-GPU run must not
be their first execution): the in-process bench in "multi" mode (one process,
ncclCommInitAll over devices [0], the grouped plane broadcast of
sv_multi_pipeline inside the timed steps) and in "ranks" mode (torchrun's
RANK / WORLD_SIZE / LOCAL_RANK at world size 1: the TCP control plane, an RCCL
communicator per rank, sv_comm_broadcast_plane_dev + sv_batch_pipeline_dev).
Small settings; every frame's K1 and pipeline digests are checked by the bench
itself against tests/golden/frame_digests.npz (parity.pass)."""
import pytest

pytestmark = pytest.mark.gpu

ARGS = ["--gpus", "1", "--frames", "512", "--steps", "2", "--warmup", "1", "--ramp-ms", "20",
        "--no-extras", "--no-cpu", "--no-latency"]


def _check(out):
    assert out["n_gpus"] == 1
    assert out["parity"]["pass"], out["parity"]
    assert out["parity"]["k1"]["frames_checked"] == 512
    assert out["parity"]["pipeline"]["frames_checked"] == 512
    assert out["value"] > 0 and out["pipeline"]["value"] > 0


def test_bench_multi_driver(monkeypatch):
    import bench
    from svx import dist
    calls = []
    orig = dist.MultiComm.pipeline

    def counting(self, *a, **k):
        calls.append(len(a[0]))
        return orig(self, *a, **k)

    monkeypatch.setattr(dist.MultiComm, "pipeline", counting)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    out = bench.main(ARGS + ["--driver", "multi"])
    _check(out)
    assert "ncclCommInitAll" in out["config"]["parallelism"]
    assert out["pipeline"]["plane_broadcast"].startswith("RCCL grouped")
    assert len(calls) >= 3 and set(calls) == {1}   # warm-up + 2 timed steps, one batch each


def test_bench_ranks_driver(monkeypatch):
    import bench
    from svx import dist
    calls = []
    orig = dist.RcclComm.broadcast_plane_dev

    def counting(self, *a, **k):
        calls.append(1)
        return orig(self, *a, **k)

    monkeypatch.setattr(dist.RcclComm, "broadcast_plane_dev", counting)
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29531")
    out = bench.main(ARGS)
    _check(out)
    assert "torchrun" in out["config"]["parallelism"]
    assert out["pipeline"]["plane_broadcast"].startswith("RCCL ncclBroadcast")
    assert len(calls) >= 3


def test_bench_strong_scaling_flag(monkeypatch):
    """--global-frames (SURVEY §8d config 5's strong scaling): the given frames in all, split over the GPUs;
    at one GPU the whole batch, reported as strong scaling, with every frame's digests checked."""
    import bench
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    out = bench.main([a for a in ARGS if a not in ("--frames", "512")] + ["--global-frames", "512"])
    _check(out)
    assert out["scaling"] == "strong" and out["config"]["global_frames"] == 512


def test_bench_ranks_without_rccl(monkeypatch):
    """"ranks" mode when the RCCL communicator cannot be made (every rank fails alike, a collective init): the
    bench still measures, with rank 0's plane over the host control plane, and says so in its line."""
    import bench
    from svx import SvxError, dist

    def fail(self, *a, **k):
        raise SvxError("simulated ncclCommInitRank failure")

    monkeypatch.setattr(dist.RcclComm, "__init__", fail)
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29532")
    out = bench.main(ARGS)
    _check(out)
    assert out["pipeline"]["plane_broadcast"].startswith("RCCL communicator unavailable")
