"""bench.py's launch logic on the CPU: how `--gpus N` maps onto processes and
devices (torchrun ranks vs one process driving N GPUs), that a launcher whose
WORLD_SIZE disagrees with --gpus is refused, that the shards of every
topology cover the global frame ids exactly once, and the TCP control plane
at three ranks."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

from conftest import PKG, REPO

import bench


def test_plan_single_and_multi_process():
    p = bench.plan(1, {})
    assert p["mode"] == "single" and p["n_gpus"] == 1 and p["devices"] == [0]
    p = bench.plan(2, {})
    assert p["mode"] == "multi" and p["n_gpus"] == 2 and p["devices"] == [0, 1] and p["world"] == 1
    p = bench.plan(8, {})
    assert p["devices"] == list(range(8)) and p["n_gpus"] == 8


def test_plan_torchrun_ranks():
    for rank in range(2):
        env = {"WORLD_SIZE": "2", "RANK": str(rank), "LOCAL_RANK": str(rank)}
        p = bench.plan(2, env)
        assert p["mode"] == "ranks" and p["n_gpus"] == 2 and p["world"] == 2
        assert p["devices"] == [rank] and p["shard_base"] == rank
    p = bench.plan(1, {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p["mode"] == "ranks" and p["n_gpus"] == 1


@pytest.mark.parametrize("gpus,world", [(8, 1), (1, 8), (2, 4)])
def test_plan_refuses_mismatched_launcher(gpus, world):
    with pytest.raises(SystemExit) as e:
        bench.plan(gpus, {"WORLD_SIZE": str(world), "RANK": "0", "LOCAL_RANK": "0"})
    assert "WORLD_SIZE" in str(e.value)
    with pytest.raises(SystemExit):
        bench.plan(0, {})


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_shards_cover_global_frames(n):
    frames = 4096
    multi = bench.shards_of(bench.plan(n, {}), frames)
    ranks = [s for r in range(n)
             for s in bench.shards_of(bench.plan(n, {"WORLD_SIZE": str(n), "RANK": str(r), "LOCAL_RANK": str(r)}),
                                      frames)]
    for shards in (multi, ranks):
        assert [d for d, _, _ in shards] == list(range(n))
        ids = np.concatenate([np.arange(f, f + c) for _, f, c in shards])
        assert np.array_equal(ids, np.arange(frames * n))   # every global id once, in order
        assert all(c == frames for _, _, c in shards)       # weak scaling: 4096 per GPU
    assert multi == ranks


def _tcp_worker(rank, world, path, q):
    for p in (REPO, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from svx.control import TcpControl
    c = TcpControl(rank, world, path=path, timeout=60)
    try:
        got = c.broadcast_bytes(bytes([7] * 128) if rank == 0 else b"")
        mx = c.max([rank, -rank, 0.5])
        sm = c.sum([rank, 1.0])
        c.barrier()
        q.put((rank, got, list(mx), list(sm)))
    finally:
        c.close()


@pytest.mark.timeout(120)
def test_tcp_control_three_ranks(tmp_path):
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "rdzv")
    procs = [ctx.Process(target=_tcp_worker, args=(r, world, path, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for rank, got, mx, sm in res:
        assert got == bytes([7] * 128)
        assert mx == [2.0, 0.0, 0.5] and sm == [3.0, 3.0]
    assert not os.path.exists(path)   # rank 0 removes the rendezvous file once everyone is in


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_strong_scaling_shards(n):
    """--global-frames 32768 (SURVEY §8d config 5, strong scaling): the same 32768 global frame ids split over
    n GPUs in contiguous ranges, by the one-process driver and by n ranks alike."""
    total = 32768
    multi = bench.shards_of(bench.plan(n, {}), 4096, total)
    ranks = [s for r in range(n)
             for s in bench.shards_of(bench.plan(n, {"WORLD_SIZE": str(n), "RANK": str(r), "LOCAL_RANK": str(r)}),
                                      4096, total)]
    assert multi == ranks
    ids = np.concatenate([np.arange(f, f + c) for _, f, c in multi])
    assert np.array_equal(ids, np.arange(total)) and all(c == total // n for _, _, c in multi)
    assert bench.parse(["--global-frames", str(total)]).global_frames == total
    with pytest.raises(SystemExit):
        bench.shards_of(bench.plan(8, {}), 4096, 4)


def _traffic_file(tmp_path, **kw):
    import json
    tj = {"frames": 4096, "step": 1, "pipeline_kernels": {
        "svx::frame_planes_kernel": {"launches": 1, "fetch_bytes_total": 1.0, "write_bytes_total": 2.0},
        "svx::resident_fused_kernel<1, 4, true, true, true, false>": {
            "launches": 1, "fetch_bytes_total": 9e9, "write_bytes_total": 18e9}},
        "pipeline_hbm_bytes_per_call": 27e9, "source_ids": {"pipeline": bench.kernel_source_id("pipeline")}}
    tj.update(kw)
    p = tmp_path / "traffic.json"
    p.write_text(json.dumps(tj))
    return str(p)


def test_profile_traffic_only_for_the_timed_kernel(tmp_path):
    """bench.py reports PMC traffic only for a profile of the same kernel instance built from the same sources
    (a stale profile of another instance or of older sources gives null and the reason)."""
    name = "svx::resident_fused_kernel<1, 4, true, true, true, false>"
    p = _traffic_file(tmp_path)
    assert bench.profile_traffic(p, 4096, 1, name, "pipeline") == (27e9, None)
    # another instance (round 3's five-parameter kernel): null, with the reason
    v, why = bench.profile_traffic(p, 4096, 1, "svx::resident_fused_kernel<1, 4, true, true, true>", "pipeline")
    assert v is None and "timed kernel" in why
    # the same name from other sources
    v, why = bench.profile_traffic(_traffic_file(tmp_path, source_ids={"pipeline": "0" * 16}), 4096, 1, name,
                                   "pipeline")
    assert v is None and "sources" in why
    # another workload, a missing file
    v, why = bench.profile_traffic(p, 2048, 1, name, "pipeline")
    assert v is None and "2048" in why
    v, why = bench.profile_traffic(str(tmp_path / "none.json"), 4096, 1, name, "pipeline")
    assert v is None and why


def test_committed_profiles_name_their_kernel():
    """Every committed traffic profile bench.py reads names its kernel instance and the sources it measured."""
    import json
    for f, key in (("traffic.json", "k1_kernel"), ("traffic_pipeline.json", "pipeline_kernels"),
                   ("traffic_planes.json", "pipeline_kernels")):
        tj = json.load(open(os.path.join(REPO, "profiles", f)))
        assert tj.get(key), f
        assert tj.get("source_ids"), f


def _record(extra_bytes=0):
    """A line with every record bench.py emits at N = 1 (numbers and short keys only), optionally bloated."""
    stage = {k: 1.234 for k in ("input", "prepass", "maskpoints", "draw", "eval", "pipeline", "road")}
    pl = {"tried_ms": [4.2345, 4.3456, 4.4567], "kept": 1}
    loop = {"ms_per_batch": 14.38, "frames": 4096, "frames_per_s": 284840.1, "slots": 2, "batches_timed": 4,
            "stage_ms": stage, "draw_overlap_ms": 5.123}
    out = {"metric": bench.METRIC, "value": 534406.4, "unit": "Mpoints/s", "n_gpus": 1, "steps": 20, "warmup": 3,
           "ms_per_step": 4.2576, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8->f32",
           "data": "synthetic", "config": {"workload": "configs[2]", "frames_per_gpu": 4096, "parallelism": "x1"},
           "roofline": {"bound": "hbm", "achieved": 6972.5, "peak": 8000.0, "unit": "GB/s", "frac": 0.8716,
                        "traffic": 29607724672.0, "kernel": "svx::project_dense_kernel<1, true, 1, 0>",
                        "kernel_ms": 4.2422, "placement": dict(pl, junk="x" * extra_bytes)},
           "cpu_baseline": {"value": 1.52, "unit": "Mpoints/s", "cores": 1, "kind": "port", "sample": "configs[0]"},
           "latency_1frame_us": 6.8,
           "pipeline": {"gpu_ms_per_call": 5.256, "frac": 0.649, "value": 432900.1, "placement": pl,
                        "kernel": "svx::resident_fused_kernel<1, 4, true, true, true, false>", "traffic": 2.7e10},
           "parity": {"k1": {"frames_checked": 4096, "mismatched_frames": 0}, "pass": True},
           "extras": {"device_frame_loop": loop, "device_frame_loop_serial": dict(loop),
                      "device_frame_loop_with_input": dict(loop),
                      "sgbm_disparity": {"us_per_frame": 236.4, "placement": dict(pl, junk="y" * extra_bytes)}}}
    return out


def test_json_line_within_limit():
    """The driver keeps the last 8 KB of the run's output: the line is at most LINE_LIMIT bytes, the contract fields
    come first, and an over-long line loses placements and stage breakdowns before any contract or headline
    field (the pipeline's own figures had fallen out of the driver's record)."""
    import json
    for extra in (0, 3000, 9000):
        o = bench.finalize(_record(extra))
        line = json.dumps(o, separators=(",", ":"))
        assert len(line.encode()) <= bench.LINE_LIMIT, (extra, len(line))
        assert line.startswith('{"metric":')
        for k in ("value", "unit", "ms_per_step", "roofline", "cpu_baseline", "pipeline", "parity",
                  "latency_1frame_us"):
            assert k in o, (extra, k)
        assert o["pipeline"]["gpu_ms_per_call"] == 5.256 and o["pipeline"]["frac"] == 0.649
        assert o["extras"]["device_frame_loop"]["ms_per_batch"] == 14.38
    # the unbloated line needs no drop at all
    assert bench.finalize(_record(0)) == bench.finalize(_record(0), limit=10 ** 9)
