#!/usr/bin/env python3
"""Benchmark: Mpoints/s of disparity->3D at 1024x544 and achieved HBM GB/s vs peak.

Headline workload (BASELINE.json configs[2], the north-star target): a batch of
4096 synthetic 1024x544 disparity maps per GPU, step 1 (555,489 grid points per
frame), resident in HBM, projected by K1 into dense fp32 X/Y/Z planes. One
"step" = one K1 pass over the whole batch. Multi-GPU (configs[4]): 4096 frames
per GPU (weak scaling), frames sharded by global id, no data-path collective.

How N GPUs are driven (`--gpus N`):
  * under torchrun (WORLD_SIZE set; it must equal N): one process per GPU,
    LOCAL_RANK's device, host control over TCP (svx/control.py), RCCL
    communicator per rank;
  * plain `python bench.py --gpus N`, N > 1: ONE process drives devices
    0..N-1: one sv_batch per device, ncclCommInitAll, the plane
    broadcast of all devices in one RCCL group (sv_multi_pipeline).
Either way: barrier + device sync on both sides of the K timed steps, the
max over ranks, `value` = grid points of all GPUs / that time.

Also reported (same JSON line):
  pipeline      configs[3]/[4]: plane threshold + hue histogram + ordered
                compaction + int32 back-projection over the same batch; for
                N > 1 every step starts with the RCCL broadcast of the plane
                into device memory (read there by the pipeline).
  parity        every frame of every shard (K1 and pipeline outputs) checked
                on the device against tests/golden/frame_digests.npz (the
                pinned C oracle's per-frame digests, global frame ids).
  latency_1frame_us  configs[1]: one frame, step 1, K1 kernel time.
  extras        SURVEY §8f components (N = 1): road raster + walk, pre-pass,
                RANSAC (drop-in and batched), the per-frame-plane pipeline,
                the drop-in chain, the SGBM disparity stage on 128 resident
                stereo pairs and the whole device frame loop from the pairs.
  cpu_baseline  configs[0]: the nested-loop CPU port (oracle/cpu_loop.py, the
                numpy-scalar semantics of functions.py:178-323) on one pinned
                host core: stereovision.py:84-113 for frame 0 at step 2, per
                stage; rank 0 at N = 1 only.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "stereo.vision_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = "Mpoints/sec disparity→3D at 1024×544; achieved HBM GB/s vs peak"
PEAK_HBM_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
H, W = 544, 1024
K1_BYTES_PER_POINT = 13        # 1 B disparity read + 12 B fp32 XYZ written
GOLDEN_DIGESTS = os.path.join(REPO, "tests", "golden", "frame_digests.npz")
GOLDEN_PLANES = os.path.join(REPO, "tests", "golden", "plane_digests.npz")
DIGEST_FIELDS = ("n_valid", "n_kept", "n_kept2", "disp_hash", "hist_hash", "pts_hash")
CARMASK = os.path.join(REPO, "tests", "golden", "carmask.npz")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=4096, help="frames per GPU (weak scaling)")
    ap.add_argument("--global-frames", type=int, default=0,
                    help="strong scaling (SURVEY §8d config 5): this many frames in all, split over the GPUs "
                         "(overrides --frames; 0 = weak scaling, --frames per GPU)")
    ap.add_argument("--step", type=int, default=1, help="grid step (reference hard-codes 2)")
    ap.add_argument("--chunk", type=int, default=0, help="pipeline frames per wave (0 = default)")
    ap.add_argument("--qpl", type=int, default=1, help="K1 quads (4 points) per lane: 1, 2, 4")
    ap.add_argument("--nt", type=int, default=1, help="non-temporal K1 stores (1 = measured faster)")
    ap.add_argument("--ramp-ms", type=float, default=300.0,
                    help="untimed launches before the warmup steps of K1 and of the pipeline (a third of it before the "
                         "§8f stage timings), to let clocks settle")
    ap.add_argument("--no-pipeline", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="skip the 1-frame latency probe")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the SURVEY §8f component timings")
    ap.add_argument("--no-parity", action="store_true", help="skip the per-frame digest check")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--driver", choices=("auto", "single", "multi"), default="auto",
                    help="auto: torchrun ranks when WORLD_SIZE is set, else one process (multi for N > 1); "
                         "multi: force the one-process RCCL driver (ncclCommInitAll) even at N = 1 (tests)")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--traffic-pipeline", default=os.path.join(REPO, "profiles", "traffic_pipeline.json"))
    ap.add_argument("--traffic-planes", default=os.path.join(REPO, "profiles", "traffic_planes.json"))
    return ap.parse_args(argv)


def plan(gpus, environ, driver="auto"):
    """How this process takes part in an N-GPU run:
    mode "ranks" (torchrun: one process per GPU), "multi" (one process, N GPUs)
    or "single". Returns dict(mode, n_gpus, rank, world, devices, shard_base):
    this process drives `devices`, which hold global shards shard_base.. of n_gpus.
    driver="multi" takes the one-process RCCL path at any N (N = 1 included)."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    if driver == "multi":
        if "WORLD_SIZE" in environ:
            raise SystemExit("bench.py: --driver multi is one process driving every GPU; do not launch it per rank")
        return dict(mode="multi", n_gpus=gpus, rank=0, world=1, devices=list(range(gpus)), shard_base=0)
    if "WORLD_SIZE" in environ:
        world = int(environ["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: launched with WORLD_SIZE={world} but --gpus {gpus}; "
                             f"use torchrun --nproc-per-node {gpus} (one process per GPU) or run "
                             f"`python bench.py --gpus {gpus}` without a launcher (one process, {gpus} GPUs)")
        rank, local = int(environ.get("RANK", 0)), int(environ.get("LOCAL_RANK", 0))
        return dict(mode="ranks", n_gpus=world, rank=rank, world=world, devices=[local], shard_base=rank)
    if gpus == 1 or driver == "single":
        if gpus != 1:
            raise SystemExit("bench.py: --driver single drives one GPU (--gpus 1)")
        return dict(mode="single", n_gpus=1, rank=0, world=1, devices=[0], shard_base=0)
    return dict(mode="multi", n_gpus=gpus, rank=0, world=1, devices=list(range(gpus)), shard_base=0)


def shards_of(pl, frames_per_gpu, global_frames=0):
    """(device, first global frame id, frames) of each GPU this process drives: frames_per_gpu each (weak
    scaling), or global_frames > 0 in all, split in contiguous ranges (strong scaling)."""
    from svx.dist import shard
    total = global_frames if global_frames > 0 else frames_per_gpu * pl["n_gpus"]
    if total < pl["n_gpus"]:
        raise SystemExit(f"bench.py: {total} frames over {pl['n_gpus']} GPUs")
    return [(dev, *shard(total, pl["n_gpus"], pl["shard_base"] + j)) for j, dev in enumerate(pl["devices"])]


def aggregate(ctrl, n_gpus, points_local, steps, dt_local):
    """Whole-job rate: all GPUs' grid points over the max-over-ranks wall time."""
    dt = float(ctrl.max([dt_local])[0])
    points = float(ctrl.sum([points_local])[0]) * steps
    return {"n_gpus": n_gpus, "value": points / dt / 1e6, "ms_per_step": dt / steps * 1e3, "points": points}


def carmask():
    z = np.load(CARMASK)
    shape = tuple(int(v) for v in z["shape"])
    return np.unpackbits(z["bits"])[: shape[0] * shape[1]].reshape(shape).astype(np.uint8) * 255


def cpu_baseline(budget_s):
    """configs[0]: stereovision.py:84-113 for synthetic frame 0 at step 2 on ONE pinned host core, per stage, through
    the CPU port (oracle/cpu_loop.py + oracle/ransac.py: a nested-loop restatement of functions.py:178-323 and its
    RANSAC, :240-298, with the reference's numpy-scalar fp64 semantics, pinned to the reference-run fixtures in
    tests/golden/) — `value` is the port's projectDisparityTo3d rate — then a bounded step-1 projection sample (the
    headline workload's unit). The reference's own Python never runs on the GPU box."""
    import random
    import warnings

    import oracle
    from oracle import cpu_loop
    from oracle import ransac as oransac
    try:
        cpu = sorted(os.sched_getaffinity(0))[0]
        os.sched_setaffinity(0, {cpu})
    except (AttributeError, OSError):
        cpu = None
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    disp, bgr = oracle.synth_frame(0)
    mdisp = oracle.mask_disparity(disp, carmask())   # maskDisparity (cv2 in the reference; not timed)
    abc_syn = np.asarray(oracle.synthetic_plane(), np.float64).reshape(3, 1)
    ng2 = ((H - 1 + 1) // 2) * ((W - 1 + 1) // 2)   # grid of range(0,H-1,2) x range(0,W-1,2)

    def stage(fn):
        t = time.perf_counter()
        out = fn()
        return out, (time.perf_counter() - t) * 1e3

    def port_run():
        s = {}
        points, s["a1_project_rgb"] = stage(lambda: cpu_loop.project(disp, bgr, 2))      # stereovision.py:84
        mpts, s["a1_project_masked"] = stage(lambda: cpu_loop.project(mdisp, None, 2))   # :85
        random.seed(0)
        (abc, _), s["ransac_600"] = stage(lambda: oransac.ransac(np.asarray(mpts), 600))  # :94
        abc = abc if abc is not None else abc_syn
        dist, s["a2_point_errors"] = stage(lambda: cpu_loop.point_errors(abc, points))     # :97
        kept, s["a3_planar_threshold"] = stage(lambda: cpu_loop.plane_keep(points, dist, 0.05))   # :100
        hist, s["a5_colour_histogram"] = stage(lambda: cpu_loop.colour_hist(kept))        # :103
        kept2, s["a6_histogram_filter"] = stage(lambda: cpu_loop.hist_keep(kept, hist, 10))   # :106
        _, s["a7_a8_backproject_int32"] = stage(                                          # :111-113
            lambda: np.array(cpu_loop.backproject(kept2), np.int32).reshape((-1, 1, 2)))
        return s

    reps, st = 0, {}
    t_all = time.perf_counter()
    state = random.getstate()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", DeprecationWarning)
        while True:
            for k, v in port_run().items():
                st.setdefault(k, []).append(v)
            reps += 1
            if (reps >= 2 and time.perf_counter() - t_all >= budget_s * 0.6) or reps >= 5:
                break
    random.setstate(state)
    med = {k: round(float(np.median(v)), 1) for k, v in st.items()}
    # bounded step-1 projection sample (the reference hard-codes step 2)
    t1, frames1, pts1 = time.perf_counter(), 0, 0
    while frames1 == 0 or time.perf_counter() - t1 < budget_s * 0.4:
        d1, _ = oracle.synth_frame(frames1)
        cpu_loop.project(d1, None, step=1)
        pts1 += (H - 1) * (W - 1)
        frames1 += 1
    s1 = time.perf_counter() - t1
    return {"value": round(ng2 / med["a1_project_rgb"] / 1e3, 4), "unit": "Mpoints/s", "cores": 1, "kind": "port",
            "port": "oracle/cpu_loop.py+oracle/ransac.py",
            "sample": f"configs[0]: frame 0, step 2 ({ng2} pts), stereovision.py:84-113, median of {reps}",
            "config1_stage_ms": med, "config1_chain_ms_per_frame": round(sum(med.values()), 1),
            "step1_projection": {"Mpoints_per_s": round(pts1 / s1 / 1e6, 4), "frames": frames1,
                                 "seconds": round(s1, 1)},
            "cpu": model, "cpu_index": cpu}


def kernel_source_id(kind):
    """The library's build-time id of the sources that define a timed kernel (kind "k1" or "pipeline";
    sv_source_id): a PMC profile records it (tools/prof.py traffic_json, from the library it profiled) beside the
    kernel's name, and bench.py uses the profile only when both match the library it timed."""
    import ctypes

    from svx import _abi
    buf = ctypes.create_string_buffer(64)
    _abi.call("sv_source_id", {"k1": 0, "pipeline": 1}[kind], buf, 64)
    return buf.value.decode()


def profile_traffic(path, frames, step, kernel, kind):
    """PMC HBM bytes per launch (k1) or per call (pipeline) from a traffic JSON (tools/prof.py pmc --traffic), and
    why it was not used if it was not: only a profile of this workload, of the same kernel instance (`kernel`, the
    name the batch reports for its timed launch) built from the same sources (kernel_source_id) counts."""
    try:
        with open(path) as fh:
            tj = json.load(fh)
    except (OSError, ValueError) as e:
        return None, f"no traffic profile ({type(e).__name__}: {os.path.relpath(path, REPO)})"
    if tj.get("frames") != frames or tj.get("step") != step:
        return None, f"profile is of {tj.get('frames')} frames step {tj.get('step')}, not {frames} step {step}"
    names = [tj.get("k1_kernel")] if kind == "k1" else list(tj.get("pipeline_kernels", {}))
    if kernel not in names:
        return None, f"profile measured {names}, the timed kernel is {kernel}"
    src, have = kernel_source_id(kind), tj.get("source_ids", {}).get(kind)
    if have != src:
        return None, f"profile built from sources {have}, the timed kernel from {src}"
    return tj.get("k1_hbm_bytes_per_launch" if kind == "k1" else "pipeline_hbm_bytes_per_call"), None


LINE_LIMIT = 6144   # bytes of the JSON line: the driver keeps the last 8 KB of stdout + stderr


def finalize(out, limit=LINE_LIMIT):
    """Order the line (the driver's contract fields, then the headline's sub-records, extras last) and hold it
    within `limit` bytes: the prose lives in DESIGN.md §6, the line carries numbers and short keys. If it is still
    too long, the least important records go first (placements, then extras' stage breakdowns), so the contract
    fields, roofline, cpu_baseline, pipeline and parity always survive."""
    order = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "latency_1frame_us", "pipeline",
             "parity"]
    o = {k: out[k] for k in order if k in out}
    o.update((k, v) for k, v in out.items() if k not in o)
    o["doc"] = "DESIGN.md §6"

    def size():
        return len(json.dumps(o, separators=(",", ":")).encode())
    drops = [("roofline", "placement"), ("pipeline", "placement"), ("extras", "sgbm_disparity", "placement"),
             ("extras", "device_frame_loop_serial", "stage_ms"), ("extras", "device_frame_loop_with_input", "stage_ms"),
             ("cpu_baseline", "step1_projection"), ("extras", "road_from_bitmap"), ("extras", "road_raster_nonzero")]
    for path in drops:
        if size() <= limit:
            break
        d = o
        for k in path[:-1]:
            d = d.get(k, {}) if isinstance(d, dict) else {}
        if isinstance(d, dict):
            d.pop(path[-1], None)
    return o


def ramp(fn, syncs, ms):
    """untimed calls of fn for `ms` of wall time, then a sync: the GPU's clocks settle before a timed region.
    A kernel run cold after host-side work (parity checks, the CPU legs) starts slow and speeds up over its first
    ~8 calls (the resident pipeline 6.8-7.0 ms -> 5.7-5.8 ms, profiles/r03/resident_dispatches_s*.json), as K1 did
    before --ramp-ms."""
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        fn()
        for s in syncs:
            s()


def ramp_agreed(fn, syncs, ms, ctrl):
    """ramp() for a step that holds a collective (the RCCL plane broadcast of the per-rank driver): every rank
    runs the SAME number of calls — one timed call each, then the largest count that fills `ms` on any rank
    (ctrl.max) — so the collectives pair up; a wall-clock loop per rank could run one call more or less on one
    of them and hang the next collective. Returns the number of calls made."""
    import math
    t0 = time.perf_counter()
    fn()
    for s in syncs:
        s()
    dt_ms = (time.perf_counter() - t0) * 1e3
    n = int(ctrl.max([float(math.ceil(ms / max(dt_ms, 1e-3)))])[0])
    for _ in range(n - 1):
        fn()
        for s in syncs:
            s()
    return max(n, 1)


def _timed(b, fn, reps, reset=False, ramp_ms=0.0):
    """mean ms of fn() over reps, HIP-synchronised around the loop (device work on the batch stream);
    reset: the batch's kernel timing starts after the warm-up call too; ramp_ms: untimed calls first (ramp)."""
    fn()
    b.sync()
    ramp(fn, (b.sync,), ramp_ms)
    if reset:
        b.reset_timing()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    b.sync()
    return (time.perf_counter() - t0) / reps * 1e3


def dropin_chain(fmod, disp, bgr, reps=5):
    """stereovision.py:84-113 for one host frame through the installed drop-ins,
    per stage (ms, median of reps): what a user of the reference sees after
    svx.dropin.install(functions), step 2 as the reference hard-codes."""
    import random
    st = {}
    n_pp = 0
    state = random.getstate()
    random.seed(0)
    for r in range(reps + 1):
        s = {}
        t = time.perf_counter()
        points = fmod.projectDisparityTo3d(disp, 128, bgr)
        s["a1_project_rgb"] = time.perf_counter() - t
        t = time.perf_counter()
        maskpoints = fmod.projectDisparityTo3d(fmod.maskDisparity(disp), 128)
        s["a1_project_masked"] = time.perf_counter() - t
        t = time.perf_counter()
        _, abc = fmod.RANSAC(maskpoints, 600)
        s["ransac_600"] = time.perf_counter() - t
        t = time.perf_counter()
        diffs = fmod.calculatePointErrors(abc, points)
        s["a2_point_errors"] = time.perf_counter() - t
        t = time.perf_counter()
        points = fmod.computePlanarThreshold(points, diffs, 0.05)
        s["a3_planar_threshold"] = time.perf_counter() - t
        t = time.perf_counter()
        hist = fmod.calculateColourHistogram(points)
        s["a5_colour_histogram"] = time.perf_counter() - t
        t = time.perf_counter()
        points = fmod.filterPointsByHistogram(points, hist, 10)
        s["a6_histogram_filter"] = time.perf_counter() - t
        t = time.perf_counter()
        pp = np.array(fmod.project3DPointsTo2DImagePoints(points), np.int32).reshape((-1, 1, 2))
        s["a7_a8_backproject_int32"] = time.perf_counter() - t
        n_pp = len(pp)
        if r > 0:   # the first run warms the device buffers
            for k, v in s.items():
                st.setdefault(k, []).append(v * 1e3)
    random.setstate(state)
    med = {k: round(float(np.median(v)), 2) for k, v in st.items()}
    return {"ms_per_frame": round(sum(med.values()), 2), "stage_ms": med, "plane_points": n_pp}


def check_plane_parity(b, first):
    """The per-frame-plane loop vs tests/golden/plane_digests.npz (the oracle's pre-pass -> maskpoints ->
    RANSAC(random.seed(F)) -> pipeline chain, make_plane_digests.py): each frame's winning trial, its error and
    plane bit for bit (numpy's rounding, functions.py:267-289) and its pipeline digests; (frames checked,
    mismatching)."""
    if b.step != 1 or not os.path.exists(GOLDEN_PLANES):
        return 0, 0
    gold = np.load(GOLDEN_PLANES)["planes"]
    n = min(b.frames, len(gold) - first)
    if first != 0 or n <= 0:
        return 0, 0
    got = b.digest("pipeline")[:n]
    want = gold[first:first + n]
    ok = got[:, 6] == 0
    for k, name in enumerate(DIGEST_FIELDS):
        ok &= got[:, k] == want[name].astype(np.uint64)
    for f in range(n):
        r = b.read_ransac(f)
        ok[f] &= bool(r["trial"] == want["trial"][f] and r["err"] == want["err"][f] and
                      np.array_equal(r["abc"].view(np.uint64), want["abc"][f].view(np.uint64)))
    return n, int((~ok).sum())


def extras(b, args, with_cpu, first=0):
    """SURVEY §8f components on the same resident batch (after the headline runs):
    road raster + non-zero walk of the pipeline's points, the disparity pre-pass
    (fillDisparity recurrence + carmask) over the batch, the RANSAC drop-in
    on one frame's masked points (600 trials) next to the CPU restatement, the
    batched RANSAC of every frame and the pipeline driven by those planes."""
    import random
    import types

    from svx import dropin, ransac

    import oracle
    from oracle import ransac as oransac
    ex = {}
    px = b.frames * H * W
    n2 = int(b.read_counts()[:, 2].sum())
    ms = _timed(b, lambda: (b.road_raster(sync=False), b.nonzero(sync=False)), 3, ramp_ms=args.ramp_ms / 3)
    # one pass (road_kernel): the points in (8 B each), the images out once, 4 B per non-zero pixel out (the walk's
    # packed x | y << 16 entries, widened to int32 pairs on read-back; at most one per point: counted as one per
    # point, so approx_GBps is an upper bound)
    byts = 8 * n2 + px + 4 * n2
    ex["road_raster_nonzero"] = {"ms_per_batch": round(ms, 3), "approx_GBps": round(byts / ms / 1e6, 1),
                                 "points": n2}
    mask = carmask()
    b.set_mask(mask)
    ms = _timed(b, lambda: b.prepass("previous", sync=False), 3, ramp_ms=args.ramp_ms / 3)
    # fillDisparity's recurrence: the disparity read, the cleaned frame written in place (maskDisparity is applied
    # by maskpoints as it reads the cleaned frame, not materialised)
    ex["prepass_fill_previous"] = {"ms_per_batch": round(ms, 3), "GBps": round(2 * px / ms / 1e6, 1),
                                   "frac": round(2 * px / ms / 1e6 / PEAK_HBM_GBS, 4)}
    # the per-frame-plane workload below is pinned end to end (tests/golden/plane_digests.npz): fresh frames,
    # ONE pre-pass over the batch in frame order (the timing above cleaned them four times), RANSAC with
    # random.seed(F), the pipeline with each frame's plane
    b.synth(first)
    b.prepass("previous", sync=True)
    disp, _ = oracle.synth_frame(0)
    pts = list(oracle.project(oracle.mask_disparity(disp, mask), None, 2)[0])
    st = random.getstate()
    random.seed(0)
    ransac.RANSAC(pts, 600)
    t0 = time.perf_counter()
    for s in range(5):
        random.seed(s)
        ransac.RANSAC(pts, 600)
    gpu_ms = (time.perf_counter() - t0) / 5 * 1e3
    r = {"points": len(pts), "trials": 600, "ms_per_call": round(gpu_ms, 2)}
    if with_cpu:
        t0 = time.perf_counter()
        random.seed(0)
        oransac.ransac(np.asarray(pts), 600)
        r["cpu_restatement_ms_per_call"] = round((time.perf_counter() - t0) * 1e3, 1)
    random.setstate(st)
    ex["ransac_dropin"] = r
    # batched RANSAC of every frame (maskpoints + seeded CPython-random replay on the device), then the
    # pipeline driven by each frame's own plane: stereovision.py:84-113 for the whole batch
    ms = _timed(b, lambda: b.ransac(seed_base=0, trials=600, sync=False), 2, ramp_ms=args.ramp_ms / 3)
    rb = {"frames": b.frames, "trials": 600, "ms_per_batch": round(ms, 2),
          "us_per_frame": round(ms / b.frames * 1e3, 2)}
    if "cpu_restatement_ms_per_call" in r:
        rb["cpu_restatement_ms_per_frame"] = r["cpu_restatement_ms_per_call"]
    ex["ransac_batch"] = rb
    # the first call after the RANSAC batch is a warm-up (6.9-7.0 ms against 6.5-6.7 for the calls after it,
    # profiles/r02/bench_session8_resident_dispatches.json), excluded from both clocks like the headline's
    ms = _timed(b, lambda: b.pipeline_planes(sync=False), 5, reset=True, ramp_ms=args.ramp_ms)
    k_ms, k_n = b.timing("pipeline")
    kept = int(b.read_counts()[:, 2].sum())
    fp_bytes = 4 * b.Ng * b.frames + 16 * kept + 4096 * b.frames   # the config-4 accounting, this call's points
    fp_s = k_ms / max(k_n, 1) / 1e3
    ex["pipeline_frame_planes"] = {"ms_per_batch": round(ms, 3), "gpu_ms_per_call": round(fp_s * 1e3, 4),
                                   "frames": b.frames, "kept_points": kept,
                                   "algorithmic_bytes_per_call": fp_bytes,
                                   "frac": round(fp_bytes / fp_s / 1e9 / PEAK_HBM_GBS, 4) if fp_s > 0 else None,
                                   "frac_at_survey_bytes": round((fp_bytes + 4 * kept) / fp_s / 1e9 / PEAK_HBM_GBS, 4)
                                   if fp_s > 0 else None}
    fp_tr, fp_why = profile_traffic(args.traffic_planes, b.frames, args.step, b.kernel_name("pipeline"), "pipeline")
    ex["pipeline_frame_planes"]["traffic"] = fp_tr
    ex["pipeline_frame_planes"]["traffic_src"] = "profiles/traffic_planes.json" if fp_tr else None
    if fp_tr:
        ex["pipeline_frame_planes"]["frac_of_traffic"] = round(fp_tr / fp_s / 1e9 / PEAK_HBM_GBS, 4) \
            if fp_s > 0 else None
    else:
        ex["pipeline_frame_planes"]["traffic_note"] = fp_why
    if not args.no_parity:
        pc, pm = check_plane_parity(b, first)
        ex["_planes_parity"] = [pc, pm]
    # the road pass of these points two ways: from the points (road_kernel: 8 B a point read) and from the
    # bitmap the resident pipeline writes as it makes them (sv_batch_road_bits: pass 2 marks the pixels, 68 KB a
    # frame; road_rowscan + road_rows kernels, one wave a row), with the pipeline's own time in both modes
    n2p = int(b.read_counts()[:, 2].sum())
    road_pts = _timed(b, lambda: b.road_raster(sync=False), 3, ramp_ms=args.ramp_ms / 3)
    b.road_bits(True)
    b.pipeline_planes(sync=True)
    _timed(b, lambda: b.pipeline_planes(sync=False), 5, reset=True, ramp_ms=args.ramp_ms / 3)
    kb_ms, kb_n = b.timing("pipeline")
    road_bits = _timed(b, lambda: b.road_raster(sync=False), 3, ramp_ms=args.ramp_ms / 3)
    b.road_bits(False)
    b.pipeline_planes(sync=True)
    px_all = b.frames * H * W
    ex["road_from_bitmap"] = {
        "road_ms_per_batch": round(road_bits, 3), "road_from_points_ms_per_batch": round(road_pts, 3),
        "pipeline_with_bitmap_gpu_ms_per_call": round(kb_ms / max(kb_n, 1), 4),
        "pipeline_gpu_ms_per_call": ex["pipeline_frame_planes"]["gpu_ms_per_call"],
        "points": n2p, "bytes_from_bitmap": 4 * 32 * H * b.frames + px_all + 4 * n2p,
        "bytes_from_points": 8 * n2p + px_all + 4 * n2p}

    fmod = types.SimpleNamespace(camera_focal_length_px=399.9745178222656, stereo_camera_baseline_m=0.2090607502,
                                 image_centre_w=474.5, image_centre_h=262.0, carmask=mask)
    dropin.install(fmod, unpinned=True)   # the chain calls fmod.maskDisparity (fmod has no cv2 original)
    try:
        d0, bgr0 = oracle.synth_frame(0)
        ex["dropin_frame_chain"] = dropin_chain(fmod, d0, bgr0)
    finally:
        dropin.uninstall()

    return ex


def loop_extra(args, device, first, mask):
    """stereovision.py:53-136 minus the cv2 drawing over a SEQUENCE of 4096-frame batches (svx.loop.FrameLoop):
    pre-pass -> maskpoints -> RANSAC(600) -> pipeline with each frame's plane -> road raster + walk, two batches in
    flight on two streams (batch k + 1's RANSAC beside batch k's pipeline and road), against the same loop with
    one batch at a time. `device_frame_loop` / `_serial`: the raw frames stay resident in the slots (generated once;
    a caller-fed slot keeps the frames written into it and its pre-pass writes the cleaned frames elsewhere, so
    every batch cleans the same raw frames), so a batch's time is the stages' alone;
    `device_frame_loop_with_input`: every batch first generates its synthetic frames on the device (global ids).
    Steady state: `warm` batches first (buffers, tables, clocks), then `reps` batches timed host-side from the end
    of the last warm-up batch to the end of the last one. The timed region starts from a drained loop (the first
    timed batch's stages run with nothing beside them, the last one's pipeline and road with no next draw), so
    `reps` is 16: four batches read 13.86 ms a batch where 32 read 13.50 on the same box. Then the parity leg: frames 0..4095 as two 2048-frame
    batches in flight, every frame against tests/golden/plane_digests.npz. Run after the headline batch is freed
    (two slots hold ~200 GB)."""
    from svx.loop import STAGES, FrameLoop
    out = {}
    frames, warm, reps = args.frames, 2, 16
    for key, slots, source in (("device_frame_loop", 2, "caller"), ("device_frame_loop_serial", 1, "caller"),
                               ("device_frame_loop_with_input", 2, "synth")):
        with FrameLoop(frames, slots=slots, source=source, carmask=mask, device=device) as loop:
            seq = None
            for i in range(warm + reps):
                if i == warm:
                    loop.wait(seq)
                    t0 = time.perf_counter()
                if source == "caller" and i < slots:   # the slot's frames, generated once and kept
                    loop.acquire().synth(first + i * frames)
                seq = loop.submit(first + i * frames)
            loop.wait(seq)
            ms = (time.perf_counter() - t0) / reps * 1e3
            tls = [loop.timeline(q) for q in range(seq - slots + 1, seq + 1)]
        stage_ms = {name: round(float(np.mean([tl[name][1] - tl[name][0] for tl in tls])), 3) for name in STAGES}
        r = {"ms_per_batch": round(ms, 2), "frames": frames, "frames_per_s": round(frames / ms * 1e3, 1),
             "slots": slots, "batches_timed": reps, "stage_ms": stage_ms}
        if slots == 2:
            a, b = tls[0], tls[1]   # batch k and k + 1: how much of k + 1's draw ran beside k's pipeline + road
            lo, hi = max(b["draw"][0], a["pipeline"][0]), min(b["draw"][1], a["road"][1])
            r["draw_overlap_ms"] = round(max(0.0, hi - lo), 3)
        out[key] = r
    par = None
    if not args.no_parity and os.path.exists(GOLDEN_PLANES) and args.step == 1 and first == 0:
        gold = np.load(GOLDEN_PLANES)["planes"]
        half = 2048
        if len(gold) >= 2 * half:
            bad = 0
            with FrameLoop(half, slots=2, carmask=mask, device=device) as loop:
                seqs = [loop.submit(0), loop.submit(half)]
                for q in seqs:
                    loop.wait(q)
                    b, f0 = loop.batch(q)
                    got = b.digest("pipeline")
                    want = gold[f0:f0 + half]
                    ok = got[:, 6] == 0
                    for k, name in enumerate(DIGEST_FIELDS):
                        ok &= got[:, k] == want[name].astype(np.uint64)
                    for f in range(half):
                        rr = b.read_ransac(f)
                        ok[f] &= bool(rr["trial"] == want["trial"][f] and rr["err"] == want["err"][f] and
                                      np.array_equal(rr["abc"].view(np.uint64), want["abc"][f].view(np.uint64)))
                    bad += int((~ok).sum())
            par = [2 * half, bad]
    return out, par


def sgbm_extra(sb, device, with_cpu, frames=128, chunk=128):
    """§8f rank 4: the disparity stage (functions.py:104-128: StereoSGBM(0,128,21) + filterSpeckles
    + scaling) on a resident batch of synthetic rectified pairs, frame 0 checked against the C
    oracle; then the whole per-frame loop from the stereo pair on the device."""
    from oracle import sgbm as osg
    out = {}
    with sb.Batch(frames, H, W, 1, with_bgr=True, with_points=True, device=device) as b:
        b.synth(0)                 # BGR (the pipeline's colours); the disparity comes from SGBM
        b.synth_pair(0)
        b.sgbm(chunk=chunk)
        b.reset_timing()
        ms = _timed(b, lambda: b.sgbm(chunk=chunk), 3)
        k_ms, k_n = b.timing("sgbm")
        L, R = osg.synth_pair(0)
        t0 = time.perf_counter()
        ref = osg.disparity(L, R)
        cpu_ms = (time.perf_counter() - t0) * 1e3
        r = {"frames": frames, "chunk": chunk, "ms_per_batch": round(ms, 2),
             "us_per_frame": round(k_ms / max(k_n, 1) / frames * 1e3, 1),
             "frame0_matches_oracle": bool(np.array_equal(b.read_disp(0), ref)),
             "placement": b.placement("sgbm")}
        if with_cpu:
            r["cpu_restatement_ms_per_frame"] = round(cpu_ms, 1)
        out["sgbm_disparity"] = r
        b.set_mask(carmask())
        b.synth_bgr_pair(0)        # BGR stereo pairs: the loop starts at stereovision.py:44

        def loop():
            b.preprocess(1.4, sync=False)   # gamma (in place: re-applied to the resident pairs each time), grey
            b.sgbm(chunk=chunk)
            b.prepass("previous", sync=False)
            b.ransac(seed_base=0, trials=600, sync=False)
            b.pipeline_planes(sync=False)
            b.road_raster(sync=False)
            b.nonzero(sync=False)
        ms = _timed(b, loop, 2)
        out["device_frame_loop_from_pairs"] = {
            "ms_per_batch": round(ms, 2), "frames": frames, "frames_per_s": round(frames / ms * 1e3, 1)}
    return out


def latency_1frame(sb, first, device):
    """configs[1]: one 1024x544 frame, step 1: K1 kernel time (HIP events), us."""
    with sb.Batch(1, H, W, 1, with_bgr=False, device=device) as one:
        # the same K1 as a separately named instance: its 1-frame launches are a
        # rocprof row of their own, so the batch launches' average stays unmixed
        one.tune(1, 2)
        one.synth(first)
        for _ in range(200):
            one.project(sync=False)
        one.reset_timing()
        for _ in range(50):
            one.project(sync=False)
        ms, n = one.timing("project")
        return round(ms / n * 1e3, 2)


def check_parity(batches, shards, what, step):
    """Every frame's device digest vs the oracle's (global frame ids); (frames checked, mismatching)."""
    if step not in (1, 2) or not os.path.exists(GOLDEN_DIGESTS):
        return 0, 0
    gold = np.load(GOLDEN_DIGESTS)[f"step{step}"]
    checked = bad = 0
    fields = ("n_valid", "disp_hash") if what == "dense" else \
        ("n_valid", "n_kept", "n_kept2", "disp_hash", "hist_hash", "pts_hash")
    for b, (_, first, count) in zip(batches, shards):
        if first + count > len(gold):
            continue
        got = b.digest(what)
        want = gold[first:first + count]
        ok = got[:, 6] == 0
        for k, name in enumerate(("n_valid", "n_kept", "n_kept2", "disp_hash", "hist_hash", "pts_hash")):
            if name in fields:
                ok &= got[:, k] == want[name].astype(np.uint64)
        checked += count
        bad += int((~ok).sum())
    return checked, bad


def main(argv=None):
    args = parse(argv)
    pl = plan(args.gpus, os.environ, args.driver)
    from svx import batch as sb
    from svx import dist

    import svx
    ctrl = dist.Control(rank=pl["rank"], world=pl["world"])
    if pl["mode"] == "multi" and svx.device_count() < args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but {svx.device_count()} GPU(s) visible")
    want_pipe = not args.no_pipeline
    shards = shards_of(pl, args.frames, args.global_frames)
    strong = args.global_frames > 0
    comm = mcomm = None
    comm_note = None
    if pl["mode"] == "ranks":   # RCCL over every rank (also at world size 1: the collective path runs)
        try:
            comm = dist.RcclComm(ctrl, pl["devices"][0])
        except svx.SvxError as e:   # every rank fails alike (a collective init): fall back, say so in the line
            comm_note = f"RCCL communicator unavailable ({e}); rank 0's plane sent over the host control plane"
        if ctrl.sum([0.0 if comm else 1.0])[0] > 0 and comm:
            comm.close()
            comm = None
            comm_note = comm_note or "RCCL communicator failed on another rank; plane over the host control plane"
    elif pl["mode"] == "multi":
        mcomm = dist.MultiComm(pl["devices"])

    # configs[1]: one frame, before the 4096-frame batch exists (its own warm-up inside)
    lat_us = None if (args.no_latency or pl["n_gpus"] > 1) else latency_1frame(sb, shards[0][1], shards[0][0])
    batches = []
    for dev, first, count in shards:
        b = sb.Batch(count, H, W, args.step, with_bgr=want_pipe, with_points=want_pipe, device=dev)
        b.tune(args.qpl, args.nt)
        b.synth(first)
        batches.append(b)
    ng = batches[0].Ng
    points_local = sum(ng * b.frames for b in batches)

    def sync_all():
        for b in batches:
            b.sync()

    def timed_steps(fn, steps):
        sync_all()
        ctrl.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        sync_all()
        ctrl.barrier()
        return time.perf_counter() - t0

    # ---- headline: K1 dense projection --------------------------------------
    t_ramp = time.perf_counter()
    while (time.perf_counter() - t_ramp) * 1e3 < args.ramp_ms:
        for b in batches:
            b.project(sync=False)
        sync_all()
    for _ in range(args.warmup):
        for b in batches:
            b.project(sync=False)
    for b in batches:
        b.reset_timing()
    dt = timed_steps(lambda: [b.project(sync=False) for b in batches], args.steps)
    agg = aggregate(ctrl, pl["n_gpus"], points_local, args.steps, dt)
    k_avg_s = float(ctrl.max([max(ms / max(n, 1) for ms, n in (b.timing("project") for b in batches)) / 1e3])[0])
    bytes_launch = K1_BYTES_PER_POINT * ng * batches[0].frames
    achieved = bytes_launch / k_avg_s / 1e9

    k1_name = batches[0].kernel_name("project")
    traffic, traffic_why = profile_traffic(args.traffic, batches[0].frames, args.step, k1_name, "k1")

    frames_gpu = batches[0].frames
    global_frames = int(ctrl.sum([sum(b.frames for b in batches)])[0])
    par = {"ranks": "torchrun ranks, RCCL", "multi": "one process, ncclCommInitAll",
           "single": "one process"}[pl["mode"]]
    out = {
        "metric": METRIC, "value": round(agg["value"], 1), "unit": "Mpoints/s", "n_gpus": pl["n_gpus"],
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(agg["ms_per_step"], 4),
        "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u8->f32",
        "data": "synthetic (SURVEY §8d generator, on device)",
        "config": {"workload": f"configs[2]: {frames_gpu}/GPU x {W}x{H}, step {args.step}, dense fp32 XYZ (K1)"
                               + (f"; configs[4]: {global_frames} frames over {pl['n_gpus']} GPUs"
                                  + (" (strong scaling)" if strong else "") if pl["n_gpus"] > 1 or strong else ""),
                   "frames_per_gpu": frames_gpu, "global_frames": global_frames, "H": H, "W": W,
                   "step": args.step, "grid_points_per_frame": ng,
                   "parallelism": f"frame-sharded x{pl['n_gpus']}; {par}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                     "kernel": k1_name, "kernel_ms": round(k_avg_s * 1e3, 4),
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "bytes_per_point": K1_BYTES_PER_POINT,
                     "placement": batches[0].placement("project")},
    }
    if traffic_why:
        out["roofline"]["traffic_note"] = traffic_why
    parity = {}
    if not args.no_parity:
        c, m = check_parity(batches, shards, "dense", args.step)
        parity["k1"] = [c, m]

    # ---- config 2: single-frame latency (measured first, before the batch) ----
    if lat_us is not None:
        out["latency_1frame_us"] = lat_us

    # ---- config 4/5: pipeline ----------------------------------------------
    if want_pipe:
        plane = sb.synthetic_plane()
        if comm:
            def pipe_step():
                dp = comm.broadcast_plane_dev(batches[0], plane, root=0)
                batches[0].pipeline_dev(dp, chunk=args.chunk, sync=False)
        elif mcomm:
            def pipe_step():
                mcomm.pipeline(batches, plane, root=0)
        else:   # one GPU, or ranks without RCCL: rank 0's plane (the same synthetic plane) over the control plane
            if pl["mode"] == "ranks":
                plane = tuple(float(v) for v in ctrl.sum(np.asarray(plane, np.float64) * (pl["rank"] == 0)))

            def pipe_step():
                batches[0].pipeline(plane=plane, chunk=args.chunk, sync=False)
        pipe_step()   # the first call places the output planes (pipe_place)
        sync_all()
        ramp_agreed(pipe_step, (sync_all,), args.ramp_ms, ctrl)   # the same call count on every rank
        for _ in range(max(1, args.warmup)):
            pipe_step()
        for b in batches:
            b.reset_timing()
        pdt = timed_steps(pipe_step, args.steps)
        pagg = aggregate(ctrl, pl["n_gpus"], points_local, args.steps, pdt)
        p_avg_s = float(ctrl.max([max(ms / max(n, 1) for ms, n in (b.timing("pipeline") for b in batches))
                                  / 1e3])[0])
        counts_local = np.sum([b.read_counts().sum(axis=0) for b in batches], axis=0).astype(np.float64)
        counts = ctrl.sum(counts_local)
        kept2_gpu0 = int(batches[0].read_counts()[:, 2].sum())
        pbytes = 4 * ng * frames_gpu + 16 * kept2_gpu0 + 4096 * frames_gpu
        survey_bytes = pbytes + 4 * kept2_gpu0   # SURVEY 8d's 20 B per kept point (int32 x and y stored apart)
        # bytes: 4 B read a grid point + 16 B a kept point as stored (fp32 X, Y, Z + the int32 pair as
        # int16 halves of one word) + 4 KB of histogram a frame; survey_bytes: SURVEY §8d's 20 B a kept point (an
        # effective rate, frac_at_survey_bytes); traffic: PMC bytes a call of this kernel instance and sources
        out["pipeline"] = {
            "gpu_ms_per_call": round(p_avg_s * 1e3, 4), "frac": round(pbytes / p_avg_s / 1e9 / PEAK_HBM_GBS, 4),
            "value": round(pagg["value"], 1), "unit": "Mpoints/s",
            "ms_per_step": round(pagg["ms_per_step"], 4),
            "achieved_GBps": round(pbytes / p_avg_s / 1e9, 1),
            "algorithmic_bytes_per_call": pbytes,
            "frac_at_survey_bytes": round(survey_bytes / p_avg_s / 1e9 / PEAK_HBM_GBS, 4),
            "counts_total": {"valid": int(counts[0]), "kept": int(counts[1]), "kept2": int(counts[2])},
            "plane_broadcast": comm_note or {"ranks": "RCCL ncclBroadcast to device memory",
                                             "multi": "RCCL grouped ncclBroadcast", "single": "host plane"}[pl["mode"]],
            "placement": batches[0].placement("pipeline"),
        }
        pname = batches[0].kernel_name("pipeline")
        out["pipeline"]["kernel"] = pname
        ptraffic, pwhy = profile_traffic(args.traffic_pipeline, frames_gpu, args.step, pname, "pipeline")
        out["pipeline"]["traffic"] = ptraffic
        if ptraffic:
            out["pipeline"]["frac_of_traffic"] = round(ptraffic / p_avg_s / 1e9 / PEAK_HBM_GBS, 4) \
                if p_avg_s > 0 else None
        else:
            out["pipeline"]["traffic_note"] = pwhy
        if not args.no_parity:
            c, m = check_parity(batches, shards, "pipeline", args.step)
            parity["pipeline"] = [c, m]

    single = pl["n_gpus"] == 1
    if want_pipe and not args.no_extras and single:   # §8f component timings: the N=1 run only
        out["extras"] = extras(batches[0], args, not args.no_cpu, shards[0][1])
        pp = out["extras"].pop("_planes_parity", None)
        if pp is not None:
            parity["pipeline_frame_planes"] = pp
        out["extras"].update(sgbm_extra(sb, shards[0][0], not args.no_cpu))

    if pl["rank"] == 0 and single and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)

    for b in batches:
        b.close()
    if want_pipe and not args.no_extras and single:   # the frame loop needs the headline batch's memory back
        lx, lpar = loop_extra(args, shards[0][0], shards[0][1], carmask())
        out["extras"].update(lx)
        if lpar is not None:
            parity["frame_loop"] = lpar
    if parity:
        tot = ctrl.sum(np.array([v for pair in parity.values() for v in pair], np.float64))
        keys = list(parity)
        out["parity"] = {k: {"frames_checked": int(tot[2 * i]), "mismatched_frames": int(tot[2 * i + 1])}
                         for i, k in enumerate(keys)}
        out["parity"]["pass"] = all(v["mismatched_frames"] == 0 and v["frames_checked"] > 0
                                    for k, v in out["parity"].items() if isinstance(v, dict))
    if comm:
        comm.close()
    if mcomm:
        mcomm.close()
    ctrl.barrier()
    out = finalize(out)
    if pl["rank"] == 0:
        print(json.dumps(out, separators=(",", ":")), flush=True)
    ctrl.close()
    return out


if __name__ == "__main__":
    main()
