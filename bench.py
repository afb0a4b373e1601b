#!/usr/bin/env python3
"""Benchmark: Mpoints/s of disparity->3D at 1024x544 and achieved HBM GB/s vs peak.

Headline workload (BASELINE.json configs[2], the north-star target): a batch of
4096 synthetic 1024x544 disparity maps per GPU, step 1 (555,489 grid points per
frame), resident in HBM, projected by K1 into dense fp32 X/Y/Z planes. One
"step" = one K1 pass over the whole batch. Multi-GPU (configs[4]): one process
per GPU, 4096 frames per rank (weak scaling), frames sharded by global id, no
data-path collective.

Also reported (same JSON line):
  pipeline      configs[3]/[4]: plane threshold + hue histogram + ordered
                compaction + int32 back-projection over the same batch; for
                N>1 each step starts with the RCCL broadcast of the plane.
  latency_1frame_us  configs[1]: one frame, step 1, K1 kernel time.
  cpu_baseline  the nested-loop CPU port (oracle/cpu_loop.py, same numpy-scalar
                semantics as functions.py:178-198), rank 0 at N=1 only.

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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=4096, help="frames per GPU")
    ap.add_argument("--step", type=int, default=1, help="grid step (reference hard-codes 2)")
    ap.add_argument("--chunk", type=int, default=0, help="pipeline frames per wave (0 = default)")
    ap.add_argument("--qpl", type=int, default=1, help="K1 quads (4 points) per lane: 1, 2, 4")
    ap.add_argument("--nt", type=int, default=1, help="non-temporal K1 stores (1 = measured faster)")
    ap.add_argument("--ramp-ms", type=float, default=300.0,
                    help="untimed K1 launches before the warmup steps, to let clocks settle")
    ap.add_argument("--no-pipeline", action="store_true")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the 1-frame latency probe")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the SURVEY §8f component timings")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--traffic-pipeline", default=os.path.join(REPO, "profiles", "traffic_pipeline.json"))
    return ap.parse_args()


def cpu_baseline(budget_s):
    """Nested-loop port (oracle/cpu_loop.py) on 1 core; bounded sample of whole frames."""
    import oracle
    from oracle import cpu_loop
    try:
        os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
    except (AttributeError, OSError):
        pass
    pts = 0
    frames = 0
    t0 = time.perf_counter()
    while True:
        disp, _ = oracle.synth_frame(frames)
        rows = cpu_loop.project(disp, None, step=1)
        pts += (H - 1) * (W - 1)
        frames += 1
        assert len(rows) > 0
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    # C restatement, 1 thread, same frames (for scale; not the reported baseline)
    t1 = time.perf_counter()
    for f in range(frames):
        disp, _ = oracle.synth_frame(f)
        oracle.project(disp, None, 1)
    dtc = time.perf_counter() - t1
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": pts / dt / 1e6, "unit": "Mpoints/s", "cores": 1, "kind": "port",
            "sample": f"{frames} synthetic 1024x544 frames, step 1, projection only "
                      f"({pts} grid points, {dt:.1f} s): oracle/cpu_loop.py nested loop "
                      f"(functions.py:178-198 semantics)",
            "c_restatement_mpts": pts / dtc / 1e6, "cpu": model}


def pipeline_traffic(path, frames, step):
    """PMC HBM bytes per pipeline call (tools/traffic.py output), if measured at this workload."""
    try:
        with open(path) as fh:
            tj = json.load(fh)
    except (OSError, ValueError):
        return None
    if tj.get("frames") != frames or tj.get("step") != step:
        return None
    return tj.get("pipeline_hbm_bytes_per_call")


def _timed(b, fn, reps):
    """mean ms of fn() over reps, HIP-synchronised around the loop (device work on the batch stream)."""
    fn()
    b.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    b.sync()
    return (time.perf_counter() - t0) / reps * 1e3


def extras(b, sb, args, device, with_cpu):
    """SURVEY §8f components on the same resident batch (after the headline runs):
    road raster + non-zero walk of the pipeline's points, the disparity pre-pass
    (fillDisparity recurrence + carmask) over the batch, the RANSAC drop-in
    on one frame's masked points (600 trials) next to the CPU restatement, the
    batched RANSAC of every frame and the pipeline driven by those planes."""
    import random

    from svx import ransac

    import oracle
    from oracle import ransac as oransac
    ex = {}
    px = b.frames * H * W
    n2 = int(b.read_counts()[:, 2].sum())
    ms = _timed(b, lambda: (b.road_raster(sync=False), b.nonzero(sync=False)), 3)
    byts = px + 8 * n2 + px + 8 * n2          # raster: zero + point reads (+1 B each); walk: image + [j,i]
    ex["road_raster_nonzero"] = {"ms_per_batch": round(ms, 3), "approx_GBps": round(byts / ms / 1e6, 1),
                                 "points": n2, "kernels": "raster_kernel + nonzero_kernel"}
    mask = np.zeros((H, W), np.uint8)
    mask[H // 3:, 64:W - 64] = 255            # a carmask-like region (timing only)
    b.set_mask(mask)
    ms = _timed(b, lambda: b.prepass("previous", sync=False), 3)
    ex["prepass_fill_previous_masked"] = {"ms_per_batch": round(ms, 3), "GBps": round(3 * px / ms / 1e6, 1),
                                          "bytes_per_pixel": 3, "kernel": "fill_prev_kernel"}
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
    r = {"points": len(pts), "trials": 600, "ms_per_call": round(gpu_ms, 2),
         "path": "host CPython-random replay + ransac_eval_kernel + numpy re-decision of the winner"}
    if with_cpu:
        t0 = time.perf_counter()
        random.seed(0)
        oransac.ransac(np.asarray(pts), 600)
        r["cpu_restatement_ms_per_call"] = round((time.perf_counter() - t0) * 1e3, 1)
    random.setstate(st)
    ex["ransac_dropin"] = r
    # batched RANSAC of every frame (maskpoints + seeded CPython-random replay on the device), then the
    # pipeline driven by each frame's own plane: stereovision.py:84-113 for the whole batch
    ms = _timed(b, lambda: b.ransac(seed_base=0, trials=600, sync=False), 2)
    rb = {"frames": b.frames, "trials": 600, "ms_per_batch": round(ms, 2),
          "us_per_frame": round(ms / b.frames * 1e3, 2), "kernels": "maskpoints_kernel + ransac_batch_kernel",
          "rng": "random.seed(frame) per frame"}
    if "cpu_restatement_ms_per_call" in r:
        rb["cpu_restatement_ms_per_frame"] = r["cpu_restatement_ms_per_call"]
    ex["ransac_batch"] = rb
    ms = _timed(b, lambda: b.pipeline_planes(sync=False), 3)
    ex["pipeline_frame_planes"] = {"ms_per_batch": round(ms, 3), "frames": b.frames,
                                   "kept_points": int(b.read_counts()[:, 2].sum()),
                                   "kernels": "frame_planes_kernel + stage_kernel<PF> + offsets_kernel"}

    # stereovision.py:84-113 for one host frame through the installed drop-ins (what a user of the
    # reference sees after svx.dropin.install(functions)): 2 projections, RANSAC(600), the four stages,
    # back-projection and the int32 cast; step 2 as the reference hard-codes
    import types

    from svx import dropin
    fmod = types.SimpleNamespace(camera_focal_length_px=399.9745178222656, stereo_camera_baseline_m=0.2090607502,
                                 image_centre_w=474.5, image_centre_h=262.0, carmask=mask)
    dropin.install(fmod)
    try:
        disp, bgr = oracle.synth_frame(0)

        def chain():
            points = fmod.projectDisparityTo3d(disp, 128, bgr)
            maskpoints = fmod.projectDisparityTo3d(fmod.maskDisparity(disp), 128)
            _, abc = fmod.RANSAC(maskpoints, 600)
            diffs = fmod.calculatePointErrors(abc, points)
            points = fmod.computePlanarThreshold(points, diffs, 0.05)
            hist = fmod.calculateColourHistogram(points)
            points = fmod.filterPointsByHistogram(points, hist, 10)
            pp = np.array(fmod.project3DPointsTo2DImagePoints(points), np.int32).reshape((-1, 1, 2))
            return len(pp)
        st = random.getstate()
        random.seed(0)
        chain()
        t0 = time.perf_counter()
        for _ in range(5):
            n_pp = chain()
        ex["dropin_frame_chain"] = {"ms_per_frame": round((time.perf_counter() - t0) / 5 * 1e3, 2),
                                    "plane_points": n_pp,
                                    "stages": "stereovision.py:84-113 via installed drop-ins, step 2, RANSAC 600",
                                    "reference_ms_per_frame_survey": "~1,450 (SURVEY §8a, measured in the "
                                                                     "build container: a1 2x150-180, a2 30, a3 55, "
                                                                     "a5 300, a6 300, a7 45, a8 16, RANSAC ~380)"}
        random.setstate(st)
    finally:
        dropin.uninstall()

    # the whole per-frame loop of stereovision.py:53-136 that is not cv2, back to back on the resident batch:
    # fill + mask pre-pass, maskpoints + RANSAC, the pipeline with each frame's plane, road raster + walk
    def frame_loop():
        b.prepass("previous", sync=False)
        b.ransac(seed_base=0, trials=600, sync=False)
        b.pipeline_planes(sync=False)
        b.road_raster(sync=False)
        b.nonzero(sync=False)
    ms = _timed(b, frame_loop, 2)
    ex["device_frame_loop"] = {"ms_per_batch": round(ms, 2), "frames": b.frames,
                               "frames_per_s": round(b.frames / ms * 1e3, 1),
                               "stages": "prepass(previous+mask) -> maskpoints+RANSAC(600) -> pipeline(per-frame "
                                         "planes) -> road raster -> non-zero walk"}
    return ex


def latency_1frame(sb, step, first, device):
    """configs[1]: one 1024x544 frame, step 1: K1 kernel time (HIP events), us."""
    with sb.Batch(1, H, W, step, with_bgr=False, device=device) as one:
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


def main():
    args = parse()
    from svx import batch as sb
    from svx import dist

    rank, world, local = dist.env_topology()
    ctrl = dist.Control()
    # RCCL whenever launched by torchrun (also at world size 1, so the device
    # collective path is the one that runs), never for a plain `python bench.py`
    comm = dist.RcclComm(ctrl, local) if "WORLD_SIZE" in os.environ else None
    first, count = dist.shard(args.frames * world, world, rank)
    want_pipe = not args.no_pipeline

    # configs[1]: one frame, before the 4096-frame batch exists (its own warm-up inside)
    lat_us = None if args.no_latency else latency_1frame(sb, args.step, first, local)
    b = sb.Batch(count, H, W, args.step, with_bgr=want_pipe, with_points=want_pipe, device=local)
    b.tune(args.qpl, args.nt)
    b.synth(first)
    ng = b.Ng
    points_rank = ng * count

    # ---- headline: K1 dense projection --------------------------------------
    t_ramp = time.perf_counter()
    while (time.perf_counter() - t_ramp) * 1e3 < args.ramp_ms:
        b.project(sync=True)
    for _ in range(args.warmup):
        b.project(sync=False)
    b.sync()
    b.reset_timing()
    ctrl.barrier()
    b.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.project(sync=False)
    b.sync()
    ctrl.barrier()
    dt = time.perf_counter() - t0
    dt_max = float(ctrl.max([dt])[0])
    k_ms, k_n = b.timing("project")
    k_avg_s = float(ctrl.max([k_ms / max(k_n, 1) / 1e3])[0])
    total_points = points_rank * world * args.steps
    value = total_points / dt_max / 1e6
    bytes_launch = K1_BYTES_PER_POINT * points_rank
    achieved = bytes_launch / k_avg_s / 1e9

    traffic = None
    if os.path.exists(args.traffic):
        try:
            with open(args.traffic) as fh:
                tj = json.load(fh)
            if tj.get("frames") == count and tj.get("step") == args.step:
                traffic = tj.get("k1_hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "Mpoints/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt_max / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8->f32",
        "data": "synthetic (counter-based generator of SURVEY §8d, generated on device)",
        "config": {"workload": f"configs[2]: batch={count}/GPU synthetic {W}x{H} disparity maps, "
                               f"step {args.step}, dense fp32 XYZ planes (K1)",
                   "frames_per_gpu": count, "global_frames": count * world, "H": H, "W": W,
                   "step": args.step, "grid_points_per_frame": ng,
                   "parallelism": f"frame-sharded x{world} (no data-path collective)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                     "kernel": "project_dense_kernel", "kernel_ms": round(k_avg_s * 1e3, 4),
                     "algorithmic_bytes_per_launch": bytes_launch,
                     "bytes_per_point": K1_BYTES_PER_POINT},
    }

    # ---- config 2: single-frame latency (measured first, before the batch) ----
    if lat_us is not None:
        out["latency_1frame_us"] = lat_us

    # ---- config 4/5: pipeline ----------------------------------------------
    if want_pipe:
        plane = sb.synthetic_plane()
        for _ in range(max(1, args.warmup)):
            b.pipeline(plane=plane, chunk=args.chunk, sync=False)
        b.sync()
        b.reset_timing()
        ctrl.barrier()
        b.sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            pl = comm.broadcast_plane(plane, root=0) if comm else plane
            b.pipeline(plane=pl, chunk=args.chunk, sync=False)
        b.sync()
        ctrl.barrier()
        pdt = float(ctrl.max([time.perf_counter() - t0])[0])
        p_ms, p_n = b.timing("pipeline")
        p_avg_s = float(ctrl.max([p_ms / max(p_n, 1) / 1e3])[0])
        counts = b.read_counts().sum(axis=0)
        if comm:
            counts = comm.allreduce_i64(counts)
        n_kept2 = int(counts[2])
        pbytes = 4 * points_rank + (20 * int(b.read_counts()[:, 2].sum())) + 4096 * count
        out["pipeline"] = {
            "workload": "configs[3]/[4]: same batch, plane threshold 0.05 + hue histogram (thr 10) "
                        "+ ordered compaction + int32 back-projection",
            "value": round(points_rank * world * args.steps / pdt / 1e6, 1), "unit": "Mpoints/s",
            "ms_per_step": round(pdt / args.steps * 1e3, 4), "gpu_ms_per_call": round(p_avg_s * 1e3, 4),
            "achieved_GBps": round(pbytes / p_avg_s / 1e9, 1),
            "frac": round(pbytes / p_avg_s / 1e9 / PEAK_HBM_GBS, 4),
            "algorithmic_bytes_per_call": pbytes,
            "bytes_note": "algorithmic = SURVEY 8d config 4: 4 B read per grid point (disparity + BGR) + 20 B per "
                          "kept point + 4 KB histogram per frame; the resident kernel does not read the BGR (nor, "
                          "in pass 2, the disparity) of chunks the keep table rules out, so it moves fewer bytes "
                          "(traffic = PMC bytes per call, frac_of_traffic = traffic / time / peak)",
            "counts_total": {"valid": int(counts[0]), "kept": int(counts[1]), "kept2": n_kept2},
            "plane_broadcast": "RCCL ncclBroadcast over xGMI, every step" if comm else "n/a (single process)",
            "kernels": "keep_table_kernel (per call) + resident_fused_kernel (one workgroup per frame)"
                       if args.frames >= 512 else "tiled: stage_kernel + offsets_kernel",
        }
        ptraffic = pipeline_traffic(args.traffic_pipeline, count, args.step)
        if ptraffic:
            out["pipeline"]["traffic"] = ptraffic
            out["pipeline"]["frac_of_traffic"] = round(ptraffic / p_avg_s / 1e9 / PEAK_HBM_GBS, 4)

    if want_pipe and not args.no_extras and world == 1:   # §8f component timings: the N=1 run only
        out["extras"] = extras(b, sb, args, local, not args.no_cpu)

    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)

    b.close()
    if comm:
        comm.close()
    ctrl.barrier()
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctrl.close()


if __name__ == "__main__":
    main()
