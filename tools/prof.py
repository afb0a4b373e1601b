#!/usr/bin/env python3
"""The repo's one profiling entry point (GPU box; diagnostic, not product).

  prof.py workload  --what k1,pipe,planes,ransac,sgbm,prepass,raster [--frames N --reps R --mode M --chunk C]
        a fixed workload to run under rocprofv3 (nothing else on the GPU)
  prof.py time      --what ... [--sizes 1280,3840,4096] [--mode M]
        per-launch kernel ms (HIP events on the batch stream), one JSON line per size
  prof.py sweep     K1 launch shapes (--k1 qpl:nt,...) and pipeline chunk sizes (--modes, --chunks)
  prof.py ab        --modes resident,tiled --ablate 0,256 [--env NAME=v1,v2] [--what pipe|planes] [--with-k1]
        in-process A/B of pipeline variants (SVX_ABLATE diagnostics give INVALID results: times only)
  prof.py ab-lib    --libs a.so,b.so | --envs "K=V;K=V" --what pipe,planes
        A/B of libsvx builds (SVX_LIB) or environment settings, one child process per variant, alternating
  prof.py pmc       --groups "SQ_INSTS_VALU SQ_WAVE_CYCLES;FETCH_SIZE;WRITE_SIZE" [--ablate 0,256]
                    [--out gpurun_out/pmc] [--traffic FRAMES] -- <workload args>
        one `rocprofv3 --pmc` pass per group (never combined with tracing), then the summary
        (and, with --traffic, the HBM bytes JSON that bench.py reads)
  prof.py summary   DIR        mean counter value per dispatch and kernel
  prof.py traffic   DIR FRAMES STEP   per-launch HBM bytes (gfx950: fetched = 2 x FETCH_SIZE)
  prof.py trace     [--out DIR] -- <workload args>   kernel trace + per-dispatch timeline
  prof.py dropin    stereovision.py:84-113 through the installed drop-ins, ms per call

Counter limits per pass (gpurun refuses more): 8 SQ_, 4 TCC_ (FETCH_SIZE uses 3,
WRITE_SIZE 2), 4 TCP_, 2 TA_, 2 TD_, 2 GRBM_. Each rocprofv3 pass runs under
its own time limit; a fault, abort or timeout ends the command.
"""
import argparse
import csv
import glob
import json
import os
import statistics
import subprocess
import sys
import time
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "stereo.vision_amd")
sys.path[:0] = [REPO, PKG]
WHAT_TIMING = {"k1": "project", "pipe": "pipeline", "planes": "pipeline", "sgbm": "sgbm"}
# The SVX_* knobs (A/B selectors, placement probes, ablations) exist only in the diagnostic build
# (`make -C stereo.vision_amd/csrc diag`); this tool loads it unless SVX_LIB names another build.
os.environ.setdefault("SVX_LIB", os.path.join(PKG, "svx", "_lib", "libsvx_diag.so"))


def _batch(frames, what, mode="auto"):
    from svx import batch as sb
    pipe = any(w in what for w in ("pipe", "planes", "ransac", "sgbm", "raster"))
    b = sb.Batch(frames, step=1, with_bgr=pipe, with_points=pipe)
    b.synth(0)
    if pipe:
        b.pipeline_mode(mode)
    if "sgbm" in what:
        b.synth_pair(0)
    if "raster" in what:
        b.pipeline(sync=True)   # the points the raster draws
    if any(w in what for w in ("planes", "ransac", "prepass")):
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from test_prepass_cpu import carmask
        b.set_mask(carmask())
    if "planes" in what:   # as bench.py: RANSAC planes of the cleaned frames (fill previous + mask)
        b.prepass("previous", sync=True)
    return b


def _run(b, w, chunk=0, sync=False):
    if w == "k1":
        b.project(sync=sync)
    elif w == "pipe":
        b.pipeline(chunk=chunk, sync=sync)
    elif w == "planes":
        b.pipeline_planes(chunk=chunk, sync=sync)
    elif w == "ransac":
        b.ransac(seed_base=0, trials=600, sync=sync)
    elif w == "sgbm":
        b.sgbm(chunk=chunk)
    elif w == "prepass":
        b.prepass("previous", sync=sync)
    elif w == "raster":
        b.road_raster(sync=False)
        b.nonzero(sync=sync)
    else:
        raise SystemExit(f"unknown workload {w}")


def cmd_workload(a):
    if a.srcid_out:   # the sources of the library THIS process profiles (traffic_json reads them back)
        import bench
        with open(a.srcid_out, "w") as fh:
            json.dump({k: bench.kernel_source_id(k) for k in ("k1", "pipeline")}, fh)
    b = _batch(a.frames, a.what, a.mode)
    if "planes" in a.what:
        b.ransac(seed_base=0, trials=600)
    for _ in range(a.reps):
        for w in a.what.split(","):
            _run(b, w, a.chunk, sync=True)
    b.close()
    print("done", flush=True)


def cmd_time(a):
    for n in (int(s) for s in a.sizes.split(",")):
        b = _batch(n, a.what, a.mode)
        res = {"frames": n}
        if "planes" in a.what:
            b.ransac(seed_base=0, trials=600)
        for w in a.what.split(","):
            for _ in range(2):
                _run(b, w, a.chunk)
            b.sync()
            if w in WHAT_TIMING:
                b.reset_timing()
                for _ in range(a.reps):
                    _run(b, w, a.chunk)
                ms, cnt = b.timing(WHAT_TIMING[w])
                ms /= cnt
            else:   # no event timing: host wall time around synchronised launches
                t0 = time.perf_counter()
                for _ in range(a.reps):
                    _run(b, w, a.chunk)
                b.sync()
                ms = (time.perf_counter() - t0) / a.reps * 1e3
            res[w + "_ms"] = round(ms, 4)
            res[w + "_us_per_frame"] = round(ms / n * 1e3, 3)
        print(json.dumps(res), flush=True)
        b.close()


def cmd_sweep(a):
    b = _batch(a.frames, "k1,pipe")
    ng = b.Ng * a.frames
    for v in a.k1.split(","):
        qpl, nt = (int(t) for t in v.split(":"))
        b.tune(qpl, nt)
        b.project(sync=True)
        b.reset_timing()
        for _ in range(a.reps):
            b.project(sync=False)
        ms, n = b.timing("project")
        ms /= n
        print(json.dumps({"k1_qpl": qpl, "nt": nt, "ms": round(ms, 4), "GBps": round(13 * ng / ms / 1e6, 1)}),
              flush=True)
    b.tune(1, 1)
    for mode in a.modes.split(","):
        b.pipeline_mode(mode)
        for c in (int(x) for x in a.chunks.split(",")):
            b.pipeline(chunk=c, sync=True)
            b.reset_timing()
            for _ in range(a.reps):
                b.pipeline(chunk=c, sync=False)
            ms, n = b.timing("pipeline")
            print(json.dumps({"mode": mode, "chunk": c, "pipeline_ms": round(ms / n, 4)}), flush=True)
    b.close()


def cmd_ab(a):
    b = _batch(a.frames, "k1,pipe,planes" if a.what == "planes" else "k1,pipe")
    if a.what == "planes":
        b.ransac(seed_base=0, trials=600)
    ev = a.env.split("=", 1) if a.env else None   # NAME=v1,v2,... : one variant per value (in-process A/B)
    vals = ev[1].split(",") if ev else [""]
    variants = [(m, int(x), v) for m in a.modes.split(",") for x in a.ablate.split(",") for v in vals]
    if a.with_k1:   # the box's HBM speed beside the variants, to compare runs across boxes
        variants.append(("k1", 0, ""))
    res = {v: [] for v in variants}
    for _ in range(a.rounds):
        for mode, abl, v in variants:
            os.environ["SVX_ABLATE"] = str(abl)
            if ev and v:
                os.environ[ev[0]] = v
            k1 = mode == "k1"
            if not k1:
                b.pipeline_mode(mode)
            w = "k1" if k1 else a.what
            _run(b, w, sync=True)
            b.reset_timing()
            for _ in range(a.reps):
                _run(b, w)
            ms, n = b.timing(WHAT_TIMING[w])
            res[(mode, abl, v)].append(ms / n)
    os.environ["SVX_ABLATE"] = "0"
    if ev:
        os.environ.pop(ev[0], None)
    for (mode, abl, v), t in res.items():
        print(json.dumps({"mode": mode, "ablate": abl, "env": f"{ev[0]}={v}" if ev and v else "",
                          "median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4),
                          "max_ms": round(max(t), 4)}), flush=True)
    b.close()


def cmd_ab_lib(a):
    """variants = libsvx builds (--libs) or environment settings (--envs "K=V,K=V;K=V"), one child each"""
    if a.envs:
        variants = [(v, dict(kv.split("=", 1) for kv in v.split(",") if kv)) for v in a.envs.split(";")]
    else:
        variants = [(os.path.relpath(os.path.join(REPO, x), REPO), {"SVX_LIB": os.path.join(REPO, x)})
                    for x in a.libs.split(",")]
    res = {name: [] for name, _ in variants}
    for r in range(a.rounds):
        for name, extra in (variants if r % 2 == 0 else variants[::-1]):
            env = dict(os.environ, **extra)
            p = subprocess.run([sys.executable, __file__, "time", "--what", a.what, "--sizes", str(a.frames),
                                "--reps", str(a.reps)], env=env, capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print(p.stderr[-2000:], file=sys.stderr)
                sys.exit(p.returncode)
            res[name].append(json.loads(p.stdout.strip().splitlines()[-1]))
            print(name, res[name][-1], flush=True)
    for name, _ in variants:
        keys = [k for k in res[name][0] if k.endswith("_ms")]
        print(json.dumps({"variant": name, **{k: round(statistics.median(x[k] for x in res[name]), 4) for k in keys}}))


def _load_pmc(root):
    acc = defaultdict(lambda: defaultdict(list))
    files = set(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True))
    for f in sorted(files):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "")
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def cmd_summary(a):
    for k, cs in _load_pmc(a.dir).items():
        print(f"== {k[:64]}")
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} n={len(v):4d} mean={sum(v) / len(v):.4g}")


def traffic_json(root, frames, step):
    """FETCH_SIZE / WRITE_SIZE (KiB) -> HBM bytes per launch. gfx950 counts half the bytes of a
    coalesced streaming read in FETCH_SIZE (calibrated on K1's own loads: 570.4 MB read, 284.8 MB
    counted), so fetched = 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-byte streaming stores."""
    v = _load_pmc(root)
    out = {"frames": frames, "step": step, "source": root,
           "correction": "fetched = 2 x FETCH_SIZE (gfx950, calibrated on K1's loads); written = WRITE_SIZE"}
    # the sources the profiled kernels were built from, as the profiled `workload` process recorded them from the
    # library it loaded (source_ids.json beside each pass): bench.py uses a profile only for the same instance name
    # AND the same sources. Without that record (an older profile) no id is written and bench.py reports null.
    ids = {}
    for f in sorted(glob.glob(f"{root}/**/source_ids.json", recursive=True)):
        for kind, sid in json.load(open(f)).items():
            if ids.setdefault(kind, sid) != sid:
                ids[kind] = None   # passes of one profile from different libraries: no id
    kinds = {"k1": "project_dense_kernel", "pipeline": "resident_fused_kernel"}
    for kind, pat in kinds.items():
        if any(pat in k for k in v) and ids.get(kind):
            out.setdefault("source_ids", {})[kind] = ids[kind]
    for k, cs in v.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        if "project_dense_kernel" in k:
            fetch = 2 * 1024 * statistics.mean(cs["FETCH_SIZE"])
            write = 1024 * statistics.mean(cs["WRITE_SIZE"])
            out.update(k1_kernel=k, k1_fetch_bytes_per_launch=fetch, k1_write_bytes_per_launch=write,
                       k1_hbm_bytes_per_launch=fetch + write)
        if any(t in k for t in ("resident_fused_kernel", "stage_kernel", "offsets_kernel", "frame_planes_kernel")):
            out.setdefault("pipeline_kernels", {})[k] = {
                "launches": len(cs["FETCH_SIZE"]), "fetch_bytes_total": 2 * 1024 * sum(cs["FETCH_SIZE"]),
                "write_bytes_total": 1024 * sum(cs["WRITE_SIZE"])}
    if "pipeline_kernels" in out:   # `workload` runs one pipeline call per pass
        # the resident kernel runs once per call (a placement probe adds launches: count one mean launch)
        per = {k: (x["fetch_bytes_total"] + x["write_bytes_total"]) / (x["launches"] if "resident_fused" in k else 1)
               for k, x in out["pipeline_kernels"].items()}
        out["pipeline_hbm_bytes_per_call"] = sum(per.values())
    return out


def cmd_traffic(a):
    print(json.dumps(traffic_json(a.dir, a.frames, a.step), indent=1))


def _profile(args, out, workload):
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    os.makedirs(out, exist_ok=True)
    cmd = ["rocprofv3", *args, "--output-format", "csv", "-d", out, "-o", "run", "--",
           sys.executable, __file__, "workload", "--srcid-out", os.path.join(out, "source_ids.json"), *workload]
    with open(out + ".log", "w") as log:
        # no placement probes: counted bytes are per launch of the measured call
        p = subprocess.run(["timeout", "-s", "KILL", "180", *cmd], stdout=log, stderr=subprocess.STDOUT,
                           env=dict(os.environ, TMPDIR="/tmp", SVX_PIPE_TRIES="1", SVX_K1_TRIES="1"))
    return p.returncode


def cmd_pmc(a):
    groups = [g.split() for g in a.groups.split(";") if g.strip()]
    for abl in a.ablate.split(","):
        os.environ["SVX_ABLATE"] = abl
        root = os.path.join(a.out, f"a{abl}") if a.ablate != "0" else a.out
        for i, g in enumerate(groups, 1):
            rc = _profile(["--pmc", *g], os.path.join(root, f"p{i}"), a.workload)
            print(f"ablate {abl} pass {i} ({' '.join(g)}) rc={rc}", flush=True)
            if rc not in (0, 1):
                sys.exit(rc)   # fault / abort / timeout: touch the GPU no more
        a.dir = root
        cmd_summary(a)
        if a.traffic:
            with open(os.path.join(root, "traffic.json"), "w") as fh:
                json.dump(traffic_json(root, a.traffic, 1), fh, indent=1)
    os.environ["SVX_ABLATE"] = "0"


def cmd_trace(a):
    rc = _profile(["--kernel-trace"], os.path.join(a.out, "trace"), a.workload)
    if rc not in (0, 1):
        sys.exit(rc)
    rows = []
    for f in glob.glob(os.path.join(a.out, "trace", "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("svx::", "")[:32]
        print(f"q{r.get('Queue_Id', '?'):>2} {name:32s} start {(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f} us"
              f"  grid {r.get('Grid_Size_X', r.get('Grid_Size', '?'))}")


def cmd_dispatches(a):
    """Per-dispatch durations of the kernels matching a.kernel in a rocprofv3 kernel trace
    (the bench process's rocprof average mixes placement probes, timed calls and other workloads)."""
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = defaultdict(list)
    for r in rows:
        out[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(
            round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 4))
    print(json.dumps({"source": a.dir, "unit": "ms", "dispatches": out}, indent=1))


def cmd_dropin(a):
    import random
    import types

    import numpy as np

    import oracle
    from svx import dropin
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from test_prepass_cpu import carmask
    f = types.SimpleNamespace(camera_focal_length_px=399.9745178222656, stereo_camera_baseline_m=0.2090607502,
                              image_centre_w=474.5, image_centre_h=262.0, carmask=carmask())
    dropin.install(f, unpinned=True)
    disp, bgr = oracle.synth_frame(0)
    T = defaultdict(float)

    def t(name, fn, *args):
        t0 = time.perf_counter()
        r = fn(*args)
        T[name] += (time.perf_counter() - t0) * 1e3
        return r
    random.seed(0)
    for rep in range(a.reps + 1):
        if rep == 1:
            T.clear()
        points = t("a1 projectDisparityTo3d(rgb)", f.projectDisparityTo3d, disp, 128, bgr)
        mp = t("a1 projectDisparityTo3d(mask)", f.projectDisparityTo3d, t("maskDisparity", f.maskDisparity, disp), 128)
        _, abc = t("RANSAC(600)", f.RANSAC, mp, 600)
        diffs = t("a2 calculatePointErrors", f.calculatePointErrors, abc, points)
        points = t("a3 computePlanarThreshold", f.computePlanarThreshold, points, diffs, 0.05)
        hist = t("a5 calculateColourHistogram", f.calculateColourHistogram, points)
        points = t("a6 filterPointsByHistogram", f.filterPointsByHistogram, points, hist, 10)
        pp = t("a7 project3DPointsTo2DImagePoints", f.project3DPointsTo2DImagePoints, points)
        t("a8 int32 cast", lambda: np.array(pp, np.int32).reshape((-1, 1, 2)))
    for k, v in T.items():
        print(f"{k:40s} {v / a.reps:8.2f} ms")
    print(f"{'total':40s} {sum(T.values()) / a.reps:8.2f} ms")


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sp = ap.add_subparsers(dest="cmd", required=True)

    def common(p, what="pipe"):
        p.add_argument("--what", default=what)
        p.add_argument("--frames", type=int, default=4096)
        p.add_argument("--reps", type=int, default=3)
        p.add_argument("--mode", default="auto")
        p.add_argument("--chunk", type=int, default=0)
    p = sp.add_parser("workload")
    common(p, "k1,pipe")
    p.add_argument("--srcid-out", default="", help="write the loaded library's source ids here (JSON)")
    p = sp.add_parser("time")
    common(p)
    p.add_argument("--sizes", default="4096")
    p = sp.add_parser("sweep")
    p.add_argument("--frames", type=int, default=4096)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--k1", default="1:1,2:1,4:1,1:0")
    p.add_argument("--modes", default="tiled,resident")
    p.add_argument("--chunks", default="0")
    p = sp.add_parser("ab")
    p.add_argument("--frames", type=int, default=4096)
    p.add_argument("--modes", default="resident")
    p.add_argument("--ablate", default="0")
    p.add_argument("--env", default="", help="NAME=v1,v2: an environment knob read per call, one variant per value")
    p.add_argument("--what", default="pipe", choices=["pipe", "planes"])
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--with-k1", action="store_true")
    p = sp.add_parser("ab-lib")
    p.add_argument("--libs", default="")
    p.add_argument("--envs", default="")
    p.add_argument("--what", default="pipe")
    p.add_argument("--frames", type=int, default=4096)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--rounds", type=int, default=3)
    for name in ("pmc", "trace"):
        p = sp.add_parser(name)
        p.add_argument("--out", default=os.path.join(REPO, "gpurun_out", name))
        if name == "pmc":
            p.add_argument("--groups", default="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES "
                                               "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
                                               ";FETCH_SIZE;WRITE_SIZE")
            p.add_argument("--ablate", default="0")
            p.add_argument("--traffic", type=int, default=0, help="write traffic.json for this many frames")
        p.add_argument("workload", nargs=argparse.REMAINDER)
    p = sp.add_parser("summary")
    p.add_argument("dir")
    p = sp.add_parser("traffic")
    p.add_argument("dir")
    p.add_argument("frames", type=int)
    p.add_argument("step", type=int)
    p = sp.add_parser("dropin")
    p.add_argument("--reps", type=int, default=5)
    p = sp.add_parser("dispatches")
    p.add_argument("dir")
    p.add_argument("--kernel", default="resident_fused")
    a = ap.parse_args()
    if getattr(a, "workload", None) is not None:
        a.workload = [w for w in a.workload if w != "--"]
    {"workload": cmd_workload, "time": cmd_time, "sweep": cmd_sweep, "ab": cmd_ab, "ab-lib": cmd_ab_lib,
     "pmc": cmd_pmc, "summary": cmd_summary, "traffic": cmd_traffic, "trace": cmd_trace,
     "dropin": cmd_dropin, "dispatches": cmd_dispatches}[a.cmd](a)


if __name__ == "__main__":
    main()
