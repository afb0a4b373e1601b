#!/usr/bin/env python3
"""Per-launch HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Corrections (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE counts half the
bytes of a coalesced streaming read — calibrated for K1's own 4-byte-per-lane
disparity loads: 1024 frames x 544 x 1024 B = 570.4 MB read, FETCH_SIZE =
284.8 MB, ratio 0.4993 — so fetched bytes = 2 x FETCH_SIZE; WRITE_SIZE is
exact for our 16-byte-per-lane streaming stores (1024 x 543 x 1024 x 12 B =
6.833 GB, WRITE_SIZE = 6.836 GB). Both counters are in KiB.

usage: traffic.py PMC_DIR FRAMES STEP > profiles/traffic.json
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def load(root):
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    root, frames, step = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    v = load(root)
    out = {"frames": frames, "step": step, "source": root,
           "correction": "fetched = 2 x FETCH_SIZE (gfx950, calibrated on K1's loads); written = WRITE_SIZE"}
    for k, cs in v.items():
        if "project_dense_kernel" in k:
            fetch = 2 * 1024 * sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
            write = 1024 * sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
            out["k1_kernel"] = k
            out["k1_fetch_bytes_per_launch"] = fetch
            out["k1_write_bytes_per_launch"] = write
            out["k1_hbm_bytes_per_launch"] = fetch + write
        if any(t in k for t in ("resident_fused_kernel", "keep_table_kernel", "stage_kernel", "offsets_kernel")):
            pk = out.setdefault("pipeline_kernels", {})
            pk[k] = {"launches": len(cs["FETCH_SIZE"]),
                     "fetch_bytes_total": 2 * 1024 * sum(cs["FETCH_SIZE"]),
                     "write_bytes_total": 1024 * sum(cs["WRITE_SIZE"])}
    if "pipeline_kernels" in out:   # per call (prof_workload runs one pipeline call)
        out["pipeline_hbm_bytes_per_call"] = sum(v["fetch_bytes_total"] + v["write_bytes_total"]
                                                 for v in out["pipeline_kernels"].values())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
