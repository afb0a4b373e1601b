#!/bin/bash
# Horizontal-sum store-pattern probe (diagnostic build; results invalid, per-kernel times only):
# SVX_SGBM_HSUM_ABLATE = 0 the kernel, 1 its stores with no arithmetic, 2 the stores interleaved by column,
# 3 the stores of 1 without the staging. One rocprofv3 kernel trace per variant, two alternations.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
export SVX_LIB=$R/stereo.vision_amd/svx/_lib/libsvx_diag.so
for pass in 1 2; do
  for a in 0 1 2 3; do
    rm -rf "$R/gpurun_out/hsum_${a}_$pass"
    SVX_SGBM_HSUM_ABLATE=$a timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/hsum_${a}_$pass" -- python3 "$R/tools/prof.py" workload --what sgbm --frames 128 --reps 3 > "$R/gpurun_out/hsum_${a}_$pass.log" 2>&1 || { tail -20 "$R/gpurun_out/hsum_${a}_$pass.log"; exit 1; }
    python3 - "$R/gpurun_out/hsum_${a}_$pass" "$a" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "sgbm" in n:
            print(f"abl={sys.argv[2]} {n.split('(')[0].split('::')[-1][:40]:40s} calls={r['Calls']:>3s} avg_ms={float(r['AverageNs'])/1e6:.3f}")
PY
  done
done
