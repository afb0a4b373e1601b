#!/bin/bash
# Row-walk probe: per-kernel times of the SGBM stage under two libraries (the product and an A/B build
# compiled with -DSVX_ROW_ABLATE=1/2/3: the walk's loads and stores without pass A's / pass B's / both passes'
# path steps; results invalid). VARIANTS="prod x y" compares tools/_ab/libsvx_x.so ... instead.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for pass in 1 2; do
  for v in ${VARIANTS:-prod abl1 abl2 abl3}; do
    if [ $v = prod ]; then L=$R/stereo.vision_amd/svx/_lib/libsvx.so; else L=$R/tools/_ab/libsvx_$v.so; fi
    rm -rf "$R/gpurun_out/row_${v}_$pass"
    SVX_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/row_${v}_$pass" -- python3 "$R/tools/prof.py" workload --what sgbm --frames 128 --reps 3 > "$R/gpurun_out/row_${v}_$pass.log" 2>&1 || { tail -20 "$R/gpurun_out/row_${v}_$pass.log"; exit 1; }
    python3 - "$R/gpurun_out/row_${v}_$pass" "$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "sgbm" in n:
            print(f"{sys.argv[2]} {n.split('(svx::SgbmK')[0].replace('void svx::(anonymous namespace)::','')} calls={r['Calls']} avg_ms={float(r['AverageNs'])/1e6:.3f}")
PY
  done
done
