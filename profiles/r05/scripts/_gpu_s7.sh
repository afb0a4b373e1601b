#!/bin/bash
# round-5 session 7: branch-free fp32 RANSAC screen + vectorised LDS fill, deferred-return binning:
# RANSAC / loop / parity tests, then the RANSAC kernels and the frame loop under the committed library
# (libsvx_base.so) and this one
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s7"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ransac_batch.py tests/test_gpu_ransac.py tests/test_gpu_loop.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
L=stereo.vision_amd/svx/_lib
i=0
for lib in $L/libsvx_base.so $L/libsvx.so; do
  i=$((i+1))
  SVX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$i" -o run -- python3 tools/prof.py workload --what ransac --frames 4096 --reps 5 > "$OUT/prof_$i.log" 2>&1 || { echo "prof $i failed"; tail "$OUT/prof_$i.log"; exit 1; }
  python3 - "$OUT/prof_$i" "$lib" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
print("==", sys.argv[2])
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{r["Name"][:60]:62s} {r["Calls"]:>4s} {float(r["AverageNs"]) / 1e3:9.1f} us')
PY
done
for lib in $L/libsvx_base.so $L/libsvx.so $L/libsvx_base.so $L/libsvx.so; do
  echo "== loop $lib"
  SVX_LIB=$PWD/$lib PROBE_ONLY=caller2,caller1 timeout -k 10 300 python3 -u tools/_probe_loop.py > "$OUT/loop.tmp" 2>&1 || { echo "loop failed"; tail "$OUT/loop.tmp"; exit 1; }
  grep -v "batch" "$OUT/loop.tmp" | tail -6
  cat "$OUT/loop.tmp" >> "$OUT/loop.log"
done
# the pipeline's write pattern: four planes vs one plane of 16-byte records (tools/sol_pipe.hip r05 modes 8, 9)
timeout -k 10 120 ./tools/_sol_pipe r05 4096 277200 50 5 > "$OUT/sol_pipe_aos.txt" 2>&1 || { echo "sol_pipe failed"; tail "$OUT/sol_pipe_aos.txt"; exit 1; }
grep '"round": 1' "$OUT/sol_pipe_aos.txt"
# the road rows kernel, rows a wave (diagnostic build's SVX_ROAD_RPW), in one process alternating
SVX_LIB=$PWD/$L/libsvx_diag.so PROBE_RPW=1,2,4 timeout -k 10 300 python3 -u tools/_probe_road.py > "$OUT/probe_road_rpw.txt" 2>&1 || { echo "road probe failed"; tail "$OUT/probe_road_rpw.txt"; exit 1; }
cat "$OUT/probe_road_rpw.txt"
