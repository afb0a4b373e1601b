#!/bin/bash
# SGBM walk A/B: parity tests, alternating-process timing against a saved build, kernel stats of the new build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sgbm.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_sgbm.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_sgbm.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python tools/prof.py ab-lib --libs "${BASE:?set BASE to the saved build to compare against}",stereo.vision_amd/svx/_lib/libsvx.so --what sgbm --frames 128 --reps 3 --rounds ${ROUNDS:-4} > "$OUT/ab_sgbm.txt" 2>&1
rc=$?; tail -4 "$OUT/ab_sgbm.txt"; [ $rc = 0 ] || exit $rc
SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_sgbm" -o run -- python3 tools/prof.py workload --what sgbm --frames 128 --reps 2 > "$OUT/prof_sgbm.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc = 0 ] || exit $rc
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_sgbm/**/run_kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
