#!/bin/bash
# kernel-trace stats of the pipeline alone (no PMC), one chunk setting
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
for c in ${CHUNKS:-4096}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_$c" -o run -- \
    python3 tools/prof_workload.py --what pipe --frames 4096 --reps 3 --chunk $c > "$OUT/tr_$c.log" 2>&1
  rc=$?; echo "chunk $c rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
  cut -c1-150 "$OUT/tr_$c/run_kernel_stats.csv"
done
