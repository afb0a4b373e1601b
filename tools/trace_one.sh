#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT="$PWD/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl" -o run -- \
  python3 tools/prof_workload.py --what pipe --frames 4096 --reps 2 --chunk ${CHUNK:-1024} > "$OUT/tl.log" 2>&1
rc=$?; echo "rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
python3 tools/trace_timeline.py "$OUT/tl/run_kernel_trace.csv" | tail -${TAIL:-16}
