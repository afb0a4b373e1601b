#!/bin/bash
# kernel timeline of the resident pipeline (2 calls) at one launch chunk
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; OUT="$PWD/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tlr" -o run -- \
  python3 tools/prof_mode.py --reps 2 --chunk ${CHUNK:-512} > "$OUT/tlr.log" 2>&1
rc=$?; echo "rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
python3 tools/trace_timeline.py "$OUT/tlr/run_kernel_trace.csv" | tail -${TAIL:-20}
