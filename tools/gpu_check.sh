#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"
mkdir -p "$OUT"
stop_if_fatal() {  # exit codes that mean fault / abort / timeout: do not touch the GPU again
  case "$1" in 0|1|5) ;; *) echo "FATAL rc=$1 in $2"; exit "$1";; esac
}
TESTS="${TESTS:-tests}"
timeout -k 10 "${PYTEST_LIMIT:-900}" python -m pytest $TESTS -m gpu -q ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu.log"; stop_if_fatal $rc pytest
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
# The bench runs once, under rocprofv3 --kernel-trace --stats, so the JSON line
# (HIP-event kernel times) and the kernel stats come from the same process.
export TMPDIR=/tmp
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --cpu-seconds 10} > "$OUT/bench.log" 2>&1
  rc=$?; echo "bench (rocprof) rc=$rc"; tail -2 "$OUT/bench.log"; stop_if_fatal $rc bench
  find "$OUT/prof" -name "*stats*" | head
else
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --cpu-seconds 10} > "$OUT/bench.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -2 "$OUT/bench.log"; stop_if_fatal $rc bench
fi
if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 600 python tools/prof.py sweep $SWEEP > "$OUT/sweep.log" 2>&1
  rc=$?; echo "sweep rc=$rc"; cat "$OUT/sweep.log" | tail -20
fi
