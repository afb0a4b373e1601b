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
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --cpu-seconds 5} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 "$OUT/bench.log"; stop_if_fatal $rc bench
if [ "${SKIP_PROF:-0}" != 1 ]; then
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu --no-latency > "$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof.log"; stop_if_fatal $rc rocprof
find "$OUT/prof" -name "*stats*" | head
fi
if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 600 python tools/sweep.py $SWEEP > "$OUT/sweep.log" 2>&1
  rc=$?; echo "sweep rc=$rc"; cat "$OUT/sweep.log" | tail -20
fi
