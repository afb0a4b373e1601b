#!/bin/bash
# One GPU-box evidence session: the GPU suite, smoke, the default bench under rocprofv3 --kernel-trace --stats
# (JSON line + per-kernel stats from the same process), then PMC HBM traffic of K1 / the pipeline / the
# per-frame-plane pipeline at the bench workload (profiles bench.py matches by kernel instance and sources).
# Every GPU step has its own time limit; a fault, abort or timeout ends the script (no retries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-s}"
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { case "$1" in 0) ;; *) echo "FATAL rc=$1 in $2"; exit "$1";; esac; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; ok $rc pytest
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; ok $rc smoke
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; tail -c 600 "$OUT/bench.json"; ok $rc bench
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  for w in k1:3 pipe:1 planes:1; do
    timeout -k 10 300 python3 -u tools/prof.py pmc --groups "FETCH_SIZE;WRITE_SIZE" --out "$OUT/pmc_${w%%:*}" \
      --traffic 4096 -- --what "${w%%:*}" --frames 4096 --reps "${w##*:}" > "$OUT/pmc_${w%%:*}.log" 2>&1
    rc=$?; echo "pmc ${w%%:*} rc=$rc"; ok $rc "pmc ${w%%:*}"
  done
fi
echo "session done"
