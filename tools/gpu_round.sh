#!/bin/bash
# Full round-end evidence run: tests, bench, rocprofv3 kernel-trace stats of the
# bench command, PMC traffic of K1 + the pipeline at the bench workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"
SKIP_PROF=0 bash tools/gpu_check.sh || exit $?
rm -rf "$OUT/pmc"
WL="--what k1 --frames 4096 --reps 3" PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" bash tools/prof_counters.sh || exit $?
python tools/traffic.py "$OUT/pmc" 4096 1 > "$OUT/traffic_k1.json"
mv "$OUT/pmc" "$OUT/pmc_k1"
WL="--what pipe --frames 4096 --reps 1" PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" bash tools/prof_counters.sh || exit $?
python tools/traffic.py "$OUT/pmc" 4096 1 > "$OUT/traffic_pipe.json"
mv "$OUT/pmc" "$OUT/pmc_pipe"
cat "$OUT/traffic_k1.json" "$OUT/traffic_pipe.json"
