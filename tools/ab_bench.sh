#!/bin/bash
# A/B of libsvx builds through bench.py (one process per run, alternating): K1 and pipeline lines only.
# usage: tools/ab_bench.sh ROUNDS LIB_A LIB_B [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$1; A=$2; B=$3; shift 3
for r in $(seq 1 "$R"); do
  for lib in "$A" "$B"; do
    SVX_LIB="$PWD/$lib" timeout -k 10 120 python bench.py --no-extras --no-latency --no-cpu --no-parity "$@" \
      > gpurun_out/ab_bench_run.log 2>&1 || { echo "FAIL rc=$? $lib"; tail -5 gpurun_out/ab_bench_run.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_bench_run.log') if l.startswith('{\"metric')][-1])
print('$lib', d['roofline']['kernel_ms'], d['pipeline']['gpu_ms_per_call'], d['pipeline']['frac'], flush=True)"
  done
done
