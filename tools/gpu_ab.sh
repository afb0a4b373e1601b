#!/bin/bash
# Pipeline-variant parity tests + in-process A/B (tools/ab.py). MODES overrides the variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-resident or baseline_size or resident_pf2}" > gpurun_out/pt_ab.log 2>&1; rc=$?; tail -15 gpurun_out/pt_ab.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab.py --modes ${MODES:-resident,resident_pf2} --ablate ${ABLATE:-0} --rounds 5 --reps 3 > gpurun_out/ab.log 2>&1; rc=$?; cat gpurun_out/ab.log; exit $rc
