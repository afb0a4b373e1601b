#!/bin/bash
# session 17: the GPU suite on the library with the bound-checked row gathers, then PMC counters of the batched
# RANSAC kernels (maskpoints, draw, eval) at 4096 frames: where the draw's chain spends its cycles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s17"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -5 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python3 -u tools/prof.py pmc \
  --groups "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT;GRBM_GUI_ACTIVE SQ_WAVES" \
  --out "$OUT/pmc_ransac" -- --what ransac --frames 4096 --reps 2 > "$OUT/pmc_ransac.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -60 "$OUT/pmc_ransac.log"
exit $rc
