#!/bin/bash
# session 33: PMC counters of the final batched RANSAC kernels (the draw after its instruction cuts), 4096 frames,
# one pass (compare profiles/r05/pmc_ransac_s17.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s33"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/prof.py pmc \
  --groups "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVES" \
  --out "$OUT/pmc_ransac" -- --what ransac --frames 4096 --reps 2 > "$OUT/pmc_ransac.log" 2>&1
rc=$?; echo "pmc rc=$rc"; grep -A9 "ransac_draw_kernel" "$OUT/pmc_ransac.log"
exit $rc
