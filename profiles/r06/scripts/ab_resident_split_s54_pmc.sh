# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT; export TMPDIR=/tmp
export SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
for v in 0 5; do
  SVX_RES_SPLIT=$v timeout -k 10 300 python3 -u tools/prof.py pmc --groups "FETCH_SIZE;WRITE_SIZE;SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES" --out $OUT/pmc_split$v -- --what pipe --frames 4096 --reps 1 > $OUT/pmc_split$v.log 2>&1 || { echo "pmc $v failed"; tail -20 $OUT/pmc_split$v.log; exit 1; }
  echo "== SVX_RES_SPLIT=$v"; tail -25 $OUT/pmc_split$v.log
done
