#!/bin/bash
# session 18: the GPU suite on the DPP wave sums (the RANSAC screen's fp64 sums, the integer wave_sum, SGBM's
# speckle counts), then A/B of the previous library (libsvx_diag_base.so) against this one, alternating processes:
# the frame loop (two slots), the batched RANSAC, the pipeline and per-frame planes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s18"
mkdir -p "$OUT"
export TMPDIR=/tmp
LIB=stereo.vision_amd/svx/_lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -5 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for r in 1 2 3; do
  for v in base new; do
    [ $v = base ] && L=$LIB/libsvx_diag_base.so || L=$LIB/libsvx_diag.so
    SVX_LIB=$PWD/$L PROBE_ONLY=caller2 timeout -k 10 180 python3 -u tools/_probe_loop.py > "$OUT/loop_${v}_$r.txt" 2>&1 \
      || { echo "loop probe $v $r failed"; tail -5 "$OUT/loop_${v}_$r.txt"; exit 1; }
    echo "loop $v $r: $(head -1 "$OUT/loop_${v}_$r.txt")"
  done
done
timeout -k 10 600 python3 -u tools/prof.py ab-lib --libs $LIB/libsvx_diag_base.so,$LIB/libsvx_diag.so \
  --what ransac --frames 4096 --rounds 4 --reps 5 > "$OUT/ab_ransac.txt" 2>&1 || { echo "ab ransac failed"; tail -5 "$OUT/ab_ransac.txt"; exit 1; }
tail -2 "$OUT/ab_ransac.txt"
timeout -k 10 600 python3 -u tools/prof.py ab-lib --libs $LIB/libsvx_diag_base.so,$LIB/libsvx_diag.so \
  --what pipe,planes --frames 4096 --rounds 3 --reps 5 > "$OUT/ab_pipe.txt" 2>&1 || { echo "ab pipe failed"; tail -5 "$OUT/ab_pipe.txt"; exit 1; }
tail -2 "$OUT/ab_pipe.txt"
echo "session done"
