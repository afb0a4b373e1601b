#!/bin/bash
# session 31: the draw kernel advancing the next twist level while the triple's packed words are in flight
# : the RANSAC and loop tests on the release library, then A/B against HEAD (libsvx_diag_base.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s31"
mkdir -p "$OUT"
export TMPDIR=/tmp
LIB=stereo.vision_amd/svx/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_ransac_batch.py tests/test_gpu_loop.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_ransac_loop.log" 2>&1 || { echo "pytest failed"; tail -5 "$OUT/pytest_ransac_loop.log"; exit 1; }
tail -1 "$OUT/pytest_ransac_loop.log"
for r in 1 2 3 4; do
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
echo "session done"
