# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ransac_batch.py tests/test_gpu_loop.py tests/test_gpu_digests.py tests/test_gpu_ransac.py > $OUT/pytest_ransac.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_ransac.log; exit 1; }
tail -1 $OUT/pytest_ransac.log
for r in 1 2; do for L in stereo.vision_amd/svx/_lib/libsvx_diag.so _ab/libsvx_drawold.so _ab/libsvx_drawwpe5.so; do
  echo "== $L (round $r)" >> $OUT/ab_loop_draw_staged.txt
  SVX_LIB=$PWD/$L PROBE_ONLY=caller2 PROBE_RANSAC=1 timeout -k 10 200 python3 -u tools/_probe_loop.py >> $OUT/ab_loop_draw_staged.txt 2>&1 || { echo "loop $L failed"; tail $OUT/ab_loop_draw_staged.txt; exit 1; }
done; done
grep "==\|ms/batch\|alone\|batch 4" $OUT/ab_loop_draw_staged.txt
