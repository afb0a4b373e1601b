# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ransac_batch.py tests/test_gpu_loop.py tests/test_gpu_digests.py > $OUT/pytest_ransac.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_ransac.log; exit 1; }
tail -1 $OUT/pytest_ransac.log
for r in 1 2 3; do for L in stereo.vision_amd/svx/_lib/libsvx_diag.so _ab/libsvx_qb0.so; do
  echo "== $L (round $r)" >> $OUT/ab_eval_screen_qbound.txt
  SVX_LIB=$PWD/$L timeout -k 10 200 python3 -u tools/_probe_eval_phases.py >> $OUT/ab_eval_screen_qbound.txt 2>&1 || { echo "$L failed"; tail $OUT/ab_eval_screen_qbound.txt; exit 1; }
done; done
grep "==\|screen\|candidates\|per call" $OUT/ab_eval_screen_qbound.txt
