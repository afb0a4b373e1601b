# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
SVX_LIB=$PWD/_ab/libsvx_pk3.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ransac_batch.py tests/test_gpu_loop.py tests/test_gpu_digests.py > $OUT/pytest_ransac_pk3.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_ransac_pk3.log; exit 1; }
tail -1 $OUT/pytest_ransac_pk3.log
for r in 1 2; do for L in _ab/libsvx_pk3.so _ab/libsvx_pk5.so _ab/libsvx_pk0.so; do
  echo "== $L (round $r)" >> $OUT/ab_eval_screen_pk.txt
  SVX_LIB=$PWD/$L timeout -k 10 200 python3 -u tools/_probe_eval_phases.py >> $OUT/ab_eval_screen_pk.txt 2>&1 || { echo "$L failed"; tail $OUT/ab_eval_screen_pk.txt; exit 1; }
done; done
grep "==\|screen\|candidates\|per call" $OUT/ab_eval_screen_pk.txt
