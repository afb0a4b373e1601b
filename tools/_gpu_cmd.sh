# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ransac_batch.py tests/test_gpu_loop.py tests/test_gpu_digests.py > $OUT/pytest_ransac.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_ransac.log; exit 1; }
tail -1 $OUT/pytest_ransac.log
PROBE_LOOP_PIPE=1 timeout -k 10 300 python3 -u tools/_probe_pipe_beside_draw.py > $OUT/probe_loop_pipe_beside_draw.txt 2>&1 || exit 1; cat $OUT/probe_loop_pipe_beside_draw.txt
D=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
for r in 1 2; do for a in 1 0; do
  echo "== SVX_RANSAC_BOUND=$a (round $r)" >> $OUT/ab_loop_bound.txt
  SVX_LIB=$D SVX_RANSAC_BOUND=$a PROBE_BATCHES=18 PROBE_ONLY=caller2 timeout -k 10 200 python3 -u tools/_probe_loop.py >> $OUT/ab_loop_bound.txt 2>&1 || { echo "loop $a failed"; tail $OUT/ab_loop_bound.txt; exit 1; }
done; done
grep "==\|ms/batch\|batch 1[67]" $OUT/ab_loop_bound.txt
