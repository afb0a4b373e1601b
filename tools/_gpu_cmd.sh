# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ransac_batch.py tests/test_gpu_loop.py tests/test_gpu_digests.py tests/test_gpu_ransac.py > $OUT/pytest_ransac.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_ransac.log; exit 1; }
tail -1 $OUT/pytest_ransac.log
for r in 1 2; do
  timeout -k 10 200 python3 -u tools/_probe_eval_phases.py >> $OUT/probe_eval_phases.txt 2>&1 || { echo "probe failed"; tail $OUT/probe_eval_phases.txt; exit 1; }
done
grep -v "^workgroups" $OUT/probe_eval_phases.txt
for r in 1 2; do
  PROBE_ONLY=caller2 PROBE_RANSAC=1 timeout -k 10 200 python3 -u tools/_probe_loop.py >> $OUT/loop.txt 2>&1 || { echo "loop failed"; tail $OUT/loop.txt; exit 1; }
done
grep "ms/batch\|alone" $OUT/loop.txt
