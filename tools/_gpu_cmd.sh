# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ransac_batch.py -k "sample_branches" > $OUT/pytest_branches.log 2>&1; rc=$?; tail -15 $OUT/pytest_branches.log; exit $rc
