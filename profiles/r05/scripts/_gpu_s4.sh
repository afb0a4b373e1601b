mkdir -p gpurun_out/s4
timeout -k 10 600 python -u -m pytest tests/test_gpu_ransac_batch.py tests/test_gpu_loop.py tests/test_gpu_ransac.py tests/test_gpu_digests.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s4/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/s4/pytest.log; [ $rc = 0 ] || exit $rc
for lib in new old new old; do
  if [ $lib = old ]; then export SVX_LIB=$PWD/_ab/libsvx_mtlds.so; else unset SVX_LIB; fi
  echo "== $lib"; PROBE_ONLY=caller2 PROBE_RANSAC=1 timeout -k 10 300 python3 -u tools/_probe_loop.py || exit $?
done > gpurun_out/s4/probe_loop_ab.txt 2>&1
cat gpurun_out/s4/probe_loop_ab.txt
