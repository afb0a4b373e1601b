mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_digests.py -v --timeout 300 --timeout-method thread > gpurun_out/pyt_digests.log 2>&1; rc=$?; echo "digests rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pyt_digests.log | head -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -u -m pytest tests/test_gpu_ransac_batch.py tests/test_gpu_anywidth.py tests/test_gpu_parity.py tests/test_gpu_prepass.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pyt_slots.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pyt_slots.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -u tools/prof.py ab --ablate 0,2048 --what pipe --rounds 6 --with-k1 > gpurun_out/ab_slots_pipe.log 2>&1; rc=$?; cat gpurun_out/ab_slots_pipe.log; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u tools/prof.py ab --ablate 0,2048 --what planes --rounds 6 > gpurun_out/ab_slots_planes.log 2>&1; rc=$?; cat gpurun_out/ab_slots_planes.log; exit $rc
