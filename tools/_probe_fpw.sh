#!/bin/bash
# frame-loop A/B of the draw's frames per wave (SVX_DRAW_FPW, diagnostic build), loop parity tests first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
SVX_DRAW_FPW=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_loop.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_loop_fpw2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_loop_fpw2.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do for f in ${FPWS:-1 2 3}; do
  echo "== FPW=$f"; PROBE_ONLY=caller2 SVX_DRAW_FPW=$f timeout -k 10 300 python -u tools/_probe_loop.py > gpurun_out/fpw.txt 2>&1 || { cat gpurun_out/fpw.txt; exit 1; }; cat gpurun_out/fpw.txt
done; done
