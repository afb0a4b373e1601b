#!/bin/bash
# round-5 session 8: road rows a wave (diagnostic SVX_ROAD_RPW, one process alternating) and the pipeline's write
# pattern as four planes vs one plane of 16-byte records (tools/sol_pipe.hip r05 modes 8, 9)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s8"; mkdir -p "$OUT"; export TMPDIR=/tmp
L=stereo.vision_amd/svx/_lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_loop.py tests/test_gpu_digests.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_loop.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_loop.log"; exit 1; }
tail -1 "$OUT/pytest_loop.log"
SVX_LIB=$PWD/$L/libsvx_diag.so PROBE_RPW=1,2,4 timeout -k 10 300 python3 -u tools/_probe_road.py > "$OUT/probe_road_rpw.txt" 2>&1 || { echo "road probe failed"; tail "$OUT/probe_road_rpw.txt"; exit 1; }
cat "$OUT/probe_road_rpw.txt"
timeout -k 10 120 ./tools/_sol_pipe r05 4096 277200 50 5 > "$OUT/sol_pipe_aos.txt" 2>&1 || { echo "sol_pipe failed"; tail "$OUT/sol_pipe_aos.txt"; exit 1; }
grep '"round": 1' "$OUT/sol_pipe_aos.txt"
