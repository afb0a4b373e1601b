#!/bin/bash
# round-5 session 11: pipeline variants: libsvx_h1.so (committed: atomics with return), libsvx_r.so (the count
# read before a no-return add), libsvx.so (that + pass-2 stores from an SGPR base), libsvx_p.so (that + two colours
# a lane in packed fp32): parity, then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s11"; mkdir -p "$OUT"
L=stereo.vision_amd/svx/_lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_anywidth.py tests/test_gpu_loop.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
SVX_LIB=$PWD/$L/libsvx_p.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_pairs.log" 2>&1 || { echo "pytest pairs failed"; tail -30 "$OUT/pytest_pairs.log"; exit 1; }
tail -1 "$OUT/pytest_pairs.log"
timeout -k 10 700 python3 -u tools/prof.py ab-lib --libs $L/libsvx_h1.so,$L/libsvx_r.so,$L/libsvx.so,$L/libsvx_p.so --what pipe,planes --frames 4096 --reps 5 --rounds 4 > "$OUT/ab_binning.txt" 2>&1 || { echo "ab failed"; tail "$OUT/ab_binning.txt"; exit 1; }
tail -4 "$OUT/ab_binning.txt"
