#!/bin/bash
# round-5 session 12: low-bin points dropped from the keep bits via pass 1's candidate table (libsvx.so) vs the candidate-chunk re-binning
# (libsvx_h1.so): pipeline parity, then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s12"; mkdir -p "$OUT"
L=stereo.vision_amd/svx/_lib
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_anywidth.py tests/test_gpu_loop.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 600 python3 -u tools/prof.py ab-lib --libs $L/libsvx_h1.so,$L/libsvx.so --what pipe,planes --frames 4096 --reps 5 --rounds 6 > "$OUT/ab_exact_dirty.txt" 2>&1 || { echo "ab failed"; tail "$OUT/ab_exact_dirty.txt"; exit 1; }
tail -2 "$OUT/ab_exact_dirty.txt"
