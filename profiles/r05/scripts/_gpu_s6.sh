#!/bin/bash
# round-5 session 6: deferred-return binning A/B (libsvx_base.so = committed sources) + pipeline parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s6"; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_anywidth.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -20 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 500 python3 -u tools/prof.py ab-lib --libs stereo.vision_amd/svx/_lib/libsvx_base.so,stereo.vision_amd/svx/_lib/libsvx.so --what pipe,planes --frames 4096 --reps 5 --rounds 6 > "$OUT/ab.log" 2>&1 || { echo "ab failed"; tail -20 "$OUT/ab.log"; exit 1; }
tail -2 "$OUT/ab.log"
