#!/bin/bash
# session 23 (diagnostic): the draw's sample LDS capped at 848 words (n <= 27,136 points; SVX_DRAW_WORDS, diag
# build) so that a draw wave holds <= 6,144 B and two pipeline workgroups fit beside the 16 draw waves of a CU.
# First the loop tests with the cap (they pass only if no frame of the test batches exceeds it), then the loop
# probe alternating capped / default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s23"
mkdir -p "$OUT"
export TMPDIR=/tmp
export SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
SVX_DRAW_WORDS=848 timeout -k 10 300 python -u -m pytest tests/test_gpu_loop.py -m gpu -x -q --timeout 240 \
  --timeout-method thread > "$OUT/pytest_loop_capped.log" 2>&1; echo "capped loop tests rc=$?"; tail -2 "$OUT/pytest_loop_capped.log"
for r in 1 2 3 4; do
  for v in default capped; do
    if [ $v = capped ]; then export SVX_DRAW_WORDS=848; else unset SVX_DRAW_WORDS; fi
    PROBE_ONLY=caller2 timeout -k 10 180 python3 -u tools/_probe_loop.py > "$OUT/loop_${v}_$r.txt" 2>&1 \
      || { echo "loop probe $v $r failed"; tail -5 "$OUT/loop_${v}_$r.txt"; exit 1; }
    echo "$v $r: $(head -1 "$OUT/loop_${v}_$r.txt")"
  done
done
echo "session done"
