#!/bin/bash
# round-5 session 15: the frame loop's evaluation after the previous pipeline (beside its road pass) vs after the
# road pass (diagnostic build's SVX_LOOP_EVAL_AFTER), alternating processes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s15"; mkdir -p "$OUT"
L=stereo.vision_amd/svx/_lib
for i in 1 2 3; do
  for ea in road pipeline; do
    echo "== eval after $ea" >> "$OUT/loop_eval_after.txt"
    SVX_LIB=$PWD/$L/libsvx_diag.so SVX_LOOP_EVAL_AFTER=$ea PROBE_ONLY=caller2 timeout -k 10 200 python3 -u tools/_probe_loop.py >> "$OUT/loop_eval_after.txt" 2>&1 || { echo "probe failed"; tail "$OUT/loop_eval_after.txt"; exit 1; }
  done
done
grep -v "^  batch" "$OUT/loop_eval_after.txt"
