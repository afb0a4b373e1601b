#!/bin/bash
# session 21: with the evaluation at 96 VGPRs (session 19), does it now pay to start batch k's evaluation right after
# batch k-1's pipeline (beside its road pass) instead of after that road pass? Diagnostic build, alternating
# processes (SVX_LOOP_EVAL_AFTER=pipeline vs the default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s21"
mkdir -p "$OUT"
export TMPDIR=/tmp
export SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
for r in 1 2 3 4; do
  for v in road pipeline; do
    if [ $v = pipeline ]; then E=pipeline; else E=; fi
    SVX_LOOP_EVAL_AFTER=$E PROBE_ONLY=caller2 timeout -k 10 180 python3 -u tools/_probe_loop.py > "$OUT/loop_${v}_$r.txt" 2>&1 \
      || { echo "loop probe $v $r failed"; tail -5 "$OUT/loop_${v}_$r.txt"; exit 1; }
    echo "eval after $v $r: $(head -1 "$OUT/loop_${v}_$r.txt")"
  done
done
echo "session done"
