#!/bin/bash
# session 24: the frame loop's road pass on a stream of its own per slot (the next batch of the slot starts its
# pre-pass and maskpoints beside it, the evaluation then runs alone): the loop tests (release library), the whole
# GPU suite, then the loop probe alternating SVX_LOOP_ROAD_SPLIT=0 (road on the slot's stream) and the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s24"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -5 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
export SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
for r in 1 2 3 4; do
  for v in joined split; do
    if [ $v = joined ]; then export SVX_LOOP_ROAD_SPLIT=0; else unset SVX_LOOP_ROAD_SPLIT; fi
    PROBE_ONLY=caller2 timeout -k 10 180 python3 -u tools/_probe_loop.py > "$OUT/loop_${v}_$r.txt" 2>&1 \
      || { echo "loop probe $v $r failed"; tail -5 "$OUT/loop_${v}_$r.txt"; exit 1; }
    echo "$v $r: $(head -1 "$OUT/loop_${v}_$r.txt")"
  done
done
echo "session done"
