# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
D=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
for r in 1 2; do for a in road none pipeline; do
  echo "== SVX_LOOP_EVAL_AFTER=$a (round $r)" >> $OUT/ab_loop_eval_after_18.txt
  SVX_LIB=$D SVX_LOOP_EVAL_AFTER=$a PROBE_BATCHES=18 PROBE_ONLY=caller2 timeout -k 10 200 python3 -u tools/_probe_loop.py >> $OUT/ab_loop_eval_after_18.txt 2>&1 || { echo "loop $a failed"; tail $OUT/ab_loop_eval_after_18.txt; exit 1; }
done; done
grep "==\|ms/batch\|batch 16" $OUT/ab_loop_eval_after_18.txt
