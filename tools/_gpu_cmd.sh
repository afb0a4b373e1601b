# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
D=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
for r in 1 2 3; do for a in 0 131072; do
  echo "== SVX_ABLATE=$a (round $r)" >> $OUT/ab_loop_pipe_prio.txt
  SVX_LIB=$D SVX_ABLATE=$a PROBE_ONLY=caller2 timeout -k 10 200 python3 -u tools/_probe_loop.py >> $OUT/ab_loop_pipe_prio.txt 2>&1 || { echo "loop $a failed"; tail $OUT/ab_loop_pipe_prio.txt; exit 1; }
done; done
grep "==\|ms/batch\|batch 4" $OUT/ab_loop_pipe_prio.txt
