# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ransac_batch.py tests/test_gpu_loop.py tests/test_gpu_digests.py > $OUT/pytest_ransac.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_ransac.log; exit 1; }
tail -1 $OUT/pytest_ransac.log
for r in 1 2 3; do for L in stereo.vision_amd/svx/_lib/libsvx_diag.so _ab/libsvx_mpold.so; do
  echo "== $L (round $r)" >> $OUT/ab_maskpoints.txt
  SVX_LIB=$PWD/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$r_$(basename $L .so) -o run -- python3 -u tools/prof.py workload --what ransac --frames 4096 --reps 10 >> $OUT/ab_maskpoints.txt 2>&1 || { echo "$L failed"; tail $OUT/ab_maskpoints.txt; exit 1; }
  python3 - "$OUT/prof_$r_$(basename $L .so)" >> $OUT/ab_maskpoints.txt <<'PY'
import csv, glob, sys
f = sorted(glob.glob(f"{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True))[-1]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("maskpoints_kernel", "ransac_draw", "ransac_eval")):
        print(f'  {r["Name"][:50]:52s} {r["Calls"]:>4s} {float(r["AverageNs"]) / 1e3:9.1f} us')
PY
done; done
grep "==\|  " $OUT/ab_maskpoints.txt | grep -v "^\s*$"
