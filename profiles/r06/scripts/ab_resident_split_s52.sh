# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
export SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
timeout -k 10 300 python3 -u tools/prof.py ab --modes resident --ablate 0 --env SVX_RES_SPLIT=0,1,2,3,4,5 --what pipe --rounds 6 --reps 10 > $OUT/ab_split_pipe.txt 2>&1 || { echo "ab pipe failed"; tail $OUT/ab_split_pipe.txt; exit 1; }
cat $OUT/ab_split_pipe.txt
SVX_RES_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_split -o run -- python3 -u tools/prof.py workload --what pipe --frames 4096 --reps 5 > $OUT/prof_split.txt 2>&1 || { echo "prof failed"; tail $OUT/prof_split.txt; exit 1; }
python3 - "$OUT/prof_split" <<'PY'
import csv, glob, sys
f = sorted(glob.glob(f"{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True))[-1]
for r in csv.DictReader(open(f)):
    print(f'  {r["Name"][:70]:72s} {r["Calls"]:>4s} {float(r["AverageNs"]) / 1e3:9.1f} us')
PY
