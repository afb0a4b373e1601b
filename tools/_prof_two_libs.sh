#!/bin/bash
# kernel stats of the SGBM workload under two libsvx builds (same box): LIBS="a.so b.so"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
i=0
for lib in $LIBS; do
  i=$((i+1))
  SVX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_two_$i -o run -- python3 tools/prof.py workload --what ${WHAT:-sgbm} --frames ${FRAMES:-128} --reps 3 > gpurun_out/prof_two_$i.log 2>&1 || exit $?
  echo "== $lib"
  python3 - "$i" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_two_{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(f'{r["Name"][:70]:72s} {r["Calls"]:>4s} {float(r["AverageNs"]) / 1e3:9.1f} us')
PY
done
