#!/bin/bash
# One rocprofv3 --pmc pass per line of PMC_GROUPS over a workload command (default:
# the resident pipeline on 4096 frames + K1), then a per-kernel summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${PMC_DIR:-pmcg}"; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 tools/prof_workload.py ${WL:---what k1,pipe --frames 4096 --reps 1} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done <<< "$PMC_GROUPS"
python3 tools/pmc_summary.py "$OUT"
