#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, --pmc never combined with
# tracing domains) over tools/prof_workload.py. Output: gpurun_out/pmc/<pass>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/pmc"; mkdir -p "$OUT"
export TMPDIR=/tmp
WL="${WL:---what k1,pipe --frames 1024 --reps 2}"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 tools/prof_workload.py $WL > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  case $rc in 0|1) ;; *) echo "FATAL rc=$rc"; exit $rc;; esac
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE}
GROUPS
