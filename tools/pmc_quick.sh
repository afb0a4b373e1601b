#!/bin/bash
# Two PMC passes over tools/prof_mode.py (resident pipeline by default) + summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/pmcq"; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 tools/prof_mode.py ${WLARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE}
GROUPS
python3 tools/pmc_summary.py "$OUT"
