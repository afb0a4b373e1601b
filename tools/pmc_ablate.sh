#!/bin/bash
# One PMC pass per SVX_ABLATE value over tools/prof_mode.py (instruction mix per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/pmcab"; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
CNT="${CNT:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE}"
for ab in ${ABL:-0 128 256}; do
  SVX_ABLATE=$ab timeout -k 10 300 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/a$ab" -o run -- python3 tools/prof_mode.py ${WLARGS:-} > "$OUT/a$ab.log" 2>&1
  rc=$?; echo "ablate $ab rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
  echo "== ablate $ab"; python3 tools/pmc_summary.py "$OUT/a$ab" 2>/dev/null | grep -A12 "${KFILTER:-resident}"
done
