#!/bin/bash
# the RANSAC ablation that faulted in round 5 (SVX_RANSAC_ABLATE=72: bit 8 plus the
# undocumented bit 64) must now be refused by the library, and the documented bit 8 must run clean.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/${TAG:-s}"; mkdir -p "$OUT"; export TMPDIR=/tmp
SVX_RANSAC_ABLATE=72 timeout -k 10 120 python3 -u tools/prof.py workload --what ransac --frames 4096 --reps 1 \
  > "$OUT/ablate72.log" 2>&1; rc=$?
echo "ablate 72 rc=$rc (expect 1: refused)"; tail -1 "$OUT/ablate72.log"
case $rc in 1) ;; *) exit 3;; esac
SVX_RANSAC_ABLATE=8 timeout -k 10 120 python3 -u tools/prof.py workload --what ransac --frames 4096 --reps 2 \
  > "$OUT/ablate8.log" 2>&1; rc=$?
echo "ablate 8 rc=$rc"; tail -1 "$OUT/ablate8.log"; exit $rc
