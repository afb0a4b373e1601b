#!/bin/bash
# Diagnostic: resident pipeline time with parts of the work removed (results invalid).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for a in ${ABL:-0 128 256 512 1024 768}; do
  SVX_ABLATE=$a timeout -k 10 120 python tools/sweep.py --reps 5 --k1 1:1 --modes resident 2>&1 | grep mode | sed "s/^/ablate=$a /"
  rc=${PIPESTATUS[0]}; case $rc in 0|1) ;; *) exit $rc;; esac
done
