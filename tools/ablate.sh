#!/bin/bash
# Diagnostic: pipeline time with parts of the work removed (results invalid).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for a in ${ABL:-0 1 2 3 4 8 12 15}; do
  SVX_ABLATE=$a timeout -k 10 120 python tools/sweep.py --reps 5 --k1 0:1 --chunks ${CHUNK:-1024} 2>&1 | grep chunk | sed "s/^/ablate=$a /"
  rc=${PIPESTATUS[0]}; case $rc in 0|1) ;; *) exit $rc;; esac
done
