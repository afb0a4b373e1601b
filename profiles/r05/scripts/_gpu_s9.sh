#!/bin/bash
# round-5 session 9: the pipeline probe's mode 10 (next read before the writes, the writes left outstanding)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s9"; mkdir -p "$OUT"
timeout -k 10 120 ./tools/_sol_pipe r05 4096 277200 50 5 > "$OUT/sol_pipe_vmcnt.txt" 2>&1 || { echo "sol_pipe failed"; tail "$OUT/sol_pipe_vmcnt.txt"; exit 1; }
grep '"round": 1' "$OUT/sol_pipe_vmcnt.txt"
