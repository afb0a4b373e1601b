#!/bin/bash
# round-5 session 10d (with the candidate table): the pipeline's dirty-chunk pass-2 work (diagnostic build, in-process alternation):
# 0 full, 16 no chunk re-binned in pass 2, 64 binning adds without returns (no candidates), 2 no binning
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out/s10d"; mkdir -p "$OUT"
L=stereo.vision_amd/svx/_lib
SVX_LIB=$PWD/$L/libsvx_diag.so timeout -k 10 400 python3 -u tools/prof.py ab --what pipe --frames 4096 --ablate 0,16,64,2 --with-k1 --rounds 5 --reps 5 > "$OUT/ab_pipe_dirty.txt" 2>&1 || { echo "ab failed"; tail "$OUT/ab_pipe_dirty.txt"; exit 1; }
cat "$OUT/ab_pipe_dirty.txt"
