#!/bin/bash
# Full round-end evidence run: tests, bench, rocprofv3 kernel-trace stats of the
# bench command, PMC traffic of K1 + the pipeline at the bench workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="$PWD/gpurun_out"; mkdir -p "$OUT"
SKIP_PROF=0 bash tools/gpu_check.sh || exit $?
python3 tools/prof.py dispatches "$OUT/prof" --kernel resident_fused > "$OUT/resident_dispatches.json" || exit $?
python3 tools/prof.py pmc --groups "FETCH_SIZE;WRITE_SIZE" --out "$OUT/pmc_k1" --traffic 4096 -- --what k1 --frames 4096 --reps 3 || exit $?
python3 tools/prof.py pmc --groups "FETCH_SIZE;WRITE_SIZE" --out "$OUT/pmc_pipe" --traffic 4096 -- --what pipe --frames 4096 --reps 1 || exit $?
python3 tools/prof.py pmc --groups "FETCH_SIZE;WRITE_SIZE" --out "$OUT/pmc_planes" --traffic 4096 -- --what planes --frames 4096 --reps 1 || exit $?
cat "$OUT/pmc_k1/traffic.json" "$OUT/pmc_pipe/traffic.json" "$OUT/pmc_planes/traffic.json"
# HBM bytes per kernel of the SGBM stage (128 frames, one chunk) and of the batched RANSAC (4096 frames)
python3 tools/prof.py pmc --groups "FETCH_SIZE;WRITE_SIZE" --out "$OUT/pmc_sgbm" -- --what sgbm --frames 128 --reps 1 > "$OUT/pmc_sgbm.txt" || exit $?
python3 tools/prof.py pmc --groups "FETCH_SIZE;WRITE_SIZE" --out "$OUT/pmc_ransac" -- --what ransac --frames 4096 --reps 1 > "$OUT/pmc_ransac.txt" || exit $?
