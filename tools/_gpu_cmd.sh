# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
timeout -k 10 300 python3 -u tools/prof.py time --what pipe --sizes 256,1280,2560,3840,4096,5120,6400,8192 --reps 10 > $OUT/pipe_sizes.txt 2>&1; rc=$?; cat $OUT/pipe_sizes.txt; exit $rc
