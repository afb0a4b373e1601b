# ad-hoc GPU session steps (kept with the session's records under profiles/r06/scripts when used)
set -o pipefail
OUT=gpurun_out/${SESSION:-r6sX}; mkdir -p $OUT
SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so timeout -k 10 300 python3 -u tools/prof.py ab --modes resident --ablate 0,262144 --what pipe --rounds 8 > $OUT/ab_pipe_late_prio.txt 2>&1; rc=$?; cat $OUT/ab_pipe_late_prio.txt; [ $rc -eq 0 ] || exit 1
SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so timeout -k 10 300 python3 -u tools/prof.py ab --modes resident --ablate 0,262144 --what planes --rounds 6 > $OUT/ab_planes_late_prio.txt 2>&1; rc=$?; cat $OUT/ab_planes_late_prio.txt; exit $rc
