set -o pipefail
export SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so TMPDIR=/tmp
for sp in 1 0; do
  SVX_RANSAC_SPEC=$sp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rs$sp -o run -- python3 tools/_probe_ransac.py || exit $?
  f=$(find gpurun_out/prof_rs$sp -name "*kernel_stats.csv" | head -1); echo "== SPEC=$sp"; cut -d, -f1-8 "$f" | head -12
done
