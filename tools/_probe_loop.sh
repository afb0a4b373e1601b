set -o pipefail
export SVX_LIB=$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so
for v in "1 1" "0 1" "1 0" "0 0"; do
  set -- $v
  echo "== SVX_RANSAC_PRIO=$1 SVX_LOOP_RSTREAM=$2"
  SVX_RANSAC_PRIO=$1 SVX_LOOP_RSTREAM=$2 timeout -k 10 200 python -u tools/_probe_loop.py || exit $?
done
