#!/bin/bash
# Named GPU-box steps for one gpurun call: tools/gpu_steps.sh TAG step [step ...]
#   tests    the GPU suite + smoke          bench   the default bench under rocprofv3 --kernel-trace --stats
#   ablate   tools/gpu_ransac_ablate_check  pmc     PMC HBM traffic of K1 / pipeline / per-frame planes
#   ab_fill  fill_prev one-wave vs loader/writer split (SVX_FILL_SPLIT, diagnostic build, child processes)
#   ab_pipe  the resident pipeline, SVX_ABLATE / env A/B (ARGS_AB_PIPE)
#   loop     tools/_probe_loop.py timelines (PROBE_ONLY=caller2,caller1)
#   ransac1  one frame of the batched RANSAC under rocprofv3 (a single draw wave's duration)
# Every GPU step has its own time limit; the first failing step ends the script (no retries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="$1"; shift
OUT="$PWD/gpurun_out/$TAG"; mkdir -p "$OUT"; export TMPDIR=/tmp
ok() { case "$1" in 0) ;; *) echo "FATAL rc=$1 in $2"; exit "$1";; esac; }
for step in "$@"; do
  case "$step" in
  tests)
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; ok $rc pytest
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; ok $rc smoke ;;
  bench)
    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
    rc=$?; echo "bench rc=$rc"; tail -c 400 "$OUT/bench.json"; ok $rc bench ;;
  ablate)
    TAG=$TAG bash tools/gpu_ransac_ablate_check.sh; ok $? ablate ;;
  pmc)
    for w in k1:3 pipe:1 planes:1; do
      timeout -k 10 300 python3 -u tools/prof.py pmc --groups "FETCH_SIZE;WRITE_SIZE" --out "$OUT/pmc_${w%%:*}" \
        --traffic 4096 -- --what "${w%%:*}" --frames 4096 --reps "${w##*:}" > "$OUT/pmc_${w%%:*}.log" 2>&1
      rc=$?; echo "pmc ${w%%:*} rc=$rc"; ok $rc "pmc ${w%%:*}"
    done ;;
  ab_fill)
    timeout -k 10 600 python3 -u tools/prof.py ab-lib --envs "${FILL_ENVS:-SVX_FILL_SPLIT=0;SVX_FILL_SPLIT=16;SVX_FILL_SPLIT=32;SVX_FILL_SPLIT=8}" \
      --what prepass --rounds 3 --reps 5 > "$OUT/ab_fill.txt" 2>&1; rc=$?; echo "ab_fill rc=$rc"; grep variant "$OUT/ab_fill.txt"; ok $rc ab_fill ;;
  ab_libs)   # release-flavoured variant libraries (make -C stereo.vision_amd/csrc ab NAME=..), alternating processes
    timeout -k 10 900 python3 -u tools/prof.py ab-lib --libs "$AB_LIBS" --what "${AB_WHAT:-pipe,planes}" \
      --rounds "${AB_ROUNDS:-4}" --reps 5 > "$OUT/ab_libs.txt" 2>&1; rc=$?; echo "ab_libs rc=$rc"
    grep variant "$OUT/ab_libs.txt"; ok $rc ab_libs ;;
  ab_pipe)
    timeout -k 10 600 python3 -u tools/prof.py ab ${ARGS_AB_PIPE:---ablate 0} > "$OUT/ab_pipe.txt" 2>&1; rc=$?
    echo "ab_pipe rc=$rc"; cat "$OUT/ab_pipe.txt" | tail -8; ok $rc ab_pipe ;;
  ab_loop)   # the frame loop's timelines, one process per variant (LOOP_ENVS, ';'-separated), alternating twice
    IFS=';' read -ra VARS <<< "${LOOP_ENVS:-SVX_FILL_SPLIT=0;SVX_FILL_SPLIT=16}"
    for r in 1 2; do for v in "${VARS[@]}"; do
      echo "== $v (round $r)" >> "$OUT/ab_loop.txt"
      env $v SVX_LIB="$PWD/stereo.vision_amd/svx/_lib/libsvx_diag.so" PROBE_ONLY=caller2 timeout -k 10 200 \
        python3 -u tools/_probe_loop.py >> "$OUT/ab_loop.txt" 2>&1; rc=$?; ok $rc "ab_loop $v"
    done; done
    grep -A0 "==\|ms/batch" "$OUT/ab_loop.txt" ;;
  dropin)
    timeout -k 10 200 python3 -u tools/prof.py dropin --reps 20 > "$OUT/dropin.txt" 2>&1; rc=$?
    echo "dropin rc=$rc"; cat "$OUT/dropin.txt"; ok $rc dropin ;;
  probe_ransac)
    timeout -k 10 200 python3 -u tools/_probe_ransac_dropin.py > "$OUT/probe_ransac_dropin.txt" 2>&1; rc=$?
    echo "probe_ransac rc=$rc"; cat "$OUT/probe_ransac_dropin.txt"; ok $rc probe_ransac ;;
  ab_loop_libs)   # the frame loop with each library of AB_LIBS (release builds), one process each, alternating twice
    IFS=',' read -ra LIBS <<< "$AB_LIBS"
    for r in 1 2; do for l in "${LIBS[@]}"; do
      echo "== $l (round $r)" >> "$OUT/ab_loop_libs.txt"
      SVX_LIB="$PWD/$l" PROBE_ONLY=caller2 PROBE_RANSAC=1 timeout -k 10 200 \
        python3 -u tools/_probe_loop.py >> "$OUT/ab_loop_libs.txt" 2>&1; rc=$?; ok $rc "ab_loop_libs $l"
    done; done
    grep "==\|ms/batch\|ransac alone" "$OUT/ab_loop_libs.txt" ;;
  loop)
    PROBE_ONLY=${PROBE_ONLY:-caller2,caller1} timeout -k 10 400 python3 -u tools/_probe_loop.py > "$OUT/loop.txt" 2>&1
    rc=$?; echo "loop rc=$rc"; grep -v "batch" "$OUT/loop.txt" | tail -6; ok $rc loop ;;
  ransac1)
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ransac1" -o run -- \
      python3 -u tools/prof.py workload --what ransac --frames "${RANSAC_FRAMES:-1}" --reps 5 > "$OUT/ransac1.log" 2>&1
    rc=$?; echo "ransac1 rc=$rc"; ok $rc ransac1
    python3 - "$OUT/ransac1" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
    print(f'{r["Name"][:60]:62s} {r["Calls"]:>4s} {float(r["AverageNs"]) / 1e3:9.1f} us')
PY
    ;;
  *) echo "unknown step $step"; exit 2;;
  esac
done
echo "steps done"
