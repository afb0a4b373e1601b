cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/pmcabl
for ab in ${ABL:-0 128 256 512}; do
  SVX_ABLATE=$ab timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcabl/a$ab -o run -- python3 tools/prof_workload.py --what pipe --frames 4096 --reps 1 > gpurun_out/pmcabl/a$ab.log 2>&1
  rc=$?; echo "ablate $ab rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
  python3 tools/pmc_summary.py gpurun_out/pmcabl/a$ab | grep -A9 resident_fused
done
