# Round 6: issue / wait counters of the factor kernels (k_factor_fused chunks, k_factor_rb) over steady-state
# Prepares, one --pmc pass (8 SQ counters at most).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6w}; mkdir -p $O; export TMPDIR=/tmp
cd /tmp && \
PREP_DEVICE=1 timeout -s KILL 300 rocprofv3 --kernel-include-regex k_factor --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH -d $O/pmc_wait -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 2 > $O/pmc_wait.log 2>&1
rc=$?
tail -2 $O/pmc_wait.log
echo "exit $rc"
exit $rc
