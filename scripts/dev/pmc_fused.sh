# PMC passes over the fused level-0 assemble + factor kernel (default: matrix-core formation),
# one steady-state Prepare each: bash scripts/dev/pmc_fused.sh <out>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmc_fused}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
K=k_factor_fused
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES -d $O/p1 -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 2 > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM -d $O/p2 -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 2 > $O/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc FETCH_SIZE -d $O/p3 -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 2 > $O/p3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc WRITE_SIZE -d $O/p4 -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 2 > $O/p4.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/trace.log 2>&1
echo "exit $?"
