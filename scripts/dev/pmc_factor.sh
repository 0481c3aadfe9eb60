# PMC passes over the factor kernel: bash scripts/dev/pmc_factor.sh <out>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmc_factor}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp

timeout -s KILL 120 rocprofv3 --kernel-include-regex k_factor_rb --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY -d $O/p1 -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py > $O/p1.log 2>&1
echo "p1 $?"
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_factor_rb --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_IFETCH -d $O/p2 -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py > $O/p2.log 2>&1
echo "p2 $?"
