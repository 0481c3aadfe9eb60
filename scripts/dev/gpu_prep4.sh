# Round-4 Prepare evidence: steady-state Prepare, CU-reserve sweep, one kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-prep4}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/noprof.log 2>&1 && \
timeout -k 10 300 python3 scripts/ab_prepare.py MAS_PREP_CU_RESERVE=0 MAS_PREP_CU_RESERVE=16 MAS_PREP_CU_RESERVE=32 MAS_PREP_CU_RESERVE=64 --rounds 5 > $O/ab_reserve.json 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/default -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/default.log 2>&1 && \
python3 $R/scripts/dev/prepare_timeline.py $O/default k_stencil_flags k_factor_rb > $O/timeline.txt 2>&1
echo "exit $?"
