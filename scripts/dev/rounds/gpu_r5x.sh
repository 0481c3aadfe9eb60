# Round 5: Prepare kernel trace on the current code (which path ends last after the formation rewrite).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5x; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/noprof.log 2>&1 && \
PREP_SHARD=3,8 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/noprof_rank3of8.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/trace.log 2>&1 && \
python3 $R/scripts/dev/prepare_timeline.py $O/trace k_stencil_flags k_factor_rb > $O/timeline.txt 2>&1
echo "exit $?"
