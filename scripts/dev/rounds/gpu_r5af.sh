# Round 5: kernel trace of a world-8 rank's Prepare (1M + contacts), the side fold on.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5af; mkdir -p $O; export TMPDIR=/tmp
cd /tmp && PREP_SHARD=3,8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/trace.log 2>&1 && \
python3 $R/scripts/dev/prepare_timeline.py $O/trace k_stencil_flags k_factor_rb > $O/timeline.txt 2>&1
echo "exit $?"
