# Round 6: kernel traces of one world-8 rank's one-call sharded apply in mode 1 (collective + coarse on the comm
# stream) and mode 0 (inline).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6g}; mkdir -p $O; export TMPDIR=/tmp
cd /tmp && \
MAS_SHARD_MODE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_mode1 -o run --output-format csv -- python3 $R/scripts/dev/shard_rank_time.py 1M+contacts 8 one_call > $O/tr_mode1.log 2>&1 && \
MAS_SHARD_MODE=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_mode0 -o run --output-format csv -- python3 $R/scripts/dev/shard_rank_time.py 1M+contacts 8 one_call > $O/tr_mode0.log 2>&1 && \
cd $R && python3 scripts/dev/prepare_timeline.py $O/tr_mode1 k_restrict_seg k_prolong > $O/timeline_mode1.txt 2>&1 && \
python3 scripts/dev/prepare_timeline.py $O/tr_mode0 k_restrict_seg k_solve_fine > $O/timeline_mode0.txt 2>&1
rc=$?
echo "exit $rc"
exit $rc
