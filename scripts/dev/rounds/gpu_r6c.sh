# Round 6: one-call sharded apply A/B (coarse on the comm stream vs on the apply stream; HW queues), rank Prepare
# with the pre level-1 factor beside the table folds, and its kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6c}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/dev/prep_shard.py 1M+contacts 8 3 > $O/prep_shard_1M.txt 2>&1 && \
timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 8 fine_then_complete,one_call > $O/rt_side1.txt 2>&1 && \
MAS_SHARD_COARSE_SIDE=0 timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 8 one_call > $O/rt_side0.txt 2>&1 && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 8 fine_then_complete,one_call > $O/rt_side1_q8.txt 2>&1 && \
cd /tmp && PREP_SHARD=3,8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prep_rank3 -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/prep_rank3.log 2>&1 && \
cd $R && python3 scripts/dev/prepare_timeline.py $O/prep_rank3 k_stencil_flags k_rows_copy > $O/timeline_rank3.txt 2>&1
rc=$?
tail -2 $O/pytest.log
echo "exit $rc"
exit $rc
