# Round 6: the sharded coarse assembly -- shard tests (bitwise blocks / inverses / z), per-rank Prepare, per-rank apply.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6b}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_shard_cpp.py tests/test_gpu_shard_locality.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/dev/prep_shard.py 1M+contacts 8 3 > $O/prep_shard_1M.txt 2>&1 && \
timeout -k 10 400 python scripts/dev/prep_shard.py 4M-tet 8 3 > $O/prep_shard_4M.txt 2>&1 && \
timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 8 fine_then_complete,one_call > $O/rank_time_1M.txt 2>&1
rc=$?
tail -3 $O/pytest.log
echo "exit $rc"
exit $rc
