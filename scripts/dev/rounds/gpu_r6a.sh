# Round 6: sharded apply with the coarse levels on the comm stream; odd-nV PCG; per-rank timing.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6a}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_pcg.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 1,8 fine_then_complete,one_call > $O/rank_time_1M.txt 2>&1 && \
timeout -k 10 300 python scripts/dev/shard_rank_time.py 4M-tet 8 fine_then_complete,one_call > $O/rank_time_4M.txt 2>&1
rc=$?
tail -3 $O/pytest.log
echo "exit $rc"
exit $rc
