# Round 4: per-rank compute of the sharded apply (allgather replaced by a
# local copy) at 1M + contacts and 4M tet, and a kernel trace at world 8.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4p}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 300 python3 scripts/dev/shard_rank_time.py 1M+contacts 1,2,4,8 > $O/rank_time_1M.log 2>&1 && \
timeout -k 10 400 python3 scripts/dev/shard_rank_time.py 4M-tet 1,8 > $O/rank_time_4M.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace8 -o run --output-format csv -- python3 $R/scripts/dev/shard_rank_time.py 1M+contacts 8 > $O/trace8.log 2>&1
echo "exit $?"
