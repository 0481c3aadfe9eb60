# Round 5: per-rank compute of the sharded apply (virtual shards on one GPU), with the
# size-based inverse load policy (a world-8 rank's 76 MB of inverses now default-policy).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5t; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 600 python -u scripts/dev/shard_rank_time.py 1M+contacts 1,2,4,8 > $O/rank_1M.json 2> $O/rank_1M.err || { tail -5 $O/rank_1M.err; exit 1; }
cat $O/rank_1M.json
timeout -k 10 600 python -u scripts/dev/shard_rank_time.py 4M-tet 1,8 > $O/rank_4M.json 2> $O/rank_4M.err || { tail -5 $O/rank_4M.err; exit 1; }
cat $O/rank_4M.json
