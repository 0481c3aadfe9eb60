set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ranktime}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 1,2,4,8 > $O/rt.log 2>&1 || { tail $O/rt.log; exit 1; }
grep -v amdgpu $O/rt.log | tail -20
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/shard_rank_time.py 1M+contacts 8 > $O/rt2.log 2>&1
echo "exit $?"
