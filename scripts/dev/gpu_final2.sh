# round-3 evidence, part 2: per-config bench lines, per-rank sharded apply times, early-od A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-final2}; mkdir -p $O; export TMPDIR=/tmp; cd $R
for c in 256k 4M-tet 10k; do
  timeout -k 10 300 python bench.py --config $c --no-pcg --cpu-steps 3 > $O/$c.json 2> $O/$c.err || exit $?
done
timeout -k 10 300 python scripts/ab_prepare.py "MAS_EARLY_OD=0" "MAS_EARLY_OD=1" --config 1M+contacts --rounds 5 > $O/ab_earlyod.json 2>&1 && \
timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 1,2,4,8 > $O/rt_1M.log 2>&1 && \
timeout -k 10 300 python scripts/dev/shard_rank_time.py 4M-tet 1,8 > $O/rt_4M.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rtrace -o run --output-format csv -- python3 $R/scripts/dev/shard_rank_time.py 1M+contacts 8 > $O/rt_trace.log 2>&1
rc=$?; grep -v amdgpu $O/ab_earlyod.json $O/rt_1M.log $O/rt_4M.log | tail -60; echo "exit $rc"; exit $rc
