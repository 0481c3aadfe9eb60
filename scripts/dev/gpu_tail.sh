set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-tail}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_shard_cpp.py -x -v --timeout 200 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 1,8 > $O/rt.log 2>&1 || { tail $O/rt.log; exit 1; }
grep -v amdgpu $O/rt.log | grep -v '^{' | tail -8
