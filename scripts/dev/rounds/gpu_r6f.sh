# Round 6: inline one-call sharded apply (all stream forms bitwise), its per-rank time, PCG grid A/B (1024 vs 768).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6f}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_facade.py tests/test_gpu_pcg.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 8 fine_then_complete,one_call > $O/rt_mode0.txt 2>&1 && \
for i in 1 2; do \
  timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_b1024_$i.txt 2>&1 && \
  MAS_LIB_NAME=libmas_amd_ab_pcg768.so timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_b768_$i.txt 2>&1 || exit 1; \
done
rc=$?
tail -2 $O/pytest.log
echo "exit $rc"
exit $rc
