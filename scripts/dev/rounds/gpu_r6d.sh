# Round 6: full GPU suite on the pipelined folds / few-node table folds / SpMV occupancy; rank Prepare; sharded
# apply modes; PCG SpMV occupancy A/B; long-run step A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6d}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python scripts/dev/prep_shard.py 1M+contacts 8 3 > $O/prep_shard_1M.txt 2>&1 && \
MAS_LIB_NAME=libmas_amd_ab_ls128.so timeout -k 10 300 python scripts/dev/prep_shard.py 1M+contacts 8 3 > $O/prep_shard_1M_ls128.txt 2>&1 && \
timeout -k 10 400 python scripts/dev/prep_shard.py 4M-tet 8 3 > $O/prep_shard_4M.txt 2>&1 && \
timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 8 fine_then_complete,one_call > $O/rt_side1.txt 2>&1 && \
MAS_SHARD_COARSE_SIDE=2 timeout -k 10 300 python scripts/dev/shard_rank_time.py 1M+contacts 8 one_call > $O/rt_side2.txt 2>&1 && \
for i in 1 2; do \
  timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_occ8_$i.txt 2>&1 && \
  MAS_LIB_NAME=libmas_amd_ab_spmv7.so timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_occ7_$i.txt 2>&1 || exit 1; \
done
rc=$?
tail -2 $O/pytest_gpu.log
echo "exit $rc"
exit $rc
