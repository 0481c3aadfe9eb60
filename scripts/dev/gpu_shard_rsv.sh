# Round 4: the CU reserve of the fused kernel's queue for a sharded Prepare
# (world-8 rank 3: the fused kernel is 1/8 of the blocks, the replicated
# coarse chain is the longer path).  One process per setting.  One && chain.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-shard_rsv}; mkdir -p $O; export TMPDIR=/tmp
cd $R && for rsv in 32 64 96 128; do \
  MAS_PREP_CU_RESERVE=$rsv PREP_SHARD=3,8 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/rank3_rsv$rsv.log 2>&1 || exit 1; done && \
for rsv in 32 96; do \
  MAS_EARLY_OD=1 MAS_PREP_CU_RESERVE=$rsv PREP_SHARD=3,8 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/rank3_earlyod_rsv$rsv.log 2>&1 || exit 1; done && \
for rsv in 32 128; do \
  MAS_PREP_CU_RESERVE=$rsv PREP_SHARD=3,8 timeout -k 10 300 python3 scripts/dev/prep_only.py 4M-tet 4 > $O/rank3_4M_rsv$rsv.log 2>&1 || exit 1; done && \
timeout -k 10 300 python3 scripts/dev/prep_only.py 4M-tet 4 > $O/whole_4M_rsv32.log 2>&1
echo "exit $?"
