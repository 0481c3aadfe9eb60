# Round 4: CU reserve of the fused kernel's queue at 4M tet and 256k (one
# process per setting; the mask is fixed at stream creation).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4n}; mkdir -p $O; export TMPDIR=/tmp
cd $R && for rsv in 0 16 32 48 64; do \
  MAS_PREP_CU_RESERVE=$rsv timeout -k 10 300 python3 scripts/dev/prep_only.py 4M-tet 4 > $O/4M_rsv$rsv.log 2>&1 || exit 1; done && \
for rsv in 0 16 32 64; do \
  MAS_PREP_CU_RESERVE=$rsv timeout -k 10 200 python3 scripts/dev/prep_only.py 256k 6 > $O/256k_rsv$rsv.log 2>&1 || exit 1; done
echo "exit $?"
