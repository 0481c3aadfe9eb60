# Round 5: od and the record counts in the early path (MAS_EARLY_OD=1: before the fused kernel,
# on a quiet chip) with smaller CU reserves, against the default (od on the reserved CUs, 32).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5z; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for rep in 1 2; do
  for v in "0 32" "1 32" "1 24" "1 16" "1 8"; do
    set -- $v
    tag=eod$1_rsv$2_$rep
    MAS_EARLY_OD=$1 MAS_PREP_CU_RESERVE=$2 timeout -k 10 300 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_$tag.log 2>&1 || { tail -5 $O/prep_$tag.log; exit 1; }
    echo "$tag: $(grep -o 'prepare [0-9.]* ms' $O/prep_$tag.log | awk '{print $2}' | tail -5 | tr '\n' ' ') fused $(grep -o 'fused level-0 [0-9.]* from [0-9.]*' $O/prep_$tag.log | tail -2 | tr '\n' ' ')"
  done
done
