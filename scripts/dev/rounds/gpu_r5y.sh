# Round 5: CU reserve of the fused kernel's queue re-swept after the formation rewrite
# (the coarse chain is now the longer path); one process per setting (CU-masked queues).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5y; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for rep in 1 2; do
  for rsv in 32 40 48 64 24; do
    for sh in "" "3,8"; do
      tag=rsv${rsv}_${sh/,/of}_$rep
      PREP_SHARD=$sh MAS_PREP_CU_RESERVE=$rsv timeout -k 10 300 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_$tag.log 2>&1 || { tail -5 $O/prep_$tag.log; exit 1; }
      echo "$tag: $(grep -o 'prepare [0-9.]* ms' $O/prep_$tag.log | awk '{print $2}' | tail -5 | tr '\n' ' ') fused $(grep -o 'fused level-0 [0-9.]*' $O/prep_$tag.log | awk '{print $3}' | tail -2 | tr '\n' ' ')"
    done
  done
done
for rsv in 32 48; do
  MAS_PREP_CU_RESERVE=$rsv timeout -k 10 300 python3 scripts/dev/prep_only.py 4M-tet 5 > $O/prep4M_rsv$rsv.log 2>&1 || { tail -5 $O/prep4M_rsv$rsv.log; exit 1; }
  echo "4M rsv$rsv: $(grep -o 'prepare [0-9.]* ms' $O/prep4M_rsv$rsv.log | awk '{print $2}' | tail -4 | tr '\n' ' ')"
done
