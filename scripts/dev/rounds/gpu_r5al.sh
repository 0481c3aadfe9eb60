# Round 5: the side fold for the unsharded Prepare re-checked after the 256-term table folds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5al; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for rep in 1 2 3; do
  for fs in -1 1; do
    for c in 1M+contacts 4M-tet; do
      MAS_FOLD_SIDE=$fs timeout -k 10 300 python3 scripts/dev/prep_only.py $c 6 > $O/prep_fs${fs}_${c}_$rep.log 2>&1 || { tail -5 $O/prep_fs${fs}_${c}_$rep.log; exit 1; }
      echo "fs=$fs $c $rep: $(grep -o 'prepare [0-9.]* ms' $O/prep_fs${fs}_${c}_$rep.log | awk '{print $2}' | tail -4 | tr '\n' ' ')"
    done
  done
done
