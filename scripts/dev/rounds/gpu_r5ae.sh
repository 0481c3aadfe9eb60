# Round 5: the cached CSR records' fold on a side stream beside od / k_diag1 / the table
# folds (MAS_FOLD_SIDE=1) against in line (0); bitwise hashes, Prepare times, reserve 24.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ae; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_shard.py tests/test_gpu_blob.py -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for fs in 0 1; do
  for c in 1M+contacts 4M-tet; do
    MAS_FOLD_SIDE=$fs timeout -k 10 300 python3 scripts/dev/inv_hash.py $c > $O/hash_fs${fs}_$c.txt 2>&1 || { tail -5 $O/hash_fs${fs}_$c.txt; exit 1; }
    echo "fold_side=$fs: $(tail -1 $O/hash_fs${fs}_$c.txt)"
  done
done
for rep in 1 2; do
  for v in "0 32" "1 32" "1 24" "1 40"; do
    set -- $v
    for sh in "" "3,8"; do
      tag=fs$1_rsv$2_${sh/,/of}_$rep
      PREP_SHARD=$sh MAS_PREP_CU_RESERVE=$2 MAS_FOLD_SIDE=$1 timeout -k 10 300 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_$tag.log 2>&1 || { tail -5 $O/prep_$tag.log; exit 1; }
      echo "$tag: $(grep -o 'prepare [0-9.]* ms' $O/prep_$tag.log | awk '{print $2}' | tail -4 | tr '\n' ' ') fused $(grep -o 'fused level-0 [0-9.]*' $O/prep_$tag.log | awk '{print $3}' | tail -2 | tr '\n' ' ')"
    done
  done
done
