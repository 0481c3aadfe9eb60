# Round 5: sorted-order CSR row starts (k_sorted_ranges): one dependent load fewer in the
# fused assembly and k_od_lanes.  Tests, bitwise hashes against the previous build, Prepare
# times (and the CU reserve re-checked).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ad; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_shard.py tests/test_gpu_factor_mfma.py tests/test_gpu_blob.py -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in libmas_amd.so libmas_amd_ab_sr0.so; do
  for c in 1M+contacts 4M-tet; do
    MAS_LIB_NAME=$lib timeout -k 10 300 python3 scripts/dev/inv_hash.py $c > $O/hash_${lib}_$c.txt 2>&1 || { tail -5 $O/hash_${lib}_$c.txt; exit 1; }
    echo "$lib: $(tail -1 $O/hash_${lib}_$c.txt)"
  done
done
for rep in 1 2; do
  for v in "libmas_amd_ab_sr0.so 32" "libmas_amd.so 32" "libmas_amd.so 24"; do
    set -- $v
    for sh in "" "3,8"; do
      tag=${1}_rsv$2_${sh/,/of}_$rep
      PREP_SHARD=$sh MAS_PREP_CU_RESERVE=$2 MAS_LIB_NAME=$1 timeout -k 10 300 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_$tag.log 2>&1 || { tail -5 $O/prep_$tag.log; exit 1; }
      echo "$tag: $(grep -o 'prepare [0-9.]* ms' $O/prep_$tag.log | awk '{print $2}' | tail -4 | tr '\n' ' ') fused $(grep -o 'fused level-0 [0-9.]*' $O/prep_$tag.log | awk '{print $3}' | tail -2 | tr '\n' ' ')"
    done
  done
done
