# Round 5: slab assembly with all slots' adds at once where no entry is named twice
# (duplicate neighbours keep the slot-ordered path): tests incl. a duplicate-neighbour
# mesh, bitwise hashes against the previous build, fused kernel time.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ac; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_factor_mfma.py tests/test_gpu_incremental.py -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in libmas_amd.so libmas_amd_ab_asm0.so; do
  for c in 1M+contacts 4M-tet; do
    MAS_LIB_NAME=$lib timeout -k 10 300 python3 scripts/dev/inv_hash.py $c > $O/hash_${lib}_$c.txt 2>&1 || { tail -5 $O/hash_${lib}_$c.txt; exit 1; }
    echo "$lib: $(tail -1 $O/hash_${lib}_$c.txt)"
  done
done
for rep in 1 2; do
  for lib in libmas_amd.so libmas_amd_ab_asm0.so; do
    MAS_LIB_NAME=$lib timeout -k 10 300 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_${lib}_$rep.log 2>&1 || { tail -5 $O/prep_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(grep -o 'prepare [0-9.]* ms\|fused level-0 [0-9.]*' $O/prep_${lib}_$rep.log | tail -6 | tr '\n' ' ')"
  done
done
