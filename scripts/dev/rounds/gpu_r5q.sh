# Round 5: rb_step with the pivot by readlane and branch-free divisions: block-bitwise
# tests, then steady-state Prepare alternating with the previous build.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5q; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_shard.py tests/test_gpu_factor_mfma.py -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for lib in libmas_amd_ab_rb0.so libmas_amd.so; do
    for sh in "" "3,8"; do
      for c in 1M+contacts 4M-tet; do
        tag=${lib}_${c}_${sh/,/of}_$rep
        PREP_SHARD=$sh MAS_LIB_NAME=$lib timeout -k 10 300 python3 scripts/dev/prep_only.py $c 6 > $O/prep_$tag.log 2>&1 || { tail -5 $O/prep_$tag.log; exit 1; }
        echo "$tag: $(grep -o 'prepare [0-9.]* ms\|from [0-9.]*' $O/prep_$tag.log | tail -6 | tr '\n' ' ')"
      done
    done
  done
done
