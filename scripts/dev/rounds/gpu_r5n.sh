# Round 5: software-pipelined long runs in k_fold_runs (coarse record folds): block-bitwise tests,
# then steady-state Prepare (unsharded and a world-8 rank) alternating with the previous build, and a trace.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5n; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for lib in libmas_amd_ab_fold0.so libmas_amd.so; do
    for sh in "" "3,8"; do
      for c in 1M+contacts 4M-tet; do
        tag=${lib}_${c}_${sh/,/of}_$rep
        PREP_SHARD=$sh MAS_LIB_NAME=$lib timeout -k 10 300 python3 scripts/dev/prep_only.py $c 6 > $O/prep_$tag.log 2>&1 || { tail -5 $O/prep_$tag.log; exit 1; }
        echo "$tag: $(tail -3 $O/prep_$tag.log | tr '\n' ' ')"
      done
    done
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/trace.log 2>&1 && \
python3 $R/scripts/dev/prepare_timeline.py $O/trace k_stencil_flags k_factor_rb > $O/timeline.txt 2>&1
echo "exit $?"
