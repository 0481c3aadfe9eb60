# Round 5: LDS-free bank-wave transposition in k_coarse1 (6 KB LDS instead of 13 KB): bitwise tests, then
# alternating bench processes against the previous build (libmas_amd_ab_c1old.so).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5k; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_restrict.py tests/test_gpu_chain.py tests/test_gpu_failure.py -x -q --timeout 200 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for lib in libmas_amd_ab_c1old.so libmas_amd.so; do
    for c in 1M+contacts 4M-tet; do
      MAS_LIB_NAME=$lib timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-pcg > $O/b_${lib}_${c}_$rep.json 2> $O/b_${lib}_${c}_$rep.err || { tail -5 $O/b_${lib}_${c}_$rep.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/b_${lib}_${c}_$rep.json'));print('$lib $c $rep', d['value'], d['ms_per_step'], d['apply_breakdown_ms']['pre_fine'])"
    done
  done
done
