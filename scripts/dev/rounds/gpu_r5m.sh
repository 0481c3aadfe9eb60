# Round 5: size-dependent inverse load policy (fine_var): GPU tests that reach the fine kernel, then bench at 256k / 1M.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5m; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_pcg.py tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in 256k 1M+contacts; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/b_$c.json 2> $O/b_$c.err || { tail -5 $O/b_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['pcg_solve']['mas']['ms_per_iter'])"
done
