# Round 5: grouped level 3 folded inside the level-3 solve waves (MAS_C1_FOLD3): bitwise tests, A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5e; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_restrict.py tests/test_gpu_chain.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for c in 1M+contacts 4M-tet 256k; do
  timeout -k 10 300 python scripts/ab_env.py MAS_C1_FOLD3=0 MAS_C1_FOLD3=1 --config $c > $O/ab_$c.json 2> $O/ab_$c.err || { tail -5 $O/ab_$c.err; exit 1; }
  cat $O/ab_$c.json
done
