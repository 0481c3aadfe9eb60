# Round 5: fold3 (level-3 folded in the solve waves) tests + A/B; two-wave fused factor (MAS_FACTOR_WAVES=2)
# bitwise + timing; the PCG's fused p update.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5f; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_restrict.py tests/test_gpu_chain.py tests/test_gpu_pcg.py -x -q --timeout 200 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MAS_FACTOR_WAVES=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_factor_mfma.py tests/test_gpu_parity.py tests/test_gpu_failure.py -x -q --timeout 200 --timeout-method thread \
    > $O/pytest_w2.log 2>&1 || { echo "pytest w2 failed"; tail -40 $O/pytest_w2.log; exit 1; }
tail -2 $O/pytest_w2.log
timeout -k 10 300 python scripts/ab_prepare.py MAS_FACTOR_WAVES=1 MAS_FACTOR_WAVES=2 > $O/ab_prep.txt 2>&1 || { tail -5 $O/ab_prep.txt; exit 1; }
cat $O/ab_prep.txt
for c in 1M+contacts 4M-tet; do
  timeout -k 10 300 python scripts/ab_env.py MAS_C1_FOLD3=0 MAS_C1_FOLD3=1 --config $c > $O/ab_$c.json 2> $O/ab_$c.err || { tail -5 $O/ab_$c.err; exit 1; }
  cat $O/ab_$c.json
done
for f in 0 1; do
  MAS_PCG_FUSE_P=$f timeout -k 10 300 python scripts/dev/pcg_only.py > $O/pcg_fuse$f.txt 2>&1 || { tail -5 $O/pcg_fuse$f.txt; exit 1; }
  tail -3 $O/pcg_fuse$f.txt
done
