# One-launch coarse form (k_coarse1.hip): chain + restrict tests, then A/B vs the two-pass form
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-coarse1}
mkdir -p $O
export TMPDIR=/tmp
cd $R && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_restrict.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 1M+contacts > $O/ab_1M.json 2> $O/ab_1M.err && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 256k > $O/ab_256k.json 2> $O/ab_256k.err && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 4M-tet --rounds 4 > $O/ab_4M.json 2> $O/ab_4M.err
rc=$?
tail -3 $O/pytest.log
echo "exit $rc"
exit $rc
