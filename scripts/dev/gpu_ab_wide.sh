set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/wide/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_WIDE=0" "MAS_COARSE_WIDE=1" "MAS_COARSE_WIDE=0" "MAS_COARSE_WIDE=1" --config 1M+contacts --rounds 6 > gpurun_out/wide/ab_1M.json 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_WIDE=0" "MAS_COARSE_WIDE=1" --config 1M --rounds 4 > gpurun_out/wide/ab_1Mnc.json 2>&1
echo "exit $?"
