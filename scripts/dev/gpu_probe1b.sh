set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/probe1/pytest.log 2>&1 && \
timeout -k 10 200 python scripts/dev/probe_coarse1.py 1M+contacts > gpurun_out/probe1/1M.txt 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 1M+contacts --rounds 4 > gpurun_out/probe1/ab_1M.json 2>&1
echo "exit $?"
