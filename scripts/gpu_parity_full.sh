set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1100 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/t2.log 2>&1
