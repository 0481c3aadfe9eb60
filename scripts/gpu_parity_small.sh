set -o pipefail
cd $GRAFT_REPO_ROOT
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -k "small or device" > gpurun_out/t1.log 2>&1
