set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/prep4; mkdir -p $O
MAS_FACTOR_VARIANT=3 timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python scripts/ab_prepare.py "MAS_FACTOR_VARIANT=1" "MAS_FACTOR_VARIANT=2" "MAS_FACTOR_VARIANT=3" > $O/ab_prepare.json 2> $O/ab_prepare.err
echo "exit $?"
