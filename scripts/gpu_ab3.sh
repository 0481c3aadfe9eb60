set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab3; mkdir -p $O
MAS_FACTOR_VARIANT=2 timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python scripts/ab_prepare.py "MAS_FACTOR_VARIANT=3" "MAS_FACTOR_VARIANT=2" > $O/ab_prepare.json 2> $O/ab_prepare.err && \
timeout -k 10 600 python scripts/ab_env.py "MAS_OVERLAP=0" "MAS_OVERLAP=1" "MAS_OVERLAP=1,MAS_SIDE_PRIORITY=0" > $O/ab_overlap.json 2> $O/ab_overlap.err
echo "exit $?"
