set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab2; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
timeout -k 10 600 python scripts/ab_env.py "MAS_OVERLAP=0" "MAS_OVERLAP=1" > $O/ab.json 2> $O/ab.err
