set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" "MAS_COARSE_MODE=3,MAS_C1_EARLY_INV=1" --config 256k --rounds 6 > gpurun_out/c1/ab_256k.json 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" "MAS_COARSE_MODE=3,MAS_C1_EARLY_INV=1" --config 1M+contacts --rounds 4 > gpurun_out/c1/ab_1M.json 2>&1
echo "exit $?"
