set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-percu}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "factor_kernels" 2>&1 | tail -1
MAS_FUSED_PER_CU=7 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "factor_kernels" 2>&1 | tail -1
echo "default"; timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 3 2>&1 | grep -E "prepare" || exit 1
for k in 8 7 6 5; do echo "percu $k"; MAS_FUSED_PER_CU=$k timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 3 2>&1 | grep -E "prepare" || exit 1; done
for k in 8 7; do echo "percu $k serial"; MAS_PREP_SERIAL=1 MAS_FUSED_PER_CU=$k timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 3 2>&1 | grep -E "prepare" || exit 1; done
