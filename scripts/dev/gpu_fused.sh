set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fused}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "factor_kernels or small_configs" > $O/pt1.log 2>&1 && \
timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 5 > $O/prep.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pt1.log; cat $O/prep.log; tail -3 $O/pytest_gpu.log; exit $rc
