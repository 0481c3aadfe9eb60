set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fused}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "factor_kernels or small_configs or all_contact" > $O/pt1.log 2>&1 && \
for c in 0 16 32 64; do echo "reserve $c" >> $O/prep.log; MAS_PREP_CU_RESERVE=$c timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 4 >> $O/prep.log 2>&1 || exit 1; done && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pt1.log; grep -v amdgpu.ids $O/prep.log; tail -3 $O/pytest_gpu.log; exit $rc
