# Round 6: the PCG tests on the float2-ELL A/B library, PCG SpMV A/B, kernel traces of the
# one-call sharded apply (mode 1 vs inline), PCG SpMV float2-ELL A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6h}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
MAS_LIB_NAME=libmas_amd_ab_ell2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_pcg.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ell2.log 2>&1 && \
for i in 1 2; do \
  timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_ell1_$i.txt 2>&1 && \
  MAS_LIB_NAME=libmas_amd_ab_ell2.so timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_ell2_$i.txt 2>&1 || exit 1; \
done && \
bash scripts/dev/rounds/gpu_r6g.sh ${1:-r6h}/traces
rc=$?
tail -2 $O/pytest_ell2.log
echo "exit $rc"
exit $rc
