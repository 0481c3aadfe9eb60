# Round 6: the facade test alone (a hang in r6h), then the whole GPU suite, verbose.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6i}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py -x -v --timeout 120 --timeout-method thread > $O/pytest_facade.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --deselect tests/test_gpu_facade.py > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_facade.log; tail -3 $O/pytest_gpu.log
echo "exit $rc"
exit $rc
