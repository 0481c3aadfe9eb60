# Round-6 start: GPU suite + smoke + bench on the inherited code.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6base}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/pytest_gpu.log
echo "exit $rc"
exit $rc
