# Quick GPU validation through gpurun:  bash scripts/gpu_check.sh <out-name> [pytest -k expr]
# GPU tests (one process, per-test timeout), smoke, one bench line.  Each step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-check}
mkdir -p $O
export TMPDIR=/tmp
K=()
[ -n "$2" ] && K=(-k "$2")
cd $R && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/pytest_gpu.log
echo "exit $rc"
exit $rc
