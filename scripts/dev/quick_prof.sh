# Development loop on one MI355X (through gpurun): GPU tests, then a kernel
# trace of a short bench run.  bash scripts/dev/quick_prof.sh <out-name> [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-quick}
mkdir -p $O
export TMPDIR=/tmp
K=${2:+-k "$2"}
cd $R && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $K > $O/pytest.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 50 > $O/bench.json 2> $O/bench.err
echo "exit $?"
