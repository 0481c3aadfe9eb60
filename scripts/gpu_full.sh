# Full GPU check: tests, smoke, bench, kernel trace (rocprofv3) into gpurun_out/$1
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-full}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_trace.json 2> $O/trace.err
echo "exit $?"
