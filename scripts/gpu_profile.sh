# Round-end evidence on one MI355X (run through gpurun):
#   bash scripts/gpu_profile.sh <out-name>
# GPU tests, smoke, bench (with cpu_baseline), a rocprofv3 kernel trace of the
# same bench command, and separate FETCH_SIZE / WRITE_SIZE PMC passes.  Every
# GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-profile}
mkdir -p $O
export TMPDIR=/tmp
cd $R && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
cd /tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_trace.json 2> $O/trace.err && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcg > $O/bench_pmc1.json 2> $O/pmc1.err && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcg > $O/bench_pmc2.json 2> $O/pmc2.err
echo "exit $?"
