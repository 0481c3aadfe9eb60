set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/prep; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python scripts/ab_prepare.py "MAS_FACTOR_VARIANT=0" "MAS_FACTOR_VARIANT=1" > $O/ab_prepare.json 2> $O/ab_prepare.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 10 > $O/bench_prof.log 2>&1
echo "exit $?"
