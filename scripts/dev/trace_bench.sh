# Kernel trace of a short bench run (through gpurun):
#   bash scripts/dev/trace_bench.sh <out-name> [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-trace}
shift
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 50 "$@" > $O/bench.json 2> $O/bench.err
echo "exit $?"
