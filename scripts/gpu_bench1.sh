set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 200 --warmup 20 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $R/gpurun_out/bench1_prof.json 2> $R/gpurun_out/bench1_prof.err
