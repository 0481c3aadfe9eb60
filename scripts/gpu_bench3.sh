set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/t5.log 2>&1
timeout -k 10 600 python bench.py --steps 200 --warmup 20 > gpurun_out/bench4.json 2> gpurun_out/bench4.err
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof4 -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline > $R/gpurun_out/bench4_prof.json 2> $R/gpurun_out/bench4_prof.err
