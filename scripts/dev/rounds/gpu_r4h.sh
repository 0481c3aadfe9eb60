# Round 4: the XCD-chunked fine kernel as the default (tests); per-apply time against run length (ramp.py; bench.py at the
# driver's 5 + 20 applies and at 500 + 2000), then the sharded-Prepare CU
# reserve / early-od sweep (gpu_shard_rsv.sh).  One && chain.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4h}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_shard.py tests/test_gpu_pcg.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 200 python3 scripts/dev/ramp.py 1M+contacts 3 20 > $O/ramp_1M.json 2> $O/ramp.err && \
timeout -k 10 300 python3 scripts/dev/ramp.py 4M-tet 4 10 > $O/ramp_4M.json 2>> $O/ramp.err && \
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcg --steps 20 --warmup 5 > $O/bench_short.json 2> $O/bench.err && \
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcg --steps 2000 --warmup 500 > $O/bench_long.json 2>> $O/bench.err && \
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcg --steps 20 --warmup 5 > $O/bench_short2.json 2>> $O/bench.err && \
bash scripts/dev/gpu_shard_rsv.sh ${1:-r4h}/shard
echo "exit $?"
