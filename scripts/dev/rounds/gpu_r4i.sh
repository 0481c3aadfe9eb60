# Round 4: the XCD-chunked coarse bank waves as the default -- coarse-form and
# parity tests, the bench line, the 256k config.  One && chain.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4i}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 700 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_restrict.py tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_failure.py tests/test_gpu_pcg.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err && \
timeout -k 10 300 python3 bench.py --config 256k --no-pcg --no-cpu-baseline > $O/bench_256k.json 2>> $O/bench.err && \
timeout -k 10 300 python3 bench.py --config 4M-tet --no-pcg --no-cpu-baseline > $O/bench_4M.json 2>> $O/bench.err
echo "exit $?"
