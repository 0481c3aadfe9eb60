# Round-6 evidence on one MI355X: full GPU suite, smoke, bench (+ cpu_baseline, host path), the N = 2 gloo
# rehearsal, a rocprofv3 kernel trace of the bench command, separate FETCH_SIZE / WRITE_SIZE PMC passes, and the
# matrix-core counters of the factor kernels (k_factor_fused, k_factor_rb) of steady-state Prepares.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6e}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err && \
cd /tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-host-path > $O/bench_trace.json 2> $O/trace.err && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcg --no-host-path > $O/bench_pmc1.json 2> $O/pmc1.err && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcg --no-host-path > $O/bench_pmc2.json 2> $O/pmc2.err && \
timeout -s KILL 300 rocprofv3 --kernel-include-regex k_factor --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES -d $O/pmc_mfma -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 2 > $O/pmc_mfma.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
echo "exit $rc"
exit $rc
