# Round 4: tests, Prepare after the worker thread (+ CU-reserve sweep, trace),
# apply kernel stats and coarse-form A/B (grouped level 3).  One && chain: the
# first failing step ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4c}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 700 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_restrict.py tests/test_gpu_incremental.py tests/test_gpu_prepare_paths.py tests/test_gpu_parity.py tests/test_gpu_blob.py tests/test_gpu_factor_mfma.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 8 > $O/noprof.log 2>&1 && \
MAS_PREP_CU_RESERVE=0 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/noprof_rsv0.log 2>&1 && \
MAS_PREP_CU_RESERVE=16 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/noprof_rsv16.log 2>&1 && \
MAS_PREP_CU_RESERVE=32 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/noprof_rsv32.log 2>&1 && \
MAS_PREP_CU_RESERVE=48 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/noprof_rsv48.log 2>&1 && \
timeout -k 10 400 python scripts/ab_env.py MAS_COARSE_MODE=2 MAS_COARSE_MODE=3 --rounds 6 > $O/ab_mode23_1M.json 2>&1 && \
timeout -k 10 400 python scripts/ab_env.py MAS_COARSE_MODE=2 MAS_COARSE_MODE=3 --rounds 3 --config 4M-tet > $O/ab_mode23_4M.json 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prep -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/prep.log 2>&1 && \
python3 $R/scripts/dev/prepare_timeline.py $O/prep k_stencil_flags k_factor_rb > $O/timeline.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bench -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-pcg > $O/bench_prof.json 2> $O/bench_prof.err
echo "exit $?"
