# Round 4: contact pipeline (ancestor-table climbs, narrow keys): parity tests,
# Prepare (whole and one world-8 rank), traces.  One && chain.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4e}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_prepare_paths.py tests/test_gpu_incremental.py tests/test_gpu_shard.py tests/test_gpu_blob.py tests/test_gpu_factor_mfma.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 8 > $O/noprof.log 2>&1 && \
PREP_SHARD=3,8 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/noprof_rank3of8.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prep -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/prep.log 2>&1 && \
python3 $R/scripts/dev/prepare_timeline.py $O/prep k_stencil_flags k_factor_rb > $O/timeline.txt 2>&1 && \
PREP_SHARD=3,8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prep_rank -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/prep_rank.log 2>&1 && \
python3 $R/scripts/dev/prepare_timeline.py $O/prep_rank k_stencil_flags k_factor_rb > $O/timeline_rank3of8.txt 2>&1
echo "exit $?"
