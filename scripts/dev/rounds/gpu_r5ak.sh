# Round 5: tests touching the Prepare chain (bitwise coarse blocks, shards, incremental), then a
# world-8 rank's Prepare trace with the current code.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ak; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_incremental.py tests/test_gpu_shard.py tests/test_gpu_blob.py -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && PREP_SHARD=3,8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/trace.log 2>&1
echo "exit $?"
