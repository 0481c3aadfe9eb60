# Prepare changes: parity tests that check every assembled block bitwise, then steady-state Prepare times
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-prepcheck}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blob.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
for c in 1M+contacts 1M 256k 4M-tet; do timeout -k 10 200 python scripts/dev/prep_only.py $c 4 > $O/prep_$c.log 2>&1 || exit 1; done
echo "exit $?"
