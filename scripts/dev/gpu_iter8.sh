# early path queued from a second host thread vs from run_levels' hook
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-iter8}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_restrict.py tests/test_gpu_blob.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python scripts/ab_prepare.py "MAS_PREP_CU_RESERVE=64" "MAS_PREP_CU_RESERVE=48" "MAS_PREP_CU_RESERVE=56" "MAS_PREP_CU_RESERVE=72" "MAS_PREP_CU_RESERVE=0" --config 1M+contacts --rounds 5 > $O/ab_prep.json 2>&1
rc=$?; cat $O/ab_prep.json | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/ab_env.py "MAS_C1_POLL_DELAY=0" "MAS_C1_POLL_DELAY=2" "MAS_C1_POLL_DELAY=3" "MAS_COARSE_MODE=2" --config 1M+contacts --rounds 6 > $O/ab_poll_1M.json 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_C1_POLL_DELAY=0" "MAS_C1_POLL_DELAY=1" "MAS_COARSE_MODE=2" --config 256k --rounds 6 > $O/ab_poll_256k.json 2>&1
rc=$?; cat $O/ab_poll_1M.json $O/ab_poll_256k.json | grep -v amdgpu.ids; echo "exit $rc"; exit $rc
