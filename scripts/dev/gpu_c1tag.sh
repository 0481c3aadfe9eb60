# Tagged one-launch coarse form: chain + restrict tests, timeline, A/B vs the two-launch form
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-c1tag}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_restrict.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python scripts/dev/probe_coarse1.py 1M+contacts > $O/t1M.txt 2>&1 && \
timeout -k 10 200 python scripts/dev/probe_coarse1.py 256k > $O/t256k.txt 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 1M+contacts --rounds 6 > $O/ab_1M.json 2>&1 && timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=3" "MAS_COARSE_MODE=3,MAS_C1_L1DELAY=2" "MAS_COARSE_MODE=3,MAS_C1_L1DELAY=4" --config 1M+contacts --rounds 6 > $O/ab_delay.json 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 256k --rounds 6 > $O/ab_256k.json 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 4M-tet --rounds 3 > $O/ab_4M.json 2>&1
rc=$?; cat $O/t1M.txt $O/ab_delay.json $O/ab_1M.json $O/ab_256k.json $O/ab_4M.json 2>/dev/null | grep -v amdgpu.ids; echo "exit $rc"; exit $rc
