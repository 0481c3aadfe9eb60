# fold micro-benchmark, coarse tests + A/B (modes 2 / 3), Prepare CU-reserve A/B, PCG pipelined SpMV A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-iter3}; mkdir -p $O; cd $R
timeout -k 5 60 ./scripts/dev/bin/fold_rate > $O/fold_rate.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_restrict.py tests/test_gpu_pcg.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 1M+contacts --rounds 6 > $O/ab_1M.json 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 256k --rounds 6 > $O/ab_256k.json 2>&1 && \
timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_MODE=2" "MAS_COARSE_MODE=3" --config 4M-tet --rounds 3 > $O/ab_4M.json 2>&1 && \
timeout -k 10 300 python scripts/ab_prepare.py "MAS_PREP_CU_RESERVE=0" "MAS_PREP_CU_RESERVE=32" "MAS_PREP_CU_RESERVE=64" --config 1M+contacts --rounds 4 > $O/ab_prep.json 2>&1 && \
timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_pipe.txt 2>&1 && \
MAS_LIB_NAME=libmas_amd_ab_nopipe.so timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_nopipe.txt 2>&1
rc=$?; tail -2 $O/pytest.log; cat $O/fold_rate.txt $O/ab_1M.json $O/ab_256k.json $O/ab_4M.json $O/ab_prep.json $O/pcg_pipe.txt $O/pcg_nopipe.txt 2>/dev/null | grep -v amdgpu.ids; echo "exit $rc"; exit $rc
