# early fused: CU reserve around 64, fused start before / after the level build
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-iter6}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "contact or 1m" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python scripts/ab_prepare.py "MAS_PREP_CU_RESERVE=48" "MAS_PREP_CU_RESERVE=56" "MAS_PREP_CU_RESERVE=64" "MAS_PREP_CU_RESERVE=72" "MAS_PREP_CU_RESERVE=64,MAS_FUSED_AFTER_LEVELS=1" "MAS_PREP_CU_RESERVE=48,MAS_FUSED_AFTER_LEVELS=1" --config 1M+contacts --rounds 4 > $O/ab_prep.json 2>&1
rc=$?; cat $O/ab_prep.json | grep -v amdgpu.ids; echo "exit $rc"; exit $rc
