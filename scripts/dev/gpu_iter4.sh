# fold batch sizes, Prepare CU-reserve sweep, full GPU tests with coarse mode 3 as default
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-iter4}; mkdir -p $O; cd $R
timeout -k 5 60 ./scripts/dev/bin/fold_rate > $O/fold_rate.txt 2>&1 && \
timeout -k 10 300 python scripts/ab_prepare.py "MAS_PREP_CU_RESERVE=0" "MAS_PREP_CU_RESERVE=64" "MAS_PREP_CU_RESERVE=80" "MAS_PREP_CU_RESERVE=96" "MAS_PREP_CU_RESERVE=128" --config 1M+contacts --rounds 4 > $O/ab_prep.json 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; cat $O/fold_rate.txt $O/ab_prep.json | grep -v amdgpu.ids; echo "exit $rc"; exit $rc
