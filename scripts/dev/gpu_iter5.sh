# early level-0 Prepare path: GPU tests, Prepare A/B over the CU reserve, prep timeline, world-8 shards
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-iter5}; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python scripts/ab_prepare.py "MAS_PREP_CU_RESERVE=0" "MAS_PREP_CU_RESERVE=32" "MAS_PREP_CU_RESERVE=64" "MAS_PREP_CU_RESERVE=80" --config 1M+contacts --rounds 4 > $O/ab_prep.json 2>&1 && \
timeout -k 10 300 python scripts/ab_prepare.py "MAS_PREP_CU_RESERVE=0" "MAS_PREP_CU_RESERVE=64" --config 4M-tet --rounds 3 > $O/ab_prep_4M.json 2>&1 && \
timeout -k 10 300 python scripts/dev/prep_shard.py 1M+contacts 8 3 > $O/prep_shard_1M.txt 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/default -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/default.log 2>&1
rc=$?; cat $O/ab_prep.json $O/ab_prep_4M.json $O/prep_shard_1M.txt | grep -v amdgpu.ids; echo "exit $rc"; exit $rc
