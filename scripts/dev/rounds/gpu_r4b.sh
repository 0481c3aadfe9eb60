# Round 4: grouped level 3 (tests, apply A/B), Prepare evidence
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4b}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 700 python -u -m pytest tests/test_gpu_restrict.py tests/test_gpu_chain.py tests/test_gpu_shard.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcg > $O/bench.json 2> $O/bench.err && \
timeout -k 10 400 python scripts/ab_env.py MAS_REF_RESTRICT=1 MAS_REF_RESTRICT=0 --rounds 6 > $O/ab_grouped_1M.json 2>&1 && \
timeout -k 10 400 python scripts/ab_env.py MAS_REF_RESTRICT=1 MAS_REF_RESTRICT=0 --rounds 3 --config 4M-tet > $O/ab_grouped_4M.json 2>&1 && \
bash scripts/dev/gpu_prep4.sh ${1:-r4b}/prep
echo "exit $?"
