# (MAS_C1_PREFETCH was removed after this measurement: profiles/round4/ab/ab_prefetch_*.json)
# Round 4: bank waves loading their level-1 record behind the r gathers
# (MAS_C1_PREFETCH) -- interleaved A/B (bitwise check included) at 256k, 1M
# + contacts and 4M tet, and the coarse-form tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4o}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 300 python3 scripts/ab_env.py MAS_C1_PREFETCH=0 MAS_C1_PREFETCH=1 --config 256k > $O/ab_prefetch_256k.json 2> $O/ab.err && \
timeout -k 10 300 python3 scripts/ab_env.py MAS_C1_PREFETCH=0 MAS_C1_PREFETCH=1 --config 1M+contacts > $O/ab_prefetch_1M.json 2>> $O/ab.err && \
timeout -k 10 400 python3 scripts/ab_env.py MAS_C1_PREFETCH=0 MAS_C1_PREFETCH=1 --config 4M-tet > $O/ab_prefetch_4M.json 2>> $O/ab.err && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_restrict.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "exit $?"
