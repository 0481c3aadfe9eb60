# (MAS_C1_SPLIT_Z1 was removed after this measurement: profiles/round4/ab/ab_split_*.json)
# Round 4: level-1 solves in their own waves (MAS_C1_SPLIT_Z1) -- the coarse
# forms' bitwise tests, then an interleaved A/B at 1M + contacts, 4M and 256k.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4k}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python3 scripts/ab_env.py MAS_C1_SPLIT_Z1=0 MAS_C1_SPLIT_Z1=1 --config 4M-tet > $O/ab_split_4M.json 2> $O/ab.err && \
timeout -k 10 300 python3 scripts/ab_env.py MAS_C1_SPLIT_Z1=0 MAS_C1_SPLIT_Z1=1 --config 1M+contacts > $O/ab_split_1M.json 2>> $O/ab.err && \
timeout -k 10 300 python3 scripts/ab_env.py MAS_C1_SPLIT_Z1=0 MAS_C1_SPLIT_Z1=1 --config 256k > $O/ab_split_256k.json 2>> $O/ab.err
echo "exit $?"
