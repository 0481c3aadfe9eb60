# Round 4: full GPU suite, smoke, full bench line, CU-reserve fine sweep,
# per-rank sharded Prepare, counter list.  One && chain.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4d}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
MAS_PREP_CU_RESERVE=24 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/rsv24.log 2>&1 && \
MAS_PREP_CU_RESERVE=32 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/rsv32.log 2>&1 && \
MAS_PREP_CU_RESERVE=40 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/rsv40.log 2>&1 && \
timeout -k 10 400 python3 scripts/dev/prep_shard.py 1M+contacts 8 3 > $O/shard_world8_1M.txt 2>&1 && \
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1
echo "exit $?"
