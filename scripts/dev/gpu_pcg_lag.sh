# PCG lagged done-flag check: GPU tests, then MAS_PCG_LAG=0/1 A/B on the PCG, then one bench line
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pcglag}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for lag in 0 1 0 1; do
  echo "MAS_PCG_LAG=$lag" >> $O/pcg.log
  MAS_PCG_LAG=$lag timeout -k 10 200 python scripts/dev/pcg_only.py 1M+contacts 2 >> $O/pcg.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/pcg.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['pcg_solve'])"
