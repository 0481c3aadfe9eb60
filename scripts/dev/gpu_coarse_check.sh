set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-coarse}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "restrict or chain or shard or parity" > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcg > $O/b$i.json 2> $O/b$i.err || exit 1; python -c "
import json; d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['apply_breakdown_ms']['pre_fine'], d['apply_breakdown_ms']['fine_solve'])"; done
