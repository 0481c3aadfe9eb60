# A/B of library builds on the one-rank sharded apply: bash scripts/dev/gpu_ab_shard.sh <out> <libs...>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-abshard}; shift; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
for rep in 1 2; do for lib in "$@"; do
MAS_LIB_NAME=$lib timeout -k 10 300 python bench.py --sharded --no-cpu-baseline --no-pcg --steps 300 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); a=d['apply_breakdown_ms']; print('$lib', d['value'], d['ms_per_step'], a)"
done; done
