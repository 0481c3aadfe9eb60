# A/B of library builds on the apply: bash scripts/dev/gpu_ab_apply.sh <out> <config> <libs...>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-abapply}; CFG=$2; shift 2; mkdir -p $O; export TMPDIR=/tmp; cd $R
for rep in 1 2; do for lib in "$@"; do
MAS_LIB_NAME=$lib timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-pcg --steps 300 > $O/b.json 2> $O/b.err || exit 1
python -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); a=d['apply_breakdown_ms']; print('$lib', d['value'], d['ms_per_step'], a['pre_fine'], a['fine_solve'])"
done; done
