# bash scripts/dev/gpu_prep_ab.sh <out> <VAR> <a,b> [configs...]: interleaved Prepare A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp; cd $R
var=$2; vals=$3; shift 3
for c in "$@"; do timeout -k 10 300 python scripts/dev/prep_ab.py $c $var $vals 10 >> $O/ab.log 2>&1 || exit 1; done
echo "exit $?"
