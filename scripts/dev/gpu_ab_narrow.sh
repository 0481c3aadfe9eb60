# single-wave coarse workgroups at three sizes: bash scripts/dev/gpu_ab_narrow.sh <out>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-abnarrow}; mkdir -p $O; export TMPDIR=/tmp; cd $R
for c in 256k 1M+contacts; do
  timeout -k 10 300 python scripts/ab_env.py "MAS_COARSE_NARROW=0" "MAS_COARSE_NARROW=1" --config $c --rounds 5 > $O/ab_$c.json 2> $O/ab_$c.err || exit $?
done
echo "exit $?"
