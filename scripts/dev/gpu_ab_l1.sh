# level-1 solves in k_restrict12 vs k_solve123 at three sizes: bash scripts/dev/gpu_ab_l1.sh <out>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-abl1}; mkdir -p $O; export TMPDIR=/tmp; cd $R
for c in 256k 1M+contacts 4M-tet; do
  timeout -k 10 300 python scripts/ab_env.py "MAS_L1_SOLVE=0" "MAS_L1_SOLVE=1" --config $c --rounds 5 > $O/ab_$c.json 2> $O/ab_$c.err || exit $?
done
echo "exit $?"
