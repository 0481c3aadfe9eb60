# fine kernel: one wave per workgroup at three sizes: bash scripts/dev/gpu_ab_fine1.sh <out>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-abfine1}; mkdir -p $O; export TMPDIR=/tmp; cd $R
for c in 256k 1M+contacts 4M-tet; do
  timeout -k 10 300 python scripts/ab_env.py "MAS_FINE_VARIANT=1" "MAS_FINE_VARIANT=3" --config $c --rounds 5 > $O/ab_$c.json 2> $O/ab_$c.err || exit $?
done
echo "exit $?"
