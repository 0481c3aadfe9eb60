# fine-kernel variant A/B at three sizes + a 4M-tet kernel trace: bash scripts/dev/gpu_ab_fine.sh <out>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-abfine}; mkdir -p $O; export TMPDIR=/tmp; cd $R
for c in 1M+contacts 256k 4M-tet; do
  timeout -k 10 300 python scripts/ab_env.py "MAS_FINE_VARIANT=1" "MAS_FINE_VARIANT=2" --config $c --rounds 5 > $O/ab_$c.json 2> $O/ab_$c.err || exit $?
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace4m -o run --output-format csv -- python3 $R/bench.py --config 4M-tet --steps 50 --warmup 5 --no-cpu-baseline --no-pcg > $O/b4m.json 2> $O/b4m.err
echo "exit $?"
