# Round 5: default-policy (temporal) coarse inverse loads in k_coarse1, A/B at three sizes.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5h; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for c in 1M+contacts 4M-tet 256k; do
  timeout -k 10 300 python scripts/ab_env.py MAS_C1_INV_TEMPORAL=0 MAS_C1_INV_TEMPORAL=1 --config $c > $O/ab_$c.json 2> $O/ab_$c.err || { tail -5 $O/ab_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$c.json'));print('$c', {k:(v['step_us_med'],v['pre_us_med'],v['bitwise_equal_to_first']) for k,v in d.items() if isinstance(v,dict)})"
done
