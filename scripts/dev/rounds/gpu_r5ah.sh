# Round 5: k_coarse1 bank waves loading their inverse first (MAS_C1_EARLY_INV=1) against after
# the publications (0): interleaved in one process (scripts/ab_env.py), bitwise.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ah; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for c in 4M-tet 1M+contacts 256k; do
  timeout -k 10 400 python -u scripts/ab_env.py MAS_C1_EARLY_INV=0 MAS_C1_EARLY_INV=1 --config $c > $O/ab_$c.json 2> $O/ab_$c.err || { tail -5 $O/ab_$c.err; exit 1; }
  echo "== $c"; python3 -c "import json;d=json.load(open('$O/ab_$c.json'));[print(k, v) for k,v in d.items()]"
done
