# Round 5: default-policy inverse loads in the fine kernel (MAS_FINE_VARIANT=8: the Infinity
# Cache may keep the inverses between applies where they fit) against the nontemporal default (6).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5l; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for c in 256k 1M+contacts 10k; do
  timeout -k 10 300 python -u scripts/ab_env.py MAS_FINE_VARIANT=6 MAS_FINE_VARIANT=8 --config $c > $O/ab_$c.json 2> $O/ab_$c.err || { tail -5 $O/ab_$c.err; exit 1; }
  echo "== $c"; cat $O/ab_$c.json
done
for rep in 1 2; do
  for v in 6 8; do
    MAS_FINE_VARIANT=$v timeout -k 10 300 python -u scripts/dev/pcg_only.py 256k 2 > $O/pcg_256k_v${v}_$rep.txt 2>&1 || { tail -5 $O/pcg_256k_v${v}_$rep.txt; exit 1; }
    echo "pcg 256k v=$v rep=$rep: $(grep mas $O/pcg_256k_v${v}_$rep.txt | tr '\n' ' ')"
  done
done
