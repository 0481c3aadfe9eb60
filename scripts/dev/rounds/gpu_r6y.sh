# Round 6 A/B: od in the early path (MAS_EARLY_OD=1) with 4 / 6 fused launches against the default, 1M + contacts
# and 4M tet, three interleaved processes per arm, 8 steady-state Prepares each.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6y}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
for c in 1M+contacts 4M-tet; do \
  for i in 1 2 3; do \
    PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 8 > $O/${c}_default.$i.txt 2>&1 && \
    MAS_EARLY_OD=1 MAS_FUSED_CHUNKS=4 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 8 > $O/${c}_eod_c4.$i.txt 2>&1 && \
    MAS_EARLY_OD=1 MAS_FUSED_CHUNKS=6 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 8 > $O/${c}_eod_c6.$i.txt 2>&1 && \
    MAS_EARLY_OD=1 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 8 > $O/${c}_eod_c8.$i.txt 2>&1 || exit 1; \
  done; \
done
rc=$?
python3 - "$O" <<'PY'
import glob, re, statistics, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*.txt"):
    arm = f.split("/")[-1].rsplit(".", 2)[0]
    v = [float(x) for x in re.findall(r"prepare ([\d.]+) ms", open(f).read())][2:]
    d[arm] += v
for arm in sorted(d):
    print(arm, "median", round(statistics.median(d[arm]), 3), "min", min(d[arm]), "n", len(d[arm]))
PY
echo "exit $rc"
exit $rc
