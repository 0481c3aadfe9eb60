# Round 6 A/B: od in the early path with fewer fused launches at 256k and the contact-free 1M cloth; three
# interleaved processes per arm, 8 steady-state Prepares each.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6z}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
for i in 1 2 3; do \
  PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py 256k 8 > $O/256k_default.$i.txt 2>&1 && \
  MAS_EARLY_OD=1 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py 256k 8 > $O/256k_eod_c4.$i.txt 2>&1 && \
  MAS_EARLY_OD=1 MAS_FUSED_CHUNKS=2 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py 256k 8 > $O/256k_eod_c2.$i.txt 2>&1 && \
  PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py 1M 8 > $O/1M_default.$i.txt 2>&1 && \
  MAS_EARLY_OD=1 MAS_FUSED_CHUNKS=4 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py 1M 8 > $O/1M_eod_c4.$i.txt 2>&1 || exit 1; \
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
