# Round 6 A/B: the fused level-0 kernel with two blocks per workgroup (MAS_FUSED_PAIR=1) and a barrier every 8
# elimination steps (9); schedule tests, then steady-state Prepare, three processes per arm.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6ac}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_prepare_paths.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
for i in 1 2 3; do \
  for c in 1M+contacts 4M-tet; do \
    for p in 0 1 9; do \
      MAS_FUSED_PAIR=$p PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 8 > $O/${c}_pair$p.$i.txt 2>&1 || exit 1; \
    done; \
    MAS_FUSED_PAIR=9 MAS_FUSED_CHUNKS=1 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 8 > $O/${c}_pair9_c1.$i.txt 2>&1 || exit 1; \
    MAS_FUSED_CHUNKS=1 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 8 > $O/${c}_pair0_c1.$i.txt 2>&1 || exit 1; \
  done; \
done
rc=$?
tail -1 $O/pytest.log
python3 - "$O" <<'PY'
import glob, re, statistics, sys, collections
d = collections.defaultdict(list); fz = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*.txt"):
    arm = f.split("/")[-1].rsplit(".", 2)[0]
    t = open(f).read()
    d[arm] += [float(x) for x in re.findall(r"prepare ([\d.]+) ms", t)][2:]
    fz[arm] += [float(x) for x in re.findall(r"fused level-0 ([\d.]+)", t)][2:]
for arm in sorted(d):
    print(arm, "prepare median", round(statistics.median(d[arm]), 3), "fused median", round(statistics.median(fz[arm]), 3), "n", len(d[arm]))
PY
echo "exit $rc"
exit $rc
