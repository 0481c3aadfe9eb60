# Round 6: the new Prepare defaults (early od + 2 / 4 fused launches up to 32 768 blocks): schedule tests, then
# steady-state Prepare at every config and a world-8 rank, three processes each.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6aa}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_prepare_paths.py tests/test_gpu_shard.py tests/test_gpu_incremental.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
for i in 1 2 3; do \
  for c in 1M+contacts 1M 256k 4M-tet 10k; do \
    PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 8 > $O/${c}.$i.txt 2>&1 || exit 1; \
  done; \
  PREP_SHARD=3,8 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py 1M+contacts 8 > $O/rank3of8.$i.txt 2>&1 || exit 1; \
done
rc=$?
tail -1 $O/pytest.log
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
