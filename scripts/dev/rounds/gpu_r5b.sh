# Round 5: fused apply (coarseMode 4) first run: bitwise tests, then A/B bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 200 --timeout-method thread \
    > $O/pytest_fused.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_fused.log; exit 1; }
tail -3 $O/pytest_fused.log
for i in 1 2; do
  MAS_COARSE_MODE=3 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcg > $O/bench_m3_$i.json 2> $O/bench_m3_$i.err || exit 1
  MAS_COARSE_MODE=4 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcg > $O/bench_m4_$i.json 2> $O/bench_m4_$i.err || exit 1
done
for c in 256k 4M-tet; do
  MAS_COARSE_MODE=3 timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-pcg > $O/bench_m3_$c.json 2> $O/bench_m3_$c.err || exit 1
  MAS_COARSE_MODE=4 timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-pcg > $O/bench_m4_$c.json 2> $O/bench_m4_$c.err || exit 1
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r5b/bench_*.json")):
    d=json.load(open(f)); print(f.split('/')[-1], d["value"], d["ms_per_step"], d["apply_breakdown_ms"]["events_total"], d["roofline"]["avg_launch_ms"])
PY
