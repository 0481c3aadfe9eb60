# Round 5: fused apply with hold workgroups: tests, then A/B over the early budget.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5c
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 200 --timeout-method thread \
    > $O/pytest_fused.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_fused.log; exit 1; }
tail -3 $O/pytest_fused.log
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcg $BARGS > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
}
for i in 1 2; do
  BARGS="" run m3_$i MAS_COARSE_MODE=3
  for e in 0 64 256 512; do BARGS="" run m4_e${e}_$i MAS_COARSE_MODE=4 MAS_FUSE_EARLY=$e; done
done
for c in 256k 4M-tet; do
  BARGS="--config $c" run m3_$c MAS_COARSE_MODE=3
  for e in 0 128; do BARGS="--config $c" run m4_e${e}_$c MAS_COARSE_MODE=4 MAS_FUSE_EARLY=$e; done
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r5c/*.json")):
    d=json.load(open(f)); print(f.split('/')[-1], d["value"], d["ms_per_step"], d["apply_breakdown_ms"]["events_total"], d["roofline"]["avg_launch_ms"])
PY
