# Round 5: unconditional bank gathers (mode 3) and the fused form with slow-polling holds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5d
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_restrict.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python scripts/dev/fused_diag.py 256k 1M+contacts 4M-tet > $O/diag.txt 2>&1 || exit 1
cat $O/diag.txt | grep -v amdgpu.ids
for i in 1 2; do
  MAS_COARSE_MODE=3 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pcg > $O/m3_$i.json 2> $O/m3_$i.err || exit 1
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r5d/*.json")):
    d=json.load(open(f)); print(f.split('/')[-1], d["value"], d["ms_per_step"], d["apply_breakdown_ms"])
PY
