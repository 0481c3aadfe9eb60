# Round 5: profile_fine test, bench lines at every config, PCG A/B of the fused p update.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5g; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "profile_fine or device_path" \
    > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in 1M+contacts 256k 4M-tet 10k 1M; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
done
for f in 0 1 0 1; do
  MAS_PCG_FUSE_P=$f timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 1 > $O/pcg_fuse$f.txt 2>&1 || { tail -5 $O/pcg_fuse$f.txt; exit 1; }
  echo "fuse=$f $(grep mas: $O/pcg_fuse$f.txt)"
done
python3 - <<'PY'
import json
for c in ("1M+contacts","256k","4M-tet","10k","1M"):
    d=json.load(open(f"gpurun_out/r5g/bench_{c}.json"))
    print(c, d["value"], d["ms_per_step"], "fine b2b", d["roofline"]["avg_launch_ms"], "frac", d["roofline"]["frac"], "events", d["roofline"]["avg_launch_ms_per_apply_events"], "apply GB/s", d["apply_algorithmic_GBps"], "prep", d["prepare_ms"], "pcg", d.get("pcg_solve",{}).get("mas",{}).get("ms_per_iter"))
PY
