# Round 6: one bench.py run per BASELINE config on the final code (CPU baseline included, no host path).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6q}; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for c in 10k 256k 1M 1M+contacts 4M-tet; do
  timeout -k 10 500 python bench.py --config $c --no-host-path > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$c.json'));b=d['apply_breakdown_ms'];print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], b['pre_fine'], b['coarse_back_to_back'], d['apply_algorithmic_GBps'], d['prepare_ms'], (d.get('cpu_baseline') or {}).get('value'), d.get('pcg_solve',{}).get('mas',{}).get('ms_per_iter'))"
done
timeout -k 10 300 python scripts/dev/prep_shard.py 1M+contacts 8 3 > $O/prep_shard_1M.txt 2>&1 || { tail -5 $O/prep_shard_1M.txt; exit 1; }
timeout -k 10 400 python scripts/dev/prep_shard.py 4M-tet 8 3 > $O/prep_shard_4M.txt 2>&1 || { tail -5 $O/prep_shard_4M.txt; exit 1; }
tail -1 $O/prep_shard_1M.txt; tail -1 $O/prep_shard_4M.txt
