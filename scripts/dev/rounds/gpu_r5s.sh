# Round 5: coarse_back_to_back and whole-apply figures at 256k and 4M tet on the final code.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r5s}; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for c in 256k 4M-tet 10k 1M 1M+contacts; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/b_$c.json 2> $O/b_$c.err || { tail -5 $O/b_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$c.json'));b=d['apply_breakdown_ms'];print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], b['pre_fine'], b['coarse_back_to_back'], d['apply_algorithmic_GBps'], d['prepare_ms'], d.get('pcg_solve',{}).get('mas',{}).get('ms_per_iter'))"
done
