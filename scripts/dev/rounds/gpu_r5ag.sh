# Round 5: the fine kernel held to 4 waves per SIMD (128 VGPRs, 24 spilled) against 3 (148 VGPRs):
# alternating bench processes, 1M + contacts and 4M tet.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5ag; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for rep in 1 2; do
  for lib in libmas_amd.so libmas_amd_ab_w4.so; do
    for c in 1M+contacts 4M-tet 256k; do
      MAS_LIB_NAME=$lib timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-pcg > $O/b_${lib}_${c}_$rep.json 2> $O/b_${lib}_${c}_$rep.err || { tail -5 $O/b_${lib}_${c}_$rep.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/b_${lib}_${c}_$rep.json'));print('$lib $c $rep', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
    done
  done
done
