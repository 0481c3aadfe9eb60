# Round 5 timing probe (after the formation rewrite): the fused level-0 kernel with its elimination (noelim) or its
# inverse formation (noform) compiled out, against the full kernel (wrong inverses in the
# probes: timing only, no test runs against them).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5w; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for rep in 1 2; do
  for lib in libmas_amd.so libmas_amd_ab_noelim.so libmas_amd_ab_noform.so libmas_amd_ab_noasm.so; do
    MAS_LIB_NAME=$lib timeout -k 10 300 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_${lib}_$rep.log 2>&1 || { tail -5 $O/prep_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(grep -o 'fused level-0 [0-9.]*' $O/prep_${lib}_$rep.log | awk '{print $3}' | tr '\n' ' ')"
  done
done
