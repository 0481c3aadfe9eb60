# Round 5: the branch-free unrolled MFMA formation against the previous build (bitwise + fused kernel time).
# inverse formation (noform) compiled out, against the full kernel (wrong inverses in the
# probes: timing only, no test runs against them).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5v; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for rep in 1 2; do
  for lib in libmas_amd.so libmas_amd_ab_form0.so; do
    MAS_LIB_NAME=$lib timeout -k 10 300 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_${lib}_$rep.log 2>&1 || { tail -5 $O/prep_${lib}_$rep.log; exit 1; }
    echo "$lib $rep: $(grep -o 'fused level-0 [0-9.]*' $O/prep_${lib}_$rep.log | awk '{print $3}' | tr '\n' ' ')"
  done
done
for lib in libmas_amd.so libmas_amd_ab_form0.so; do
  for c in 1M+contacts 4M-tet; do
    MAS_LIB_NAME=$lib timeout -k 10 300 python3 scripts/dev/inv_hash.py $c > $O/hash_${lib}_$c.txt 2>&1 || { tail -5 $O/hash_${lib}_$c.txt; exit 1; }
    echo "$lib: $(cat $O/hash_${lib}_$c.txt | tail -1)"
  done
done
