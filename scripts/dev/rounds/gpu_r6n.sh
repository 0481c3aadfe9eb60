# Round 6: Prepare without the CU-masked queue (MAS_PREP_CU_RESERVE=0) against the kept masked queue (32 CUs,
# MAS_PREP_STREAM_KEEP=1), steady state, device Hessian, 1M + contacts and 4M tet, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6n}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
for i in 1 2; do \
  for c in 1M+contacts 4M-tet; do \
    MAS_PREP_STREAM_KEEP=1 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 6 > $O/prep_${c}_rsv32.$i.txt 2>&1 && \
    MAS_PREP_CU_RESERVE=0 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py $c 6 > $O/prep_${c}_rsv0.$i.txt 2>&1 || exit 1; \
  done; \
done
rc=$?
for f in $O/prep_*.txt; do echo "== $f"; grep prepare $f | cut -c1-60; done
echo "exit $rc"
exit $rc
