# Round 6: no CU-masked queue by default: the facade program beside a GPU-holding parent; Prepare with the fused
# kernel in 1 / 2 / 4 / 8 launches (MAS_FUSED_CHUNKS) against the opt-in 32-CU reserve, 1M + contacts, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6o}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \

for i in 1 2; do \
  for c in 8 12 16 24 32; do \
    MAS_FUSED_CHUNKS=$c PREP_DEVICE=1 timeout -k 10 200 python scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_chunks$c.$i.txt 2>&1 || exit 1; \
  done; \
  MAS_PREP_CU_RESERVE=32 PREP_DEVICE=1 timeout -k 10 200 python scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_rsv32.$i.txt 2>&1 || exit 1; \
done
rc=$?

for f in $O/prep_*.txt; do echo "== $f"; grep prepare $f | cut -c1-60 | tail -3; done
echo "exit $rc"
exit $rc
