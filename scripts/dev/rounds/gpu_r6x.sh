# Round 6 A/B on the chunked schedule: od in the early path (MAS_EARLY_OD=1) and the fused kernel after the level
# build (MAS_FUSED_AFTER_LEVELS=1); steady-state Prepare, device Hessian, 1M + contacts, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6x}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
for i in 1 2; do \
  PREP_DEVICE=1 timeout -k 10 200 python scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_default.$i.txt 2>&1 && \
  MAS_EARLY_OD=1 PREP_DEVICE=1 timeout -k 10 200 python scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_earlyod.$i.txt 2>&1 && \
  MAS_EARLY_OD=1 MAS_FUSED_CHUNKS=4 PREP_DEVICE=1 timeout -k 10 200 python scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_earlyod_c4.$i.txt 2>&1 && \
  MAS_FUSED_AFTER_LEVELS=1 PREP_DEVICE=1 timeout -k 10 200 python scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_afterlevels.$i.txt 2>&1 || exit 1; \
done
rc=$?
for f in $O/prep_*.txt; do echo "$f $(grep prepare $f | tail -3 | awk '{print $2}' | tr '\n' ' ') | $(grep -o 'fused level-0 [0-9.]*' $f | tail -1)"; done
echo "exit $rc"
exit $rc
