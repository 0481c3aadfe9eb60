# Round 6: the fused level-0 kernel in C launches (MAS_FUSED_CHUNKS) at the other sizes: 4M tet, 256k, a world-8
# rank of 1M + contacts; steady-state Prepare, device Hessian, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6p}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
for i in 1 2; do \
  for c in 1 4 8 16; do \
    MAS_FUSED_CHUNKS=$c PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py 4M-tet 5 > $O/prep_4M_chunks$c.$i.txt 2>&1 || exit 1; \
  done; \
  for c in 1 2 4 8; do \
    MAS_FUSED_CHUNKS=$c PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py 256k 6 > $O/prep_256k_chunks$c.$i.txt 2>&1 || exit 1; \
    MAS_FUSED_CHUNKS=$c PREP_SHARD=3,8 PREP_DEVICE=1 timeout -k 10 300 python scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_r3of8_chunks$c.$i.txt 2>&1 || exit 1; \
  done; \
done
rc=$?
for f in $O/prep_*.txt; do echo "== $f"; grep prepare $f | cut -c1-60 | tail -3; done
echo "exit $rc"
exit $rc
