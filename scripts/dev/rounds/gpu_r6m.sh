# Round 6: the CU-masked Prepare queue released after each Prepare (default) vs kept (MAS_PREP_STREAM_KEEP=1):
# the facade program beside a GPU-holding parent, then steady-state Prepare times of both (device and host paths).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6m}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 600 python -u scripts/dev/facade_ctx.py > $O/facade_ctx.log 2>&1 && \
for i in 1 2; do \
  for k in 0 1; do \
    MAS_PREP_STREAM_KEEP=$k PREP_DEVICE=1 timeout -k 10 200 python scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_dev_keep$k.$i.txt 2>&1 && \
    MAS_PREP_STREAM_KEEP=$k timeout -k 10 200 python scripts/dev/prep_only.py 1M+contacts 4 > $O/prep_host_keep$k.$i.txt 2>&1 || exit 1; \
  done; \
done
rc=$?
grep -E "rc|ok |STUCK" $O/facade_ctx.log | cut -c1-200
for f in $O/prep_*.txt; do echo "== $f"; grep prepare $f | cut -c1-60; done
echo "exit $rc"
exit $rc
