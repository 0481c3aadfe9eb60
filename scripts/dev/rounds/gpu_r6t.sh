# Round 6 A/B: the fused level-0 kernel as a persistent grid of W waves per CU (MAS_FUSED_PERSIST) against the
# chunked default; steady-state Prepare, device Hessian, 1M + contacts, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6t}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_prepare_paths.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
for i in 1 2; do \
  for w in 0 7 6; do \
    MAS_FUSED_PERSIST=$w PREP_DEVICE=1 timeout -k 10 200 python scripts/dev/prep_only.py 1M+contacts 6 > $O/prep_persist$w.$i.txt 2>&1 || exit 1; \
  done; \
done
rc=$?
tail -1 $O/pytest.log
for f in $O/prep_*.txt; do echo "$f $(grep prepare $f | tail -3 | awk '{print $2}' | tr '\n' ' ')"; done
echo "exit $rc"
exit $rc
