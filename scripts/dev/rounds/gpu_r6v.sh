# Round 6 A/B: the level-0 kernel as a persistent grid (MAS_FINE_PERSIST = waves per SIMD) against one block per
# wave; bitwise test first, then interleaved back-to-back applies at 1M + contacts, 4M tet and 256k.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6v}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_fine_forms.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
for c in 1M+contacts 4M-tet 256k; do \
  for i in 1 2; do \
    for w in 0 2 3; do \
      MAS_FINE_PERSIST=$w timeout -k 10 300 python scripts/dev/fine_loop.py $c 200 >> $O/fine_${c}_p$w.txt 2>&1 || exit 1; \
    done; \
  done; \
done
rc=$?
tail -2 $O/pytest.log
for f in $O/fine_*.txt; do echo "$f $(grep -o '"ms_per_apply": [0-9.]*\|"fine_us": [0-9.]*' $f | tr '\n' ' ')"; done
echo "exit $rc"
exit $rc
