# Round 6 A/B: the first K level-0 blocks' inverses with default-policy loads (Infinity Cache resident across
# applies?), the rest nontemporal (MAS_RESIDENT_SPLIT=K, two fine launches), 1M + contacts, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6j}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
for i in 1 2; do \
  for k in 0 4096 8192 10240 12288; do \
    MAS_RESIDENT_SPLIT=$k timeout -k 10 200 python scripts/dev/fine_loop.py 1M+contacts 200 >> $O/split_$k.txt 2>&1 || exit 1; \
  done; \
done
rc=$?
for k in 0 4096 8192 10240 12288; do echo "K=$k"; cat $O/split_$k.txt; done
echo "exit $rc"
exit $rc
