# Round 4: the XCD-chunked fine kernel in two-wave workgroups (variant 6)
# against four-wave ones (4, the default), interleaved in one process.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4m}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 300 python3 scripts/ab_fine.py 4,6,7 256k > $O/ab_256k.json 2> $O/ab.err && \
timeout -k 10 300 python3 scripts/ab_fine.py 4,6,7 1M+contacts > $O/ab_1M.json 2>> $O/ab.err && \
timeout -k 10 400 python3 scripts/ab_fine.py 4,6,7 4M-tet > $O/ab_4M.json 2>> $O/ab.err
echo "exit $?"
