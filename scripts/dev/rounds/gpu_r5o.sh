# Round 5: host-side view of the Prepare's early path (HIP API trace + kernel trace), to find
# the ~60 us idle gap on both queues before the level-0 contact scan.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5o; mkdir -p $O; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/trace.log 2>&1
echo "exit $?"; ls -R $O | head
