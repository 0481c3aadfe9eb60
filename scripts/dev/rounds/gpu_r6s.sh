# Round 6: kernel trace of a steady-state Prepare (device Hessian) on the final schedule (no CU mask, chunked fused kernel).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6s}; mkdir -p $O; export TMPDIR=/tmp
cd /tmp && \
PREP_DEVICE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/prep.log 2>&1 && \
cd $R && python3 scripts/dev/prepare_timeline.py $O/tr k_stencil_flags k_readback > $O/timeline.txt 2>&1
rc=$?
grep prepare $O/prep.log | cut -c1-80
tail -3 $O/timeline.txt
echo "exit $rc"
exit $rc
