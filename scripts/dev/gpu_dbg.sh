cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/dbg && \
timeout -k 10 120 python scripts/dev/dbg_coarse1.py 256 4 > gpurun_out/dbg/dbg.txt 2>&1
echo "exit $?"
