set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe0 && \
MAS_COARSE_MODE=2 timeout -k 10 200 python scripts/dev/probe_coarse.py 1024 4 > gpurun_out/probe0/1M.txt 2>&1
echo "exit $?"
