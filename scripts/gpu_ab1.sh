set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python scripts/ab_fine.py 0,1,2 > gpurun_out/ab1.json 2> gpurun_out/ab1.err
