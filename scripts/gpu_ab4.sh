set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab4; mkdir -p $O
timeout -k 10 600 python scripts/ab_env.py "MAS_OVERLAP=0" "MAS_OVERLAP=2,MAS_COARSE_CUS=16" "MAS_OVERLAP=2,MAS_COARSE_CUS=32" "MAS_OVERLAP=2,MAS_COARSE_CUS=64" > $O/ab_overlap.json 2> $O/ab_overlap.err
echo "exit $?"
