# fine kernel at 4M tet: 4-wave (default) vs one-wave workgroups: bash scripts/dev/gpu_ab_fine4m.sh <out>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-abfine4m}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python scripts/ab_env.py "MAS_FINE_VARIANT=1" "MAS_FINE_VARIANT=3" --config 4M-tet --rounds 6 > $O/ab_4M-tet.json 2> $O/ab_4M.err
echo "exit $?"
