# bench.py once per BASELINE config (the headline config comes from
# gpu_profile.sh): bash scripts/gpu_configs.sh <out-name>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-configs}
mkdir -p $O
cd $R
for c in 10k 256k 1M 4M-tet; do
  timeout -k 10 400 python bench.py --config $c --no-pcg --cpu-steps 3 > $O/$c.json 2> $O/$c.err || exit $?
done
echo "exit 0"
