# A/B of library knobs on one MI355X (run through gpurun), e.g.
#   bash scripts/gpu_ab.sh apply  "MAS_OVERLAP=0" "MAS_OVERLAP=1"
#   bash scripts/gpu_ab.sh prepare "MAS_FACTOR_VARIANT=0" "MAS_FACTOR_VARIANT=2"
# Results: gpurun_out/ab_<kind>.json (copied to profiles/round1/ab/).
set -o pipefail
cd $GRAFT_REPO_ROOT
kind=$1; shift
mkdir -p gpurun_out
if [ "$kind" = prepare ]; then
  timeout -k 10 600 python scripts/ab_prepare.py "$@" > gpurun_out/ab_prepare.json 2> gpurun_out/ab_prepare.err
else
  timeout -k 10 600 python scripts/ab_env.py "$@" > gpurun_out/ab_apply.json 2> gpurun_out/ab_apply.err
fi
echo "exit $?"
