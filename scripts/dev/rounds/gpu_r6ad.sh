# Round 6 final: every config once more (bench with the median-of-9 Prepare), then the full evidence script.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6ad}; mkdir -p $O; export TMPDIR=/tmp
cd $R && bash scripts/dev/rounds/gpu_r6q.sh ${1:-r6ad}/q && bash scripts/dev/rounds/gpu_r6e.sh ${1:-r6ad}/e
