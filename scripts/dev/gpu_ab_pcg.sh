# A/B of library builds on the PCG: bash scripts/dev/gpu_ab_pcg.sh <out> <config> <lib names...>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-abpcg}; CFG=$2; shift 2; mkdir -p $O; export TMPDIR=/tmp; cd $R
for lib in "$@"; do echo "lib $lib" >> $O/pcg.log; MAS_LIB_NAME=$lib timeout -k 10 200 python scripts/dev/pcg_only.py $CFG 2 >> $O/pcg.log 2>&1 || exit 1; done
grep -v amdgpu.ids $O/pcg.log
