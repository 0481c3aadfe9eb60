# A/B of library builds on the prepare: bash scripts/dev/gpu_ab.sh <out> <config> <lib names...>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab}; CFG=$2; shift 2; mkdir -p $O; export TMPDIR=/tmp; cd $R
for rep in 1 2; do for lib in "$@"; do echo "lib $lib" >> $O/prep.log; MAS_PREP_SERIAL=1 MAS_LIB_NAME=$lib timeout -k 10 100 python scripts/dev/prep_only.py $CFG 4 >> $O/prep.log 2>&1 || exit 1; done; done
grep -v amdgpu.ids $O/prep.log
