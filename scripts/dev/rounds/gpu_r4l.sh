# (MAS_OD_FIRST was removed after this measurement: profiles/round4/prepare/odfirst/)
# Round 4: od before the coarse contact records (MAS_OD_FIRST) with the CU
# reserve re-swept -- bitwise check (ab_prepare, one process), then steady-state
# Prepare per setting in separate processes (the CU mask is per process).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4l}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 300 python3 scripts/ab_prepare.py MAS_OD_FIRST=0 MAS_OD_FIRST=1 --config 1M+contacts > $O/ab_bitwise.json 2> $O/ab.err && \
for cfg in "0 32" "1 32" "1 16" "1 24" "0 32" "1 32"; do set -- $cfg; \
  MAS_OD_FIRST=$1 MAS_PREP_CU_RESERVE=$2 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/odfirst$1_rsv$2_$RANDOM.log 2>&1 || exit 1; done
echo "exit $?"
