set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-prio}; mkdir -p $O; export TMPDIR=/tmp; cd $R
echo "default"; timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 3 2>&1 | grep -E "prepare|prio" || exit 1
echo "serial"; MAS_PREP_SERIAL=1 timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 3 2>&1 | grep -E "prepare|prio" || exit 1
for p in 1 0; do echo "prio $p"; MAS_PREP_PRIO=$p timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 3 2>&1 | grep -E "prepare|prio" || exit 1; done
