# Kernel trace of steady-state Prepares: bash scripts/dev/gpu_trace_prep.sh <out> <config>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-traceprep}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
MAS_PREP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $2 2 > $O/trace.log 2>&1
echo "exit $?"
