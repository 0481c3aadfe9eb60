# Kernel traces of steady-state Prepares: bash scripts/dev/gpu_trace_prep.sh <out> <config>
# (serial: every kernel on one stream, each kernel's own time; default: the real overlapped timeline)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-traceprep}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
MAS_PREP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $2 3 > $O/serial.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/default -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $2 3 > $O/default.log 2>&1 && \
timeout -k 10 300 python3 $R/scripts/dev/prep_only.py $2 5 > $O/noprof.log 2>&1
echo "exit $?"
