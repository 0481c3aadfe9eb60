set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fused}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 5 > $O/prep.log 2>&1 && \
timeout -k 10 100 python scripts/dev/prep_only.py 1M 3 >> $O/prep.log 2>&1 && \
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/trace.log 2>&1) && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; cat $O/prep.log; tail -3 $O/pytest_gpu.log; exit $rc
