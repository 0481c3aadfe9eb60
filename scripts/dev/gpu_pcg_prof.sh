set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pcg.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_trace.log 2>&1
rc=$?; tail -3 $O/pytest.log; cat $O/pcg.log | tail -5; echo "exit $rc"; exit $rc
