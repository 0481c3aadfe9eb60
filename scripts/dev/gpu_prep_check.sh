# Full GPU tests, then steady-state Prepare timings: bash scripts/dev/gpu_prep_check.sh <out>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-prepcheck}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for cfg in 1M+contacts 4M-tet; do echo $cfg; timeout -k 10 100 python scripts/dev/prep_only.py $cfg 3 2>&1 | grep prepare || exit 1; done
