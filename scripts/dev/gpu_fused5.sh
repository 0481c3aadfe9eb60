set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fused}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "factor_kernels or small_configs or all_contact or 256k" > $O/pt1.log 2>&1 || { tail -30 $O/pt1.log; exit 1; }
tail -2 $O/pt1.log
bash scripts/dev/gpu_ab.sh $1 1M+contacts libmas_amd.so libmas_amd_ab_slowdiv.so
