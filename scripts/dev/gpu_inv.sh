set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-inv}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "restrict or chain or shard" > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
tail -1 $O/pt.log
bash scripts/dev/gpu_ab_apply.sh $1 1M+contacts libmas_amd.so libmas_amd_ab_early.so
