# Round 6 final: sharded Prepare ratios on the final Prepare schedule, then the full evidence script.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6ab}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 300 python scripts/dev/prep_shard.py 1M+contacts 8 3 > $O/prep_shard_1M.txt 2>&1 && \
timeout -k 10 400 python scripts/dev/prep_shard.py 4M-tet 8 3 > $O/prep_shard_4M.txt 2>&1 && \
tail -1 $O/prep_shard_1M.txt && tail -1 $O/prep_shard_4M.txt && \
bash scripts/dev/rounds/gpu_r6e.sh ${1:-r6ab}/e
