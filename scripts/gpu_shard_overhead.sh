# Cost of the sharded apply path on one GPU (run through gpurun): the unsharded
# apply, the sharded path with a one-rank RCCL group launched eagerly, and the
# same replayed as a captured HIP graph -- on the 1M workload (GPU-bound) and
# on 256k (closer to a per-rank share of 1M at N = 4, where the host launch
# cost shows).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/shardov; mkdir -p $O
for c in 1M+contacts 256k; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline --no-pcg > $O/unsharded_$c.json 2> $O/e1.err && \
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline --no-pcg --sharded > $O/sharded_eager_$c.json 2> $O/e2.err && \
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline --no-pcg --sharded --graph > $O/sharded_graph_$c.json 2> $O/e3.err || exit 1
done
echo "exit 0"
