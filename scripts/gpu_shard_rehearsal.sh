# Rehearse bench.py --gpus N on a one-GPU box (run through gpurun): N ranks
# share cuda:0 and exchange the level-1 segments over gloo (RCCL needs one
# GPU per rank; the driver runs the real N-GPU case with nccl).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/shard; mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 5 --dist-backend gloo > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 50 --warmup 5 --dist-backend gloo > $O/bench_n4_gloo.json 2> $O/bench_n4_gloo.err
echo "exit $?"
