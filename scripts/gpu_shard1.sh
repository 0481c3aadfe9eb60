set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s1; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 5 --dist-backend gloo > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err
timeout -k 10 600 python bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err
