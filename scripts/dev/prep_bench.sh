mkdir -p gpurun_out/r2_prep2 && cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && \
timeout -k 10 300 python bench.py --sharded --steps 50 --warmup 10 --no-cpu-baseline --no-pcg > gpurun_out/r2_prep2/b1.json 2> gpurun_out/r2_prep2/b1.err && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 10 --dist-backend gloo > gpurun_out/r2_prep2/b2.json 2> gpurun_out/r2_prep2/b2.err
