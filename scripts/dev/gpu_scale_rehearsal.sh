# N > 1 rehearsal of bench.py on one GPU (gloo hook transport): bash scripts/dev/gpu_scale_rehearsal.sh <out>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-scale}; mkdir -p $O; export TMPDIR=/tmp; cd $R
for n in 2 4; do
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 50 --warmup 10 --dist-backend gloo > $O/b$n.json 2> $O/b$n.err || { tail -20 $O/b$n.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/b$n.json').read().strip().splitlines()[-1]); print($n, d['value'], d['ms_per_step'], d['prepare_ms'], d.get('prepare_scope'), d.get('shard_check'), d['config']['parallelism'])"
done
