# Round 5, first GPU pass: the touched GPU tests, the plain-launch N > 1
# rehearsal (gloo, no wrapper), the nccl refusal on a one-GPU box, one bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5a
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "failure or restrict or facade" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --steps 50 --warmup 5 --no-cpu-baseline \
    > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo "gloo rehearsal failed"; tail -30 $O/bench_n2_gloo.err; exit 1; }
cat $O/bench_n2_gloo.json
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_n2_nccl.json 2> $O/bench_n2_nccl.err
rc=$?
echo "nccl --gpus 2 on one GPU: exit $rc"; tail -2 $O/bench_n2_nccl.err
[ $rc -eq 2 ] || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
