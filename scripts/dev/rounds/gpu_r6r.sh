# Round 6: the PCG SpMV's mirrored layout (MAS_PCG_SYM): PCG tests, then an interleaved A/B at 1M + contacts and a
# kernel-stats trace of one solve pair.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r6r}; mkdir -p $O; export TMPDIR=/tmp
cd $R && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_pcg.py -k "mirrored or fused" -x -v --timeout 120 --timeout-method thread > $O/pytest_pcg.log 2>&1 && \
for i in 1 2; do \
  for k in 0 1; do \
    MAS_PCG_SYM=$k timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_sym$k.$i.txt 2>&1 || exit 1; \
  done; \
done && \
cd /tmp && MAS_PCG_SYM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_sym1 -o run --output-format csv -- python3 $R/scripts/dev/pcg_only.py 1M+contacts 1 > $O/trace_sym1.log 2>&1 && \
MAS_PCG_SYM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_sym0 -o run --output-format csv -- python3 $R/scripts/dev/pcg_only.py 1M+contacts 1 > $O/trace_sym0.log 2>&1
rc=$?
tail -3 $O/pytest_pcg.log
for f in $O/pcg_sym*.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
grep -h "k_pcg_spmv" $O/trace_sym*/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
echo "exit $rc"
exit $rc
