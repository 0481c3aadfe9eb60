set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-mfma}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_factor_mfma.py -x -v -s --timeout 200 --timeout-method thread > $O/pt.log 2>&1 || { tail -30 $O/pt.log; exit 1; }
grep -E "worst|rel. error|passed" $O/pt.log
for v in 4 5; do echo "variant $v"; MAS_PREP_SERIAL=1 MAS_FACTOR_VARIANT=$v timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 3 2>&1 | grep prepare || exit 1; done
cd /tmp && MAS_PREP_SERIAL=1 MAS_FACTOR_VARIANT=5 timeout -s KILL 120 rocprofv3 --kernel-include-regex k_factor_fused --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA -d $O/p5 -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 2 > $O/p5.log 2>&1
echo "pmc $?"
