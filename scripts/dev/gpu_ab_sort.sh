# Look-back-free sort/scan (rsort.hip): unit tests, Prepare parity, then Prepare times
# for MAS_SORT (1 own, 0 rocprim) x MAS_FUSED_PULL (0 grid-per-block, 4 background waves)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-absort}; mkdir -p $O; export TMPDIR=/tmp; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_rsort.py -x -q --timeout 200 --timeout-method thread > $O/rsort.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blob.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for c in 1M+contacts 1M 256k 4M-tet; do for sp in "1 0" "1 4" "1 5" "1 6"; do set -- $sp
  MAS_SORT=$1 MAS_FUSED_PULL=$2 timeout -k 10 200 python scripts/dev/prep_only.py $c 4 > $O/prep_${c}_s$1_p$2.log 2>&1 || exit 1
done; done
echo "exit $?"
