set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fused}; mkdir -p $O; export TMPDIR=/tmp; cd $R
for sr in 1 0; do for cfg in 1M+contacts 1M 4M-tet 256k; do echo "serial $sr $cfg" >> $O/prep.log; MAS_PREP_SERIAL=$sr timeout -k 10 100 python scripts/dev/prep_only.py $cfg 3 >> $O/prep.log 2>&1 || exit 1; done; done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -v amdgpu $O/prep.log; tail -2 $O/pytest_gpu.log; exit $rc
