set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fused}; mkdir -p $O; export TMPDIR=/tmp; cd $R
for c in 1 0; do echo "serial $c" >> $O/prep.log; MAS_PREP_SERIAL=$c timeout -k 10 100 python scripts/dev/prep_only.py 1M+contacts 4 >> $O/prep.log 2>&1 || exit 1; done
echo "serial 1 1M" >> $O/prep.log; MAS_PREP_SERIAL=1 timeout -k 10 100 python scripts/dev/prep_only.py 1M 3 >> $O/prep.log 2>&1 || exit 1
cd /tmp && MAS_PREP_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/trace.log 2>&1
rc=$?; grep -v amdgpu.ids $O/prep.log; exit $rc
