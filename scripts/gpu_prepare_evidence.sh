# Prepare evidence on one MI355X: PMC of the fused level-0 kernel in both
# formations (matrix-core default, MAS_FACTOR_VARIANT=4 = the bitwise VALU one),
# and kernel traces of steady-state Prepares (serial and overlapped).
#   bash scripts/gpu_prepare_evidence.sh <out> [config]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-prep_ev}; C=${2:-1M+contacts}; mkdir -p $O; export TMPDIR=/tmp; cd /tmp
K=k_factor_fused
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES"
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc $SQ -d $O/mfma -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $C 2 > $O/mfma.log 2>&1 && \
MAS_FACTOR_VARIANT=4 timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc $SQ -d $O/valu -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $C 2 > $O/valu.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $C 2 > $O/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $C 2 > $O/write.log 2>&1 && \
MAS_PREP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $C 3 > $O/serial.log 2>&1 && \
MAS_PREP_SERIAL=1 MAS_FACTOR_VARIANT=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial_valu -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $C 3 > $O/serial_valu.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/default -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py $C 3 > $O/default.log 2>&1 && \
cd $R && timeout -k 10 300 python3 scripts/dev/prep_only.py $C 6 > $O/noprof.log 2>&1
rc=$?; tail -2 $O/noprof.log; echo "exit $rc"; exit $rc
