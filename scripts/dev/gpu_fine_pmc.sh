# Round 4, verdict item 4: why the 4M fine kernel streams slower than 1M.
# Per config (1M + contacts, 4M tet) and fine variant (1: the default, 4-wave
# workgroups; 3: one-wave workgroups; 4: 1 with XCD-chunked workgroups): an
# event-timed A/B of the variants,
# a kernel trace, then one rocprofv3 --pmc pass per counter group (each within
# the per-block limits: FETCH_SIZE alone, WRITE_SIZE alone, translation +
# TCC, SQ occupancy/stall, TCC/TCP stall).  One && chain.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fine_pmc}; mkdir -p $O; export TMPDIR=/tmp
P3="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY"
P4="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD TA_BUSY_avr TA_BUSY_max"
P5="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"
cd $R && timeout -k 10 400 python3 scripts/ab_fine.py 1,3,4 4M-tet > $O/ab_4M.json 2> $O/ab_4M.err && \
timeout -k 10 200 python3 scripts/ab_fine.py 1,3,4 1M+contacts > $O/ab_1M.json 2> $O/ab_1M.err && \
cd /tmp && \
for cv in 1M+contacts:1 4M-tet:1 4M-tet:3; do cfg=${cv%:*}; v=${cv#*:}; t=${cfg%%+*}_v$v; \
  MAS_FINE_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$t/trace -o run --output-format csv -- python3 $R/scripts/dev/fine_loop.py $cfg 20 > $O/$t.trace.log 2>&1 && \
  MAS_FINE_VARIANT=$v timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/$t/p1 -o run --output-format csv -- python3 $R/scripts/dev/fine_loop.py $cfg 10 > $O/$t.p1.log 2>&1 && \
  MAS_FINE_VARIANT=$v timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/$t/p2 -o run --output-format csv -- python3 $R/scripts/dev/fine_loop.py $cfg 10 > $O/$t.p2.log 2>&1 && \
  MAS_FINE_VARIANT=$v timeout -s KILL 300 rocprofv3 --pmc $P3 -d $O/$t/p3 -o run --output-format csv -- python3 $R/scripts/dev/fine_loop.py $cfg 10 > $O/$t.p3.log 2>&1 && \
  MAS_FINE_VARIANT=$v timeout -s KILL 300 rocprofv3 --pmc $P4 -d $O/$t/p4 -o run --output-format csv -- python3 $R/scripts/dev/fine_loop.py $cfg 10 > $O/$t.p4.log 2>&1 && \
  MAS_FINE_VARIANT=$v timeout -s KILL 300 rocprofv3 --pmc $P5 -d $O/$t/p5 -o run --output-format csv -- python3 $R/scripts/dev/fine_loop.py $cfg 10 > $O/$t.p5.log 2>&1 || exit 1; \
done
echo "exit $?"
