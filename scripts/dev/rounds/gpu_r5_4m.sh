# Round 5, verdict item 4: the 4M tet fine kernel (default variant,
# k_solve_fine<3,4,false,2>) under rocprofv3: two kernel traces of the bench
# command, FETCH_SIZE / WRITE_SIZE passes, and the latency / DRAM-stall
# counters, each pass its own run.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5_4m; mkdir -p $O; export TMPDIR=/tmp
P3="TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum GRBM_GUI_ACTIVE"
P5="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_sum TCP_PENDING_STALL_CYCLES_sum"
B="$R/bench.py --config 4M-tet --no-cpu-baseline --no-pcg"
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace1 -o run --output-format csv -- python3 $B --steps 100 > $O/bench_trace1.json 2> $O/trace1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace2 -o run --output-format csv -- python3 $B --steps 100 > $O/bench_trace2.json 2> $O/trace2.err && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/p1 -o run --output-format csv -- python3 $B --steps 20 --warmup 5 > $O/p1.json 2> $O/p1.err && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/p2 -o run --output-format csv -- python3 $B --steps 20 --warmup 5 > $O/p2.json 2> $O/p2.err && \
timeout -s KILL 300 rocprofv3 --pmc $P3 -d $O/p3 -o run --output-format csv -- python3 $B --steps 20 --warmup 5 > $O/p3.json 2> $O/p3.err && \
timeout -s KILL 300 rocprofv3 --pmc $P5 -d $O/p5 -o run --output-format csv -- python3 $B --steps 20 --warmup 5 > $O/p5.json 2> $O/p5.err && \
cd $R && timeout -k 10 300 python3 bench.py --config 4M-tet --no-cpu-baseline --no-pcg > $O/bench_plain.json 2> $O/bench_plain.err
echo "exit $?"
