# Round 4: sharded Prepare with od in the early path (tests, one rank);
# in-kernel timeline of the one-launch coarse form (grouped level 3)
# at 1M + contacts and 4M tet (probe build, lib/libmas_amd_probe.so); then, on
# the same box, the 4M fine kernel interleaved in one process with three
# handles (scripts/ab_fine.py) against one handle per process (fine_loop.py).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-probe4}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_prepare_paths.py tests/test_gpu_restrict.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
PREP_SHARD=3,8 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/rank3.log 2>&1 && \
timeout -k 10 200 python3 scripts/dev/probe_coarse1.py 1M+contacts > $O/probe_1M.txt 2>&1 && \
timeout -k 10 300 python3 scripts/dev/probe_coarse1.py 4M-tet > $O/probe_4M.txt 2>&1 && \
timeout -k 10 300 python3 scripts/ab_fine.py 1,4 4M-tet > $O/ab_4M.json 2> $O/ab.err && \
MAS_FINE_VARIANT=1 timeout -k 10 300 python3 scripts/dev/fine_loop.py 4M-tet 400 > $O/loop_4M_v1.json 2>> $O/ab.err && \
MAS_FINE_VARIANT=4 timeout -k 10 300 python3 scripts/dev/fine_loop.py 4M-tet 400 > $O/loop_4M_v4.json 2>> $O/ab.err && \
timeout -k 10 300 python3 scripts/ab_fine.py 4,1 4M-tet > $O/ab_4M_rev.json 2>> $O/ab.err && \
timeout -k 10 300 python3 scripts/ab_env.py MAS_C1_CHUNK=0 MAS_C1_CHUNK=1 --config 1M+contacts > $O/ab_c1chunk_1M.json 2>> $O/ab.err && \
timeout -k 10 400 python3 scripts/ab_env.py MAS_C1_CHUNK=0 MAS_C1_CHUNK=1 --config 4M-tet > $O/ab_c1chunk_4M.json 2>> $O/ab.err && \
cd /tmp && MAS_FINE_VARIANT=4 timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum GRBM_GUI_ACTIVE GRBM_UTCL2_BUSY -d $O/4M-tet_v4/p3 -o run --output-format csv -- python3 $R/scripts/dev/fine_loop.py 4M-tet 10 > $O/4M-tet_v4.p3.log 2>&1 && \
MAS_FINE_VARIANT=4 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/4M-tet_v4/p1 -o run --output-format csv -- python3 $R/scripts/dev/fine_loop.py 4M-tet 10 > $O/4M-tet_v4.p1.log 2>&1
echo "exit $?"
