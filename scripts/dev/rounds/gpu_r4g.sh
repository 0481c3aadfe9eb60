# (lib/libmas_amd_ab_split3.so was a one-off build of 96b66d9 for this A/B; results in profiles/round4/ab/)
# Round 4: the one-hand-off level-3 wave (solve3_wave) and the deferred
# early-path join: parity tests, apply A/B against the previous build
# (lib/libmas_amd_ab_split3.so: fold waves + level-3 solve waves), Prepare
# (whole and one world-8 rank) with kernel traces; PCG with the residual
# replacement inside the SpMV launch vs the previous build.  One && chain.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4g}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_restrict.py tests/test_gpu_parity.py tests/test_gpu_prepare_paths.py tests/test_gpu_incremental.py tests/test_gpu_shard.py tests/test_gpu_blob.py tests/test_gpu_factor_mfma.py tests/test_gpu_failure.py tests/test_gpu_pcg.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
for i in 1 2 3; do \
  MAS_LIB_NAME=libmas_amd_ab_split3.so timeout -k 10 200 python3 scripts/dev/fine_loop.py 1M+contacts 400 >> $O/ab_1M.jsonl 2>> $O/ab.err && \
  timeout -k 10 200 python3 scripts/dev/fine_loop.py 1M+contacts 400 >> $O/ab_1M.jsonl 2>> $O/ab.err || exit 1; done && \
for i in 1 2; do \
  MAS_LIB_NAME=libmas_amd_ab_split3.so timeout -k 10 300 python3 scripts/dev/fine_loop.py 4M-tet 100 >> $O/ab_4M.jsonl 2>> $O/ab.err && \
  timeout -k 10 300 python3 scripts/dev/fine_loop.py 4M-tet 100 >> $O/ab_4M.jsonl 2>> $O/ab.err || exit 1; done && \
for i in 1 2; do \
  MAS_LIB_NAME=libmas_amd_ab_split3.so timeout -k 10 200 python3 scripts/dev/pcg_only.py 1M+contacts 2 >> $O/pcg_ab_old.log 2>&1 && \
  timeout -k 10 200 python3 scripts/dev/pcg_only.py 1M+contacts 2 >> $O/pcg_ab_new.log 2>&1 || exit 1; done && \
timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 8 > $O/noprof.log 2>&1 && \
PREP_SHARD=3,8 timeout -k 10 200 python3 scripts/dev/prep_only.py 1M+contacts 6 > $O/noprof_rank3of8.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prep -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/prep.log 2>&1 && \
python3 $R/scripts/dev/prepare_timeline.py $O/prep k_stencil_flags k_factor_rb > $O/timeline.txt 2>&1 && \
PREP_SHARD=3,8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prep_rank -o run --output-format csv -- python3 $R/scripts/dev/prep_only.py 1M+contacts 3 > $O/prep_rank.log 2>&1 && \
python3 $R/scripts/dev/prepare_timeline.py $O/prep_rank k_stencil_flags k_factor_rb > $O/timeline_rank3of8.txt 2>&1
echo "exit $?"
