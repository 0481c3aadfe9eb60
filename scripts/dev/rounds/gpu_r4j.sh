# Round 4: poll delay of the one-launch coarse form's waiting waves with the
# grouped level 3 and XCD-chunked banks (ab_env, interleaved in one process).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r4j}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 300 python3 scripts/ab_env.py MAS_C1_POLL_DELAY=0 MAS_C1_POLL_DELAY=1 MAS_C1_POLL_DELAY=2 MAS_C1_POLL_DELAY=3 --config 1M+contacts > $O/ab_poll_1M.json 2> $O/ab.err && \
timeout -k 10 400 python3 scripts/ab_env.py MAS_C1_POLL_DELAY=0 MAS_C1_POLL_DELAY=2 MAS_C1_POLL_DELAY=4 --config 4M-tet > $O/ab_poll_4M.json 2>> $O/ab.err && \
timeout -k 10 300 python3 scripts/ab_env.py MAS_C1_POLL_DELAY=0 MAS_C1_POLL_DELAY=1 MAS_C1_POLL_DELAY=2 --config 256k > $O/ab_poll_256k.json 2>> $O/ab.err
echo "exit $?"
