# A/B: coarse inverse formation VALU (default lib) vs matrix cores (ab_cmfma)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab_coarse_formation && \
timeout -k 10 300 python -u scripts/dev/ab_coarse_formation.py valu > gpurun_out/ab_coarse_formation/valu.txt 2>&1 && \
MAS_LIB_NAME=libmas_amd_ab_cmfma.so timeout -k 10 300 python -u scripts/dev/ab_coarse_formation.py mfma > gpurun_out/ab_coarse_formation/mfma.txt 2>&1 && \
timeout -k 10 300 python -u scripts/dev/ab_coarse_formation.py valu2 > gpurun_out/ab_coarse_formation/valu2.txt 2>&1 && \
MAS_LIB_NAME=libmas_amd_ab_cmfma.so timeout -k 10 300 python -u scripts/dev/ab_coarse_formation.py mfma2 > gpurun_out/ab_coarse_formation/mfma2.txt 2>&1 && \
python scripts/dev/ab_coarse_formation.py --compare valu mfma > gpurun_out/ab_coarse_formation/compare.json && \
python scripts/dev/ab_coarse_formation.py --compare valu valu2 > gpurun_out/ab_coarse_formation/compare_valu_runs.json && \
rm -f gpurun_out/ab_coarse_formation/*.npz && \
tail -n 2 gpurun_out/ab_coarse_formation/*.txt gpurun_out/ab_coarse_formation/*.json
