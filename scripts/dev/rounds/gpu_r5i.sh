# Round 5: PCG r.z partial count (fine-kernel workgroup size in the PCG's applies), interleaved processes.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5i; mkdir -p $O; export TMPDIR=/tmp
cd $R || exit 1
for rep in 1 2; do
for w in 2 4 8; do
  MAS_RZ_WPB=$w timeout -k 10 300 python scripts/dev/pcg_only.py 1M+contacts 2 > $O/pcg_wpb${w}_$rep.txt 2>&1 || { tail -5 $O/pcg_wpb${w}_$rep.txt; exit 1; }
  echo "wpb=$w rep=$rep $(grep mas: $O/pcg_wpb${w}_$rep.txt | tr '\n' ' ')"
done
done
MAS_RZ_WPB=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_pcg.py -x -q --timeout 200 --timeout-method thread > $O/pytest_wpb8.log 2>&1; tail -1 $O/pytest_wpb8.log
