# round-3 call: cold-start seed GEMM skip -- panel parity subset, C4 A/B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py tests/test_errors.py tests/test_boundary.py -x -q -k "panel or pair or c4 or c3 or handoff or finisher or boundary or solve" --timeout 200 --timeout-method thread > gpurun_out/r3s_tests.log 2>&1 || { tail -30 gpurun_out/r3s_tests.log; exit 1; }
tail -1 gpurun_out/r3s_tests.log
bash tools/ab.sh 4 "base|tools/abl/base.so|" "skip||" > gpurun_out/r3s_ab.txt 2>&1
cat gpurun_out/r3s_ab.txt
