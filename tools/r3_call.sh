# round-3 call: quad finisher parity, fresh-input timeline, C4 A/B duo vs quad
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "finisher_queue" --timeout 120 --timeout-method thread > gpurun_out/r3q_fin_tests.log 2>&1 || { tail -40 gpurun_out/r3q_fin_tests.log; exit 1; }
tail -1 gpurun_out/r3q_fin_tests.log
timeout -k 10 300 python -u -m pytest tests/test_configs.py -x -v -k "c4" --timeout 200 --timeout-method thread > gpurun_out/r3q_c4_tests.log 2>&1 || { tail -40 gpurun_out/r3q_c4_tests.log; exit 1; }
tail -1 gpurun_out/r3q_c4_tests.log
TAG=tlq GPAD_QUAD=1 bash tools/tl_run.sh
bash tools/ab.sh 3 "duo||" "quad||GPAD_QUAD=1" > gpurun_out/r3q_ab.txt 2>&1
cat gpurun_out/r3q_ab.txt
