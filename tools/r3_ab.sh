# round-3 call: finisher parity tests on the tree, duo anatomy and A/Bs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1 || { tail -30 gpurun_out/r3x_tests.log; exit 1; }
tail -1 gpurun_out/r3x_tests.log
for v in cur6 duo4 duo5; do GPAD_LIB=$PWD/tools/abl/$v.so timeout -k 10 120 python3 tools/duo_solo.py 2>/dev/null | sed "s/^/$v /"; done
bash tools/ab.sh 3 "cur6|tools/abl/cur6.so|" "duo4|tools/abl/duo4.so|" "duo5|tools/abl/duo5.so|" > gpurun_out/r3x_ab.txt 2>&1
cat gpurun_out/r3x_ab.txt
