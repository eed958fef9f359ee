# round-3 call: pair-layout wave order (role index reversed so the double waves are the youngest)
# o1 = reversed in pair mode, o2 = reversed in pair and one-panel mode; parity on o1/o2, anatomy, A/Bs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in o1 o2; do
  GPAD_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py tests/test_errors.py -x -q -k "panel or pair or c4 or c3 or handoff" --timeout 200 --timeout-method thread > gpurun_out/r3o_tests_$v.log 2>&1 || { tail -30 gpurun_out/r3o_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r3o_tests_$v.log)"
done
for v in stamp stamp_o1; do
  GPAD_LIB=$PWD/tools/abl/$v.so timeout -k 10 120 python3 tools/stamp_panel.py --batch 8192 > gpurun_out/r3o_$v.txt 2>&1
  cat gpurun_out/r3o_$v.txt
done
bash tools/ab.sh -t micro 3 "base|tools/abl/base.so|" "o1|tools/abl/o1.so|" "o2|tools/abl/o2.so|" > gpurun_out/r3o_ab.txt 2>&1
bash tools/ab.sh 3 "base|tools/abl/base.so|" "o1|tools/abl/o1.so|" "o2|tools/abl/o2.so|" >> gpurun_out/r3o_ab.txt 2>&1
cat gpurun_out/r3o_ab.txt
