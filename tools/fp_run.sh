set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fp_tests.log 2>&1 || { tail -40 gpurun_out/fp_tests.log; exit 1; }
tail -3 gpurun_out/fp_tests.log
timeout -k 10 240 python -u tools/flat_bench.py > gpurun_out/fp_bench.jsonl 2>&1
cat gpurun_out/fp_bench.jsonl
if [ -f tools/fpt/fptime.so ]; then
  GPAD_LIB=$PWD/tools/fpt/fptime.so timeout -k 10 120 python tools/fp_time.py 4 10 8192 200 > gpurun_out/fpt_c1.txt 2>&1
  GPAD_LIB=$PWD/tools/fpt/fptime.so timeout -k 10 120 python tools/fp_time.py 4 50 8192 100 > gpurun_out/fpt_n50.txt 2>&1
  grep "^fpt" gpurun_out/fpt_c1.txt | sort -t w -k2 -n | head -16
  grep "^fpt" gpurun_out/fpt_n50.txt | sort -t w -k2 -n | head -16
fi
