set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fp_tests.log 2>&1 || { tail -40 gpurun_out/fp_tests.log; exit 1; }
tail -3 gpurun_out/fp_tests.log
timeout -k 10 240 python -u tools/flat_bench.py > gpurun_out/fp_bench.jsonl 2>&1
cat gpurun_out/fp_bench.jsonl
