set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a_tests.log 2>&1 || { tail -30 gpurun_out/r2a_tests.log; exit 1; }
tail -2 gpurun_out/r2a_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r2a_bench.json 2> gpurun_out/r2a_bench.err || { tail -20 gpurun_out/r2a_bench.err; exit 1; }
tail -c 600 gpurun_out/r2a_bench.json
