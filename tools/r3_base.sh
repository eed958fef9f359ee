# round-3 first GPU call: the new error-path tests, every -m gpu test, a short bench, a timeline
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_errors.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3a_err_tests.log 2>&1 || { tail -40 gpurun_out/r3a_err_tests.log; exit 1; }
tail -3 gpurun_out/r3a_err_tests.log
timeout -k 10 200 python -u bench.py --no-cpu --no-extra --steps 20 > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err || { tail -20 gpurun_out/r3a_bench.err; exit 1; }
tail -c 400 gpurun_out/r3a_bench.json
TAG=r3a_tl timeout -k 10 320 bash tools/tl_run.sh > /dev/null
tail -30 gpurun_out/r3a_tl_timeline.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1 || { tail -30 gpurun_out/r3a_tests.log; exit 1; }
tail -2 gpurun_out/r3a_tests.log
