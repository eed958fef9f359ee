# Round-2: async phase-plan refresh check + bench + profile
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "plan or phased or async" > gpurun_out/r2p_tests.log 2>&1 || { tail -30 gpurun_out/r2p_tests.log; exit 1; }
tail -2 gpurun_out/r2p_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r2p_bench.json 2> gpurun_out/r2p_bench.err || { tail -20 gpurun_out/r2p_bench.err; exit 1; }
timeout -k 10 900 bash tools/profile.sh r02 > gpurun_out/r2p_prof.log 2>&1 || { tail -20 gpurun_out/r2p_prof.log; exit 1; }
tail -c 300 gpurun_out/r2p_prof.log
