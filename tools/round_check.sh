# Full GPU check for the round: gpu tests, default bench line, rocprof profile (tools/profile.sh).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rc_tests.log 2>&1 || { tail -30 gpurun_out/rc_tests.log; exit 1; }
tail -2 gpurun_out/rc_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/rc_bench.json 2> gpurun_out/rc_bench.err || { tail -20 gpurun_out/rc_bench.err; exit 1; }
tail -c 1500 gpurun_out/rc_bench.json
timeout -k 10 900 bash tools/profile.sh r01 > gpurun_out/rc_prof.log 2>&1 || { tail -20 gpurun_out/rc_prof.log; exit 1; }
tail -c 600 gpurun_out/rc_prof.log
