# Round-2 full GPU check: every -m gpu test, the default bench line, the rocprofv3 profile
# (tools/profile.sh: kernel trace + separate PMC passes) of the C4 solves.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2f}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 900 bash tools/profile.sh r02 > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
tail -c 300 gpurun_out/${T}_prof.log
