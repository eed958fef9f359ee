# Round-2 GPU check: the new boundary / multi-rank / config tests first, then the whole -m gpu
# suite, then the default bench line.  Every GPU step under its own time limit, chained with &&.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2b}
timeout -k 10 400 python -u -m pytest tests/test_boundary.py tests/test_dist_gpu.py tests/test_configs.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_new.log 2>&1 || { tail -40 gpurun_out/${T}_new.log; exit 1; }
tail -3 gpurun_out/${T}_new.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 400 gpurun_out/${T}_bench.json
