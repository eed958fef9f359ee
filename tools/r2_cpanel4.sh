set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_condensed.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2cp_tests.log 2>&1 || { tail -40 gpurun_out/r2cp_tests.log; exit 1; }
tail -2 gpurun_out/r2cp_tests.log
timeout -k 10 400 python3 tools/cond_take_sweep.py > gpurun_out/cond_take3.jsonl 2> gpurun_out/cond_take3.err
cut -c1-130 gpurun_out/cond_take3.jsonl
