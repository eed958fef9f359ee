set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/microbench.py --reps 3 --case panel,200,200,2816,100 --case panel,200,200,3968,100 --case panel,200,200,4096,100 --case panel,200,200,4112,100 --case panel,200,200,8192,100 --case panel,200,200,1024,100 --case panel,200,200,256,100 > gpurun_out/r3_probe_mb.jsonl
cat gpurun_out/r3_probe_mb.jsonl
timeout -k 10 300 python -u -m pytest tests/test_value.py tests/test_errors.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_probe_tests.log 2>&1 || { tail -30 gpurun_out/r3_probe_tests.log; exit 1; }
tail -3 gpurun_out/r3_probe_tests.log
TAG=r3_probe_tl timeout -k 10 320 bash tools/tl_run.sh > /dev/null
head -12 gpurun_out/r3_probe_tl_timeline.txt
