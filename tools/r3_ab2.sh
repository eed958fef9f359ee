set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_errors.py tests/test_gpu_parity.py -x -q -m gpu -k "errors or panel or shared or termination" --timeout 120 --timeout-method thread > gpurun_out/r3_ab2_tests.log 2>&1 || { tail -30 gpurun_out/r3_ab2_tests.log; exit 1; }
tail -2 gpurun_out/r3_ab2_tests.log
for rep in 1 2 3; do
  for v in base cur cur2 spd4; do
    GPAD_LIB=$PWD/tools/abl/$v.so timeout -k 10 120 python3 tools/microbench.py --reps 3 --case panel,200,200,8192,200 --case panel,200,200,4096,200 2>gpurun_out/ab_mb.err | python3 -c "import json,sys; print('$v rep $rep mb', ' '.join(f\"B={d['batch']}:{d['us_per_iter']}us\" for d in map(json.loads, sys.stdin)))"
  done
done
BENCH_ARGS="--no-cpu --no-extra --steps 10" timeout -k 10 600 bash tools/ab.sh 2 "base|tools/abl/base.so|" "cur2|tools/abl/cur2.so|" "spd4|tools/abl/spd4.so|"
