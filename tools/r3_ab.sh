set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_errors.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3i_err.log 2>&1 || { tail -30 gpurun_out/r3i_err.log; exit 1; }
tail -1 gpurun_out/r3i_err.log
MICRO_ARGS="--reps 3 --case panel,200,200,8192,200 --case panel,200,200,4096,200 --case panel,200,200,64,200" bash tools/ab.sh -t micro 3 "base|tools/abl/base.so|" "cur3|tools/abl/cur3.so|" "cur4|tools/abl/cur4.so|" > gpurun_out/r3i_ab.txt 2>&1
bash tools/ab.sh 2 "base|tools/abl/base.so|" "cur4|tools/abl/cur4.so|" >> gpurun_out/r3i_ab.txt 2>&1
cat gpurun_out/r3i_ab.txt
