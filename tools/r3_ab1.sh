set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in base e3 cur; do
    GPAD_LIB=$PWD/tools/abl/$v.so timeout -k 10 120 python3 tools/microbench.py --reps 3 --case panel,200,200,8192,200 --case panel,200,200,4096,200 2>gpurun_out/ab_mb.err | python3 -c "import json,sys; print('$v rep $rep mb', ' '.join(f\"B={d['batch']}:{d['us_per_iter']}us\" for d in map(json.loads, sys.stdin)))"
  done
done
BENCH_ARGS="--no-cpu --no-extra --steps 10" timeout -k 10 600 bash tools/ab.sh 2 "base|tools/abl/base.so|" "e3|tools/abl/e3.so|" "cur|tools/abl/cur.so|"
