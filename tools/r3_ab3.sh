set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GPAD_LIB=$PWD/tools/abl/stamp.so timeout -k 10 120 python3 tools/stamp_panel.py --batch 8192 > gpurun_out/r3_stamp_8192.txt 2>&1 || { tail gpurun_out/r3_stamp_8192.txt; exit 1; }
cat gpurun_out/r3_stamp_8192.txt
GPAD_LIB=$PWD/tools/abl/stamp.so timeout -k 10 120 python3 tools/stamp_panel.py --batch 4096 > gpurun_out/r3_stamp_4096.txt 2>&1 || { tail gpurun_out/r3_stamp_4096.txt; exit 1; }
cat gpurun_out/r3_stamp_4096.txt
for rep in 1 2 3; do
  for v in base cur2 nodrop; do
    GPAD_LIB=$PWD/tools/abl/$v.so timeout -k 10 120 python3 tools/microbench.py --reps 3 --case panel,200,200,8192,200 --case panel,200,200,4096,200 2>gpurun_out/ab_mb.err | python3 -c "import json,sys; print('$v rep $rep mb', ' '.join(f\"B={d['batch']}:{d['us_per_iter']}us\" for d in map(json.loads, sys.stdin)))"
  done
done
