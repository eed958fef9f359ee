#!/bin/bash
# plan model pricing the one-panel relay (3.5 chains): fresh-input C4 solve, interleaved A/B
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for v in base rmodel; do
  GPAD_LIB=$PWD/tools/abx/$v.so timeout -k 10 120 python3 tools/plan_sweep.py --one --fresh --reps 16 >> gpurun_out/rm_sweep.jsonl 2>gpurun_out/rm_err.log || { tail gpurun_out/rm_err.log; exit 1; }
  tail -1 gpurun_out/rm_sweep.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['best_ms'], d['median_ms'], d['plan']['ends'], d['plan']['fins'])"
done
done
