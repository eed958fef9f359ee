#!/bin/bash
# C4 fresh-input solve time vs the plan model's finisher cost scale, more reps, interleaved
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for fc in 100 200 300; do
  GPAD_PLAN_FIN_COST=$fc timeout -k 10 120 python3 tools/plan_sweep.py --one --fresh --reps 16 >> gpurun_out/fc2_sweep.jsonl 2>gpurun_out/fc2_err.log || { tail gpurun_out/fc2_err.log; exit 1; }
  tail -1 gpurun_out/fc2_sweep.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($fc, d['best_ms'], d['median_ms'], d['plan']['ends'])"
done
done
