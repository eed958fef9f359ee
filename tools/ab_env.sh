#!/bin/bash
# Interleaved A/B of library builds x environment knobs on one box:
#   bash tools/ab_env.sh REPS "name|lib|ENV=v ENV2=v" ...
REPS=$1; shift
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    IFS='|' read -r name lib envs <<< "$spec"
    v=$(env GPAD_LIB=$PWD/$lib $envs timeout -k 10 200 python bench.py --no-cpu --no-extra --steps 8 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d['batching'])")
    echo "$name rep=$rep M it/s, ms/step, kernel_ms, batching: $v"
  done
done
