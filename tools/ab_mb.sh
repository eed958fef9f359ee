#!/bin/bash
# Interleaved A/B of library builds x env on the fixed-N panel microbenchmark:
#   bash tools/ab_mb.sh REPS "name|lib|ENV=v ..." ...
REPS=$1; shift
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    IFS='|' read -r name lib envs <<< "$spec"
    env GPAD_LIB=$PWD/$lib $envs timeout -k 10 120 python3 tools/microbench.py --only panel 2>/dev/null | \
      python3 -c "import json,sys; print('$name rep=$rep', ' '.join(f\"B={d['batch']}:{d['us_per_iter']}us\" for d in map(json.loads, sys.stdin)))"
  done
done
