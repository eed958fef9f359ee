#!/bin/bash
# Interleaved A/B of library builds (tools/ab/*.so) on the fixed-N panel microbenchmark:
#   bash tools/ab_mb.sh [reps] [extra microbench args]
REPS=${1:-2}; shift || true
for rep in $(seq 1 $REPS); do
  for lib in tools/ab/*.so; do
    GPAD_LIB=$PWD/$lib timeout -k 10 120 python3 tools/microbench.py --only panel "$@" 2>/dev/null | \
      python3 -c "import json,sys; print('$(basename $lib .so) rep=$rep', ' '.join(f\"B={d['batch']}:{d['us_per_iter']}us\" for d in map(json.loads, sys.stdin)))"
  done
done
