#!/bin/bash
# A/B builds of libgpad on one box, interleaved (cross-box variance is several %):
#   bash tools/ab_lib.sh [reps]    -- every tools/ab/*.so, via GPAD_LIB, on the C4 bench
REPS=${1:-2}
for rep in $(seq 1 $REPS); do
  for lib in tools/ab/*.so; do
    v=$(GPAD_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --no-extra --steps 8 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))")
    echo "$(basename $lib .so) rep=$rep M it/s, ms/step, kernel_ms: $v"
  done
done
