#!/bin/bash
# A/B two builds of libgpad on one box (interleaved): current tree vs tools/ab/libgpad_static.so
for rep in 1 2; do
  for lib in cur static cur256; do
    unset GPAD_LIB GPAD_PANEL_MAX_GRID
    [ "$lib" = "static" ] && export GPAD_LIB=$PWD/tools/ab/libgpad_static.so
    [ "$lib" = "cur256" ] && export GPAD_PANEL_MAX_GRID=256
    v=$(timeout -k 10 200 python bench.py --no-cpu --no-extra --steps 8 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],3))")
    echo "$lib rep=$rep value(M it/s), ms/step: $v"
  done
done
