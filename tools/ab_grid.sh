#!/bin/bash
# A/B the panel kernel's persistent grid on one box (interleaved, same process state).
for rep in 1 2; do
  for g in 0 256 384; do
    if [ "$g" = "0" ]; then unset GPAD_PANEL_MAX_GRID; else export GPAD_PANEL_MAX_GRID=$g; fi
    v=$(timeout -k 10 200 python bench.py --no-cpu --no-extra --steps 8 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],3))")
    echo "grid=$g rep=$rep value(M it/s), ms/step: $v"
  done
done
