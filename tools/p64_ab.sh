#!/bin/bash
# Interleaved A/B of f64 panel library builds (GPAD_LIB) on tools/p64_ab.py:
#   bash tools/p64_ab.sh REPS "name|lib" ...
set -o pipefail
REPS=$1; shift
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    IFS='|' read -r name lib <<< "$spec"
    libenv=""
    [ -n "$lib" ] && libenv="GPAD_LIB=$PWD/$lib GPAD_LIB_TOLERANT=1"
    env $libenv timeout -k 10 200 python3 tools/p64_ab.py --rounds 2 2>/dev/null | sed "s/^/$name rep=$rep /" || exit 1
  done
done
