#!/bin/bash
# A/B of the solve phases (phase-1 pairs, phase 2, compaction, duo finisher) on fresh-input C4
# solves: per-kernel time per solve from a rocprofv3 kernel trace, for each library, REPS rounds
# interleaved (the GPU box's clocks drift between runs):
#   bash tools/tail_ab.sh REPS "name|lib" ...     (lib empty: the in-tree library)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
REPS=$1; shift
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    IFS='|' read -r name lib <<< "$spec"
    libenv=""
    [ -n "$lib" ] && libenv="GPAD_LIB=$PWD/$lib GPAD_LIB_TOLERANT=1"
    d=gpurun_out/tab_${name}_${rep}
    rm -rf $d
    (cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && env $libenv timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/timeline.py run --fresh --reps 9 --out $d.npy > $d.log 2>&1)
    python3 tools/timeline.py stats $d --label "$name/$rep"
  done
done
