#!/bin/bash
# Profiling recipe for the GPAD bench (run on the GPU box from the repo root):
#   bash tools/profile.sh <tag> [bench args...]
# 1. rocprofv3 --kernel-trace --stats over the bench command  -> per-kernel durations
# 2. separate --pmc passes (MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and
#    WRITE_SIZE cannot share a pass) -> HBM bytes, MFMA/VALU instruction mix, busy cycles
# 3. tools/pmc_summary.py -> gpurun_out/prof_<tag>/summary.json (copy into profiles/)
set -e
TAG=${1:-r01}
shift || true
ARGS=${@:---steps 12 --warmup 1 --no-cpu --no-extra}  # C4 solves only: the legs launch the same kernels
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- python3 $SCRIPT $ARGS \
      > $OUT/$name.log 2>&1
}
SCRIPT=${PROFILE_SCRIPT:-bench.py}  # e.g. PROFILE_SCRIPT=tools/c5_run.py for the C5 stream leg alone
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT
PROFILE_ARGS="$ARGS" python3 tools/pmc_summary.py $OUT > $OUT/summary.json
cat $OUT/summary.json
