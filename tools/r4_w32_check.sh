#!/bin/bash
# One GPU call for the W32 pair layout (round 4): the microbenchmark, its parity tests, then an
# interleaved A/B of the C4 bench with the W32 layout on / off (tools/ab.sh, GPAD_PAIR32).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r4d}
timeout -k 10 120 ./tools/lat/w32 > gpurun_out/${T}_w32.txt 2>&1 || { cat gpurun_out/${T}_w32.txt; exit 1; }
cat gpurun_out/${T}_w32.txt
timeout -k 10 400 python -u -m pytest tests/test_pair32.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 600 bash tools/ab.sh 3 "w32||GPAD_PAIR32=1" "w16||GPAD_PAIR32=0" > gpurun_out/${T}_ab.txt 2>&1 || { cat gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
