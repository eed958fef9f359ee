#!/bin/bash
# hand-off generalised to T = 9, 11: panel parity, then A/B of the C4 path (must be unchanged)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread \
    -k "panel or shared or termination" > gpurun_out/gen_tests.log 2>&1 || { tail -30 gpurun_out/gen_tests.log; exit 1; }
tail -3 gpurun_out/gen_tests.log
timeout -k 10 300 bash tools/ab_mb.sh 2 "relay3|tools/abx/relay3.so|" "gen|tools/abx/gen.so|" > gpurun_out/gen_ab.txt 2>&1 || exit 1
cat gpurun_out/gen_ab.txt
