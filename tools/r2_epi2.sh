#!/bin/bash
# epilogue LDS-operand hoisting A/B: x0 (round start), x2 (packed), x3 (hoist G all, W/P singles), x4 (hoist G)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 bash tools/ab_mb.sh 2 "x0|tools/abx/x0.so|" "x2|tools/abx/x2.so|" "x3|tools/abx/x3.so|" "x4|tools/abx/x4.so|" > gpurun_out/epi2_ab.txt 2>&1 || exit 1
for rep in 1 2 3; do
  for v in x0 x2 x3 x4; do
    GPAD_LIB=$PWD/tools/abx/$v.so timeout -k 10 200 python bench.py --no-cpu --no-extra --steps 10 > gpurun_out/epi2_bench.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/epi2_bench.json')); print('$v rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['value_repeated_inputs']/1e6,1))" | tee -a gpurun_out/epi2_ab.txt
  done
done
