#!/bin/bash
# one-panel relay (3 hops) and pair hand-off priorities: parity, then interleaved A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread \
    -k "panel or shared or termination" > gpurun_out/r3_tests.log 2>&1 || { tail -30 gpurun_out/r3_tests.log; exit 1; }
tail -3 gpurun_out/r3_tests.log
timeout -k 10 400 bash tools/ab_mb.sh 3 "ho|tools/abx/ho.so|" "relay3|tools/abx/relay3.so|" "relay3p|tools/abx/relay3p.so|" > gpurun_out/r3_ab.txt 2>&1 || exit 1
cat gpurun_out/r3_ab.txt
for rep in 1 2; do
  for v in ho relay3 relay3p; do
    GPAD_LIB=$PWD/tools/abx/$v.so timeout -k 10 200 python bench.py --no-cpu --no-extra --steps 10 > gpurun_out/r3_bench_$v.$rep.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3_bench_$v.$rep.json')); print('$v rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['value_repeated_inputs']/1e6,1))" | tee -a gpurun_out/r3_ab.txt
  done
done
