#!/bin/bash
# panel pairs: A ring 2 blocks deep for the double waves (no spills since the packed epilogues)
set -o pipefail
mkdir -p gpurun_out
GPAD_LIB=$PWD/tools/abx/pd2.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread \
    -k "panel_two_wave or phased_compaction or shared_batch" > gpurun_out/pd2_tests.log 2>&1 || { tail -30 gpurun_out/pd2_tests.log; exit 1; }
tail -3 gpurun_out/pd2_tests.log
timeout -k 10 300 bash tools/ab_mb.sh 3 "base|tools/abx/base.so|" "pd2|tools/abx/pd2.so|" > gpurun_out/pd2_ab.txt 2>&1 || exit 1
cat gpurun_out/pd2_ab.txt
for rep in 1 2; do
  for v in base pd2; do
    GPAD_LIB=$PWD/tools/abx/$v.so timeout -k 10 200 python bench.py --no-cpu --no-extra --steps 10 > gpurun_out/pd2_bench_$v.$rep.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/pd2_bench_$v.$rep.json')); print('$v rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['value_repeated_inputs']/1e6,1))" | tee -a gpurun_out/pd2_ab.txt
  done
done
