#!/bin/bash
# pair hand-off split point S (helper blocks): 5 / 6 (default) / 7, fixed-N microbench + C4 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 bash tools/ab_mb.sh 3 "s5|tools/abx/s5.so|" "s6|tools/abx/s6.so|" "s7|tools/abx/s7.so|" > gpurun_out/split_ab.txt 2>&1 || exit 1
cat gpurun_out/split_ab.txt
for rep in 1 2; do
  for v in s5 s6 s7; do
    GPAD_LIB=$PWD/tools/abx/$v.so timeout -k 10 200 python bench.py --no-cpu --no-extra --steps 10 > gpurun_out/split_bench_$v.$rep.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/split_bench_$v.$rep.json')); print('$v rep $rep', round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['value_repeated_inputs']/1e6,1))" | tee -a gpurun_out/split_ab.txt
  done
done
