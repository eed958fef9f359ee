#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root).  Writes under gpurun_out/prof/.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/kt_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/pmc3.log 2>&1
