#!/bin/bash
# shader clock under f32 MFMA load: the probe (by operand data), then GRBM counters on the panel microbench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/lat/mfma_clock > gpurun_out/mfma_clock.txt 2>&1 || { cat gpurun_out/mfma_clock.txt; exit 1; }
cat gpurun_out/mfma_clock.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d gpurun_out/clk -o clk -- python3 tools/microbench.py --only panel > gpurun_out/clk_mb.txt 2>&1 || { tail -20 gpurun_out/clk_mb.txt; exit 1; }
ls -R gpurun_out/clk | head
