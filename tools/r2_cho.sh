#!/bin/bash
# condensed panels' chain hand-off: condensed parity, then interleaved A/B of the C4 condensed solve
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_condensed.py -x -q -m gpu --timeout 200 --timeout-method thread \
    > gpurun_out/cho_tests.log 2>&1 || { tail -30 gpurun_out/cho_tests.log; exit 1; }
tail -3 gpurun_out/cho_tests.log
for rep in 1 2 3; do
  for v in relay3 cho; do
    GPAD_LIB=$PWD/tools/abx/$v.so timeout -k 10 120 python3 tools/cond_ab.py 2>>gpurun_out/cho_err.log | tee -a gpurun_out/cho_ab.txt || exit 1
  done
done
