# Round-2: condensed batches with the latency finisher -- parity and the C4 condensed leg
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_condensed.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2cp_tests.log 2>&1 || { tail -40 gpurun_out/r2cp_tests.log; exit 1; }
tail -2 gpurun_out/r2cp_tests.log
timeout -k 10 300 python -u -c "
import json, torch, bench
dev = torch.device('cuda:0')
print(json.dumps(bench.condensed_leg(dev)))
print(json.dumps(bench.condensed_leg(dev, batch=4096)))
" > gpurun_out/r2cp_leg.json 2> gpurun_out/r2cp_leg.err || { tail -20 gpurun_out/r2cp_leg.err; exit 1; }
cat gpurun_out/r2cp_leg.json
