# Round-2: flat-panel phased compaction parity + tol-mode flat legs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_flat.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2fl_tests.log 2>&1 || { tail -40 gpurun_out/r2fl_tests.log; exit 1; }
tail -3 gpurun_out/r2fl_tests.log
timeout -k 10 300 python -u -c "
import json, torch, bench
dev = torch.device('cuda:0')
for kw in ({}, {'horizon': 50, 'tol': 1e-3, 'batch': 4096}):
    print(json.dumps(bench.flat_tol_leg(dev, **kw)))
" > gpurun_out/r2fl_leg.json 2> gpurun_out/r2fl_leg.err || { tail -20 gpurun_out/r2fl_leg.err; exit 1; }
cat gpurun_out/r2fl_leg.json
