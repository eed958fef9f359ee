# Round-2: condensed panels, 8-wave shared-A vs 16-wave single-unit deal
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_condensed.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2cp_tests.log 2>&1 || { tail -40 gpurun_out/r2cp_tests.log; exit 1; }
tail -2 gpurun_out/r2cp_tests.log
timeout -k 10 300 python -u -c "
import json, torch, bench
dev = torch.device('cuda:0')
for cp in (1, 2):
    for B in (8192, 4096):
        r = bench.condensed_leg(dev, batch=B, cpanel=cp)
        print(cp, B, round(r['condensed']['solve_ms'], 3), round(r['bit_exact']['solve_ms'], 3), round(r['speedup'], 3), flush=True)
" > gpurun_out/r2cp3.txt 2> gpurun_out/r2cp3.err || { tail -20 gpurun_out/r2cp3.err; exit 1; }
cat gpurun_out/r2cp3.txt
