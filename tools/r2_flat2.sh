# Round-2: flat phased compaction -- parity, then phased vs one launch over batch sizes
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_flat.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "flat or finisher or phased or plan" > gpurun_out/r2fl_tests.log 2>&1 || { tail -40 gpurun_out/r2fl_tests.log; exit 1; }
tail -2 gpurun_out/r2fl_tests.log
timeout -k 10 400 python -u -c "
import json, torch, bench
dev = torch.device('cuda:0')
for kw in ({'batch': 2048}, {'batch': 8192}, {'batch': 32768}, {'batch': 65536}, {'horizon': 50, 'tol': 1e-3, 'batch': 4096}, {'horizon': 50, 'tol': 1e-3, 'batch': 16384}):
    r = bench.flat_tol_leg(dev, **kw)
    print(r['config'], 'phased', round(r['phased']['solve_ms'], 3), r['phased']['launches'], 'one', round(r['one_launch']['solve_ms'], 3), r['phased']['column_util_est'], r['one_launch']['column_util_est'], flush=True)
" > gpurun_out/r2fl2.txt 2> gpurun_out/r2fl2.err || { tail -20 gpurun_out/r2fl2.err; exit 1; }
cat gpurun_out/r2fl2.txt
