# Full GPU check of the tree: every -m gpu test, smoke, the default bench (TAG prefix).
set -e
cd $GRAFT_REPO_ROOT
T=${1:-full}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1])
L=d['legs']; print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'hbm', d['roofline']['hbm_algorithmic_frac'], 'c3', L['c3_batch4096']['iters_per_s'], 'f64', L['f64_value_c4']['roofline']['frac'], 'c4g', L['c4_global_1gpu']['ms_per_solve'])"
rocprofv3 --list-avail > gpurun_out/${T}_counters.txt 2>&1 || true
