# Round-2 closing check: every -m gpu test, smoke(), the default bench line, rocprof of the bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r2y}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'rep', d['value_repeated_inputs'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])
c=d['legs']['c4_condensed']; print('condensed', c['condensed']['solve_ms'], c['bit_exact']['solve_ms'], c['speedup'])"
timeout -k 10 900 bash tools/profile.sh ${PTAG:-r02} > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
echo profiled
