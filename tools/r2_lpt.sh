# Round-2: after the LPT-prediction fix -- full GPU suite, default bench, fresh-input timeline
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2l_tests.log 2>&1 || { tail -30 gpurun_out/r2l_tests.log; exit 1; }
tail -2 gpurun_out/r2l_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r2l_bench.json 2> gpurun_out/r2l_bench.err || { tail -20 gpurun_out/r2l_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r2l_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'rep', d['value_repeated_inputs'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])"
TAG=tl_lpt timeout -k 10 400 bash tools/tl_run.sh > /dev/null 2>&1 || { echo timeline failed; exit 1; }
tail -14 gpurun_out/tl_lpt_timeline.txt
