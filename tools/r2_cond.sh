# Round-2: condensed-operator kernel parity + bench single-instance legs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_condensed.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1 || { tail -40 gpurun_out/r2c_tests.log; exit 1; }
tail -3 gpurun_out/r2c_tests.log
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/r2c_bench.json 2> gpurun_out/r2c_bench.err || { tail -20 gpurun_out/r2c_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r2c_bench.json').read().strip().splitlines()[-1])
for k in ('single_instance','single_instance_c1'): print(k, json.dumps(d[k]))
print('value', d['value'])"
