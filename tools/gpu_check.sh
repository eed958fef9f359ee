#!/bin/bash
# GPU check of the tree (run on the box: gpurun -- 'bash tools/gpu_check.sh TAG [steps]'):
#   tests  : every -m gpu test        -> gpurun_out/TAG_tests.log
#   smoke  : __graft_entry__.smoke()  -> gpurun_out/TAG_smoke.log
#   bench  : the default bench line   -> gpurun_out/TAG_bench.json
#   tl     : fresh-input C4 solve timeline (tools/tl_run.sh) -> gpurun_out/TAG_tl_timeline.txt
#   prof   : rocprofv3 kernel trace + PMC passes (tools/profile.sh TAG) -> gpurun_out/prof_TAG/
# default steps: tests smoke bench.  Every step has its own time limit; the first failure ends
# the call.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; shift
STEPS=${@:-tests smoke bench}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
      tail -2 gpurun_out/${T}_tests.log ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
      tail -1 gpurun_out/${T}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'rep', d['value_repeated_inputs'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'c2', d['single_instance']['iters_per_s'])" ;;
    quickbench)
      timeout -k 10 200 python -u bench.py --no-cpu --no-extra --steps 20 > gpurun_out/${T}_qbench.json 2> gpurun_out/${T}_qbench.err || { tail -20 gpurun_out/${T}_qbench.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_qbench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'rep', d['value_repeated_inputs'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'c2', d['single_instance']['iters_per_s'], d['batching']['phase_ends'])" ;;
    tl)
      TAG=${T}_tl timeout -k 10 320 bash tools/tl_run.sh > /dev/null
      tail -25 gpurun_out/${T}_tl_timeline.txt ;;
    prof)
      timeout -k 10 900 bash tools/profile.sh ${T} > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
      tail -c 600 gpurun_out/${T}_prof.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
