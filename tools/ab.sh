#!/bin/bash
# Interleaved A/B on one GPU box (cross-box variance is several %, so variants are compared
# within one call, round-robin, REPS times):
#
#   bash tools/ab.sh [-t bench|micro|plan] REPS "name|lib|ENV=v ENV2=v" ...
#
#   name : label printed with every result
#   lib  : a libgpad.so build to load through GPAD_LIB (empty: the in-tree library)
#   ENV  : legacy GPAD_* tuning knobs, mapped onto handle options (gpad_set_option) by
#          tools/tune_env.py for every handle the target creates
#   -t bench (default): bench.py on the C4 shard ($BENCH_ARGS, default
#          "--no-cpu --no-extra --steps 8"): M it/s, ms/step, device ms/step, batching
#   -t micro: tools/microbench.py $MICRO_ARGS (default "--only panel": fixed-N panel iterations,
#          us/iteration per batch)
#   -t plan : tools/plan_sweep.py --one --fresh --reps 8 (fresh-input C4 solve best/median ms)
set -o pipefail
TARGET=bench
if [ "$1" = "-t" ]; then TARGET=$2; shift 2; fi
REPS=$1; shift
BENCH_ARGS=${BENCH_ARGS:-"--no-cpu --no-extra --steps 8"}
MICRO_ARGS=${MICRO_ARGS:-"--only panel"}
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    IFS='|' read -r name lib envs <<< "$spec"
    libenv=""
    [ -n "$lib" ] && libenv="GPAD_LIB=$PWD/$lib GPAD_LIB_TOLERANT=1"
    case $TARGET in
      bench)
        v=$(env $libenv $envs timeout -k 10 200 python3 tools/tuned_bench.py $BENCH_ARGS 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), d['batching'].get('phase_ends'))") || exit 1
        echo "$name rep=$rep M it/s, ms/step, device ms/step, phase ends: $v" ;;
      micro)
        env $libenv $envs timeout -k 10 120 python3 tools/microbench.py $MICRO_ARGS 2>/dev/null | \
          python3 -c "import json,sys; print('$name rep=$rep', ' '.join(f\"B={d['batch']}:{d['us_per_iter']}us\" for d in map(json.loads, sys.stdin)))" || exit 1 ;;
      plan)
        v=$(env $libenv $envs timeout -k 10 120 python3 tools/plan_sweep.py --one --fresh --reps 8 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['best_ms'], d['median_ms'], d['plan'])") || exit 1
        echo "$name rep=$rep best/median ms, plan: $v" ;;
    esac
  done
done
