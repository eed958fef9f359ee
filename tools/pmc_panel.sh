#!/bin/bash
# Dynamic instruction mix of the panel-pair kernel (fixed N, no tests; and the tol path with a
# tolerance no instance meets, so every 10th iteration runs the test): one PMC pass per counter
# group, each under its own time limit.  Output: gpurun_out/pmc_panel_<tag>/<case>_<group>/
set -e
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${1:-x}
OUT=gpurun_out/pmc_panel_$TAG
mkdir -p $OUT
for cs in "fixed|--tol 0" "tol|--tol 1e-12"; do
  IFS='|' read -r name targs <<< "$cs"
  for grp in "inst|SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES" \
             "busy|SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
    IFS='|' read -r gname ctrs <<< "$grp"
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/${name}_${gname} -o run -- \
        python3 tools/microbench.py --only panel --batch 8192 --reps 2 $targs > $OUT/${name}_${gname}.log 2>&1
    echo "$name $gname done"
  done
done
