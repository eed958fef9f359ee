# Per-phase cost with uniform 20-iteration phases and no finisher (C4 8192 and C3 4096, fresh inputs).
set -e
cd $GRAFT_REPO_ROOT
T=${TAG:-tlu}
mkdir -p gpurun_out
for B in 8192 4096; do
  rm -rf gpurun_out/${T}_$B
  (cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && GPAD_PANEL_NOPLAN=1 GPAD_PANEL_PHASE=20 GPAD_FINISH_THRESH=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_$B -o run -- python3 tools/timeline.py run --fresh --reps 4 --batch $B --out gpurun_out/${T}_${B}_iters.npy > gpurun_out/${T}_${B}_run.log 2>&1)
  python3 tools/timeline.py parse gpurun_out/${T}_$B --iters gpurun_out/${T}_${B}_iters.npy > gpurun_out/${T}_${B}_timeline.txt
  cat gpurun_out/${T}_${B}_timeline.txt | head -40
done
