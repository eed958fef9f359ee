# Fresh-input solve timelines of C4 (8192) and C3 (4096): kernel trace + parse + per-kernel stats.
set -e
cd $GRAFT_REPO_ROOT
T=${TAG:-tlb}
mkdir -p gpurun_out
for B in 8192 4096; do
  rm -rf gpurun_out/${T}_$B
  (cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_$B -o run -- python3 tools/timeline.py run --fresh --reps 8 --batch $B --out gpurun_out/${T}_${B}_iters.npy > gpurun_out/${T}_${B}_run.log 2>&1)
  python3 tools/timeline.py parse gpurun_out/${T}_$B --iters gpurun_out/${T}_${B}_iters.npy > gpurun_out/${T}_${B}_timeline.txt
  python3 tools/timeline.py stats gpurun_out/${T}_$B --label B$B >> gpurun_out/${T}_${B}_timeline.txt
  cat gpurun_out/${T}_${B}_timeline.txt; grep "rep " gpurun_out/${T}_${B}_run.log | tail -3
done
