# Fresh-input C4 solves: kernel-trace timelines for several finisher settings (GPAD_FINISH_SOLO).
set -e
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for S in ${SOLOS:-0 16 48}; do
  T=tls$S
  rm -rf gpurun_out/$T
  GPAD_FINISH_SOLO=$S timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T -o run -- python3 tools/timeline.py run --fresh --reps 8 --out gpurun_out/${T}_iters.npy > gpurun_out/${T}_run.log 2>&1
  python3 tools/timeline.py parse gpurun_out/$T --iters gpurun_out/${T}_iters.npy > gpurun_out/${T}_timeline.txt
  echo "== solo $S"; grep "duo_kernel" gpurun_out/${T}_timeline.txt | awk '$6 > 50 {print $6}' | tr '\n' ' '; echo
  grep "panel2" gpurun_out/${T}_timeline.txt | awk '$6 > 50 {print $6}' | tr '\n' ' '; echo
done
