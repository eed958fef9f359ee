# Timeline of a C4 solve on fresh inputs (the bench's honest mode): kernel trace + parse.
set -e
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
T=${TAG:-tl}
mkdir -p gpurun_out
rm -rf gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T -o run -- python3 tools/timeline.py run --fresh --reps 6 --out gpurun_out/${T}_iters.npy > gpurun_out/${T}_run.log 2>&1
python3 tools/timeline.py parse gpurun_out/$T --iters gpurun_out/${T}_iters.npy > gpurun_out/${T}_timeline.txt
cat gpurun_out/${T}_timeline.txt
