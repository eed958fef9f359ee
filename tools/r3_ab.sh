# round-3 call: all GPU tests on the tree, then A/Bs
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_check.sh r3r tests tl
for v in cur6 duo2; do GPAD_LIB=$PWD/tools/abl/$v.so timeout -k 10 120 python3 tools/duo_solo.py | sed "s/^/$v /"; done > gpurun_out/r3r_duo.txt 2>&1
cat gpurun_out/r3r_duo.txt
bash tools/ab.sh 3 "cur5|tools/abl/cur5.so|" "cur6|tools/abl/cur6.so|" "duo2|tools/abl/duo2.so|" > gpurun_out/r3r_ab.txt 2>&1
cat gpurun_out/r3r_ab.txt
