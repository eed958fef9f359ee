mkdir -p gpurun_out
timeout -k 10 300 bash tools/ab.sh -t micro 2 "prio|" "noprio|tools/abx/libgpad_noprio.so" > gpurun_out/r5f_prio_micro.txt 2>&1 && cat gpurun_out/r5f_prio_micro.txt && \
timeout -k 10 400 bash tools/ab.sh 2 "prio|" "noprio|tools/abx/libgpad_noprio.so" > gpurun_out/r5f_prio_c4.txt 2>&1 && cat gpurun_out/r5f_prio_c4.txt && \
BENCH_ARGS="--no-cpu --no-extra --steps 8 --batch 4096" timeout -k 10 400 bash tools/ab.sh 2 "prio|" "noprio|tools/abx/libgpad_noprio.so" > gpurun_out/r5f_prio_c3.txt 2>&1 && cat gpurun_out/r5f_prio_c3.txt && \
for b in 4096 8192; do GPAD_LIB=$PWD/tools/abx/libgpad_stamp.so GPAD_LIB_TOLERANT=1 timeout -k 10 120 python3 tools/stamp_panel.py --batch $b > gpurun_out/r5f_stamp_$b.txt 2>&1 || exit 1; done
