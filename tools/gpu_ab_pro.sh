mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j_tests.log 2>&1 && tail -2 gpurun_out/r5j_tests.log && \
timeout -k 10 500 bash tools/ab.sh 3 "new|" "pro|tools/abx/libgpad_pro.so" "base|tools/abx/libgpad_base.so" > gpurun_out/r5j_ab_c4.txt 2>&1 && cat gpurun_out/r5j_ab_c4.txt && \
BENCH_ARGS="--no-cpu --no-extra --steps 8 --batch 4096" timeout -k 10 400 bash tools/ab.sh 3 "new|" "pro|tools/abx/libgpad_pro.so" "base|tools/abx/libgpad_base.so" > gpurun_out/r5j_ab_c3.txt 2>&1 && cat gpurun_out/r5j_ab_c3.txt && \
for b in 4096 8192; do GPAD_LIB=$PWD/tools/abx/libgpad_stamp.so GPAD_LIB_TOLERANT=1 timeout -k 10 120 python3 tools/phase_stamps.py --batch $b > gpurun_out/r5j_phase_$b.txt 2>&1 || exit 1; done; tail -3 gpurun_out/r5j_phase_4096.txt gpurun_out/r5j_phase_8192.txt
