// Micro-benchmark: do f32 MFMA and f32 VALU FMAs from different waves on the same SIMD add up?
// (MI355X_MICROARCH: "MFMA and VALU pipes are separate"; f32 MFMA peak = f32 VALU peak.)
// 512-thread workgroups (two waves per SIMD), one per CU x 4 (every CU busy).
//   mode 0: waves 0-3 MFMA (v_mfma_f32_16x16x4_f32, 4 accumulators), waves 4-7 exit
//   mode 1: waves 0-3 VALU (16 independent v_fma_f32 chains), waves 4-7 exit
//   mode 2: waves 0-3 MFMA, waves 4-7 VALU
//   mode 3: all 8 waves MFMA
//   mode 4: all 8 waves VALU
// Build: hipcc --offload-arch=gfx950 -O3 -o coexec coexec.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kIters = 2048;

__device__ __forceinline__ void do_mfma(float* out, float s) {
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    float a = s * threadIdx.x, b = s + threadIdx.x;
    for (int i = 0; i < kIters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
    f4 r = c0 + c1 + c2 + c3;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r.x + r.y + r.z + r.w;
}

__device__ __forceinline__ void do_valu(float* out, float s) {
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = s * (threadIdx.x + j);
    const float a = 0.999f * s, b = 1e-3f * s;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = __builtin_fmaf(acc[j], a, b);
    }
    float r = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) r += acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE>
__global__ __launch_bounds__(512) void probe(float* out, float s) {
    const int w = threadIdx.x >> 6;
    const bool lo = w < 4;
    if (MODE == 0) { if (lo) do_mfma(out, s); }
    if (MODE == 1) { if (lo) do_valu(out, s); }
    if (MODE == 2) { if (lo) do_mfma(out, s); else do_valu(out, s); }
    if (MODE == 3) do_mfma(out, s);
    if (MODE == 4) do_valu(out, s);
}

template <int MODE>
void run(const char* name, float* out, int grid) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(probe<MODE>, dim3(grid), dim3(512), 0, 0, out, 1.0f);
    hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(probe<MODE>, dim3(grid), dim3(512), 0, 0, out, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double per = ms / reps * 1e-3;
    const double mfma_waves = MODE == 0 || MODE == 2 ? 4 : MODE == 3 ? 8 : 0;
    const double valu_waves = MODE == 1 || MODE == 2 ? 4 : MODE == 4 ? 8 : 0;
    const double fl_m = mfma_waves * grid * kIters * 4.0 * 16 * 16 * 4 * 2;
    const double fl_v = valu_waves * grid * kIters * 16.0 * 64 * 2;
    printf("%-34s %8.3f ms  MFMA %6.1f TF  VALU %6.1f TF  total %6.1f TF\n", name, per * 1e3,
           fl_m / per * 1e-12, fl_v / per * 1e-12, (fl_m + fl_v) / per * 1e-12);
}

int main() {
    int dev;
    hipGetDevice(&dev);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, dev);
    const int grid = p.multiProcessorCount;  // one 512-thread block per CU
    float* out;
    hipMalloc(&out, (size_t)grid * 4 * 512 * sizeof(float));
    printf("CUs %d\n", grid);
    for (int g : {grid, 2 * grid}) {
        printf("grid %d blocks\n", g);
        run<0>("4 MFMA waves", out, g);
        run<1>("4 VALU waves", out, g);
        run<2>("4 MFMA + 4 VALU waves", out, g);
        run<3>("8 MFMA waves", out, g);
        run<4>("8 VALU waves", out, g);
    }
    return 0;
}
