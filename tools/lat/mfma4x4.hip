// Micro-benchmark + numerics check of v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4x1, f32 in/out)
// on gfx950, as the engine of a register-resident "quad" GEMV (lane l holds matrix row l of a
// 64-row group in A, four instance vectors in B):
//  (1) cycles per MFMA for a dependent accumulator chain, 1 or 2 waves per SIMD, 1 or 2 chains
//      per wave; 16x16x4 for comparison;
//  (2) is D = fma(A, B, C) bitwise per k-step (one accumulation chain over k = 0..K-1, checked
//      against the host's fmaf chain on random data)?
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma4x4 mfma4x4.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kSteps = 4096;

template <int CH, bool BIG>
__global__ void chain(float* out, float s, int active) {
    const int w = threadIdx.x >> 6;
    f4 c0 = {0, 0, 0, 0}, c1 = c0;
    float a = s * (threadIdx.x & 7) * 1e-3f, b = s * 1e-3f;
    if (w < active) {
        for (int i = 0; i < kSteps; ++i) {
            if constexpr (BIG) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
                if constexpr (CH == 2) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
            } else {
                c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
                if constexpr (CH == 2) c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
            }
        }
    }
    f4 r = c0 + c1;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r.x + r.y + r.z + r.w;
}

// numerics: lane l holds A[l][k] (row l = 4*(l/4) + l%4 of block l/4) and B = x_{l%4}[k];
// D_b[i][j] = sum_k A[4b+i][k] * x_j[k] accumulated k = 0..K-1.
__global__ void numerics(const float* A, const float* X, float* D, int K) {
    const int l = threadIdx.x;
    f4 acc = {0, 0, 0, 0};
    for (int k = 0; k < K; ++k) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l * K + k], X[(l & 3) * K + k], acc, 0, 0, 0);
    // lane l holds D_b[i][j] for b = l/4, j = l%4, i = 0..3
    for (int i = 0; i < 4; ++i) D[((l >> 2) * 4 + i) * 4 + (l & 3)] = acc[i];
}

template <int CH, bool BIG>
void run(const char* name, float* out, int grid, int threads, int active) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((chain<CH, BIG>), dim3(grid), dim3(threads), 0, 0, out, 1.0f, active);
    const int reps = 20;
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((chain<CH, BIG>), dim3(grid), dim3(threads), 0, 0, out, 1.0f, active);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ns = ms / reps * 1e6 / kSteps;  // per step of one chain (CH MFMAs per step)
    printf("%-40s %7.3f ns/step (%5.2f cyc @2.4GHz) per chain-step, %d MFMA/step\n", name, ns, ns * 2.4, CH);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int grid = p.multiProcessorCount;
    float* out;
    hipMalloc(&out, (size_t)grid * 512 * sizeof(float));
    run<1, false>("4x4x1_16b dep chain, 1 wave/SIMD", out, grid, 256, 4);
    run<1, false>("4x4x1_16b dep chain, 2 waves/SIMD", out, grid, 512, 8);
    run<2, false>("4x4x1_16b 2 chains, 1 wave/SIMD", out, grid, 256, 4);
    run<2, false>("4x4x1_16b 2 chains, 2 waves/SIMD", out, grid, 512, 8);
    run<1, true>("16x16x4 dep chain, 1 wave/SIMD", out, grid, 256, 4);
    run<2, true>("16x16x4 2 chains, 1 wave/SIMD", out, grid, 256, 4);

    const int K = 200;
    std::vector<float> A(64 * K), X(4 * K), D(256), R(256);
    srand(1);
    auto rnd = [] { return (float)((rand() / (double)RAND_MAX) * 2.0 - 1.0) * (rand() % 7 == 0 ? 1e-3f : 1.0f); };
    for (auto& v : A) v = rnd();
    for (auto& v : X) v = rnd();
    float *dA, *dX, *dD;
    hipMalloc(&dA, A.size() * 4);
    hipMalloc(&dX, X.size() * 4);
    hipMalloc(&dD, 256 * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(numerics, dim3(1), dim3(64), 0, 0, dA, dX, dD, K);
    hipMemcpy(D.data(), dD, 256 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int row = 0; row < 64; ++row)
        for (int j = 0; j < 4; ++j) {
            float acc = 0.0f;
            for (int k = 0; k < K; ++k) acc = std::fmaf(A[row * K + k], X[j * K + k], acc);
            const float g = D[row * 4 + j];
            if (memcmp(&g, &acc, 4) != 0) ++bad;
        }
    printf("4x4x1_16b chain vs host fmaf chain (64 rows x 4 cols, K=%d): %d of 256 differ\n", K, bad);
    return 0;
}
