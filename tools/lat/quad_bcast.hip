// Micro-benchmark + numerics check of the "quad" chain: v_mfma_f32_4x4x1_16b_f32 with the A
// operand broadcast from one block (cbsz:4 abid:t) -- lane 4t + i of one register holds x_i[k] for
// 16 k-steps, the matrix row of lane l sits in B (register-resident, one row per lane), and
// D_b[i][j] (lane 4b + j, VGPR i) = sum_k x_i[k] * M[4b + j][k]: row = lane, instance = VGPR.
//  (1) numerics: the chain vs the host's fmaf chain (bitwise) for 64 rows x 4 instances, K = 200;
//  (2) cycles per chain step with the broadcast, 1 and 2 waves per SIMD; an MFMA chain beside a
//      DPP fmac chain on the other wave of the SIMD (the finisher's ping-pong partner).
// Build: hipcc --offload-arch=gfx950 -O3 -o quad_bcast quad_bcast.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kSteps = 4096;

template <int T>
__device__ __forceinline__ f4 step16(f4 c, float x, const float (&r)[16]) {
    if constexpr (T < 16) {
        c = __builtin_amdgcn_mfma_f32_4x4x1f32(x, r[T], c, 4, T, 0);
        return step16<T + 1>(c, x, r);
    }
    return c;
}

// MODE 0: every wave an MFMA chain; MODE 1: waves < 4 MFMA chains, waves >= 4 DPP fmac chains;
// MODE 2: waves < 4 idle, waves >= 4 DPP fmac chains
template <int MODE>
__global__ void chain(float* out, float s, int active) {
    const int w = threadIdx.x >> 6;
    f4 c = {0, 0, 0, 0};
    float acc = 0.0f;
    float r[16];
    for (int q = 0; q < 16; ++q) r[q] = s * (threadIdx.x & 7) * 1e-3f + q;
    const float x = s * 1e-3f * (threadIdx.x & 3);
    if (w < active && !(MODE == 2 && w < 4)) {
        if (MODE == 0 || (MODE == 1 && w < 4)) {
            for (int i = 0; i < kSteps / 16; ++i) c = step16<0>(c, x, r);
        } else {
            for (int i = 0; i < kSteps / 16; ++i) {
#pragma unroll
                for (int q = 0; q < 16; q += 4)
                    asm volatile(
                        "v_fmac_f32_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %0, %1, %3 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %0, %1, %4 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                        "v_fmac_f32_dpp %0, %1, %5 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                        : "+v"(acc)
                        : "v"(x), "v"(r[q]), "v"(r[q + 1]), "v"(r[q + 2]), "v"(r[q + 3]));
            }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c[0] + c[1] + c[2] + c[3] + acc;
}

// numerics: lane l holds M[l][k] (B), X lane 4t + i holds x_i[16 g + t] (A, broadcast from block t)
__global__ void numerics(const float* M, const float* X, float* D, int K) {
    const int l = threadIdx.x;
    f4 acc = {0, 0, 0, 0};
    float r[16];
    for (int g = 0; g < K / 16; ++g) {
        const float x = X[(l & 3) * K + 16 * g + (l >> 2)];
        for (int q = 0; q < 16; ++q) r[q] = M[l * K + 16 * g + q];
        acc = step16<0>(acc, x, r);
    }
    for (int i = 0; i < 4; ++i) D[l * 4 + i] = acc[i];  // row l, instance i
}

template <int MODE>
void run(const char* name, float* out, int grid, int threads, int active) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((chain<MODE>), dim3(grid), dim3(threads), 0, 0, out, 1.0f, active);
    const int reps = 20;
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((chain<MODE>), dim3(grid), dim3(threads), 0, 0, out, 1.0f, active);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ns = ms / reps * 1e6 / kSteps;
    printf("%-52s %7.3f ns/step (%5.2f cyc @2.4GHz)\n", name, ns, ns * 2.4);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int grid = p.multiProcessorCount;
    float* out;
    hipMalloc(&out, (size_t)grid * 512 * sizeof(float));
    run<0>("4x4x1 bcast chain, 1 wave/SIMD", out, grid, 256, 4);
    run<0>("4x4x1 bcast chain, 2 waves/SIMD", out, grid, 512, 8);
    run<1>("4x4x1 bcast chain + DPP fmac chain on the SIMD", out, grid, 512, 8);
    run<2>("DPP fmac chain alone (1 wave/SIMD)", out, grid, 512, 8);

    const int K = 208;
    std::vector<float> M(64 * K), X(4 * K), D(256);
    srand(1);
    auto rnd = [] { return (float)((rand() / (double)RAND_MAX) * 2.0 - 1.0) * (rand() % 7 == 0 ? 1e-3f : 1.0f); };
    for (auto& v : M) v = rnd();
    for (auto& v : X) v = rnd();
    float *dM, *dX, *dD;
    hipMalloc(&dM, M.size() * 4);
    hipMalloc(&dX, X.size() * 4);
    hipMalloc(&dD, 256 * 4);
    hipMemcpy(dM, M.data(), M.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(numerics, dim3(1), dim3(64), 0, 0, dM, dX, dD, K);
    hipMemcpy(D.data(), dD, 256 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int row = 0; row < 64; ++row)
        for (int i = 0; i < 4; ++i) {
            float acc = 0.0f;
            for (int k = 0; k < K; ++k) acc = std::fmaf(X[i * K + k], M[row * K + k], acc);
            const float g = D[row * 4 + i];
            if (memcmp(&g, &acc, 4) != 0) ++bad;
        }
    printf("4x4x1 broadcast chain vs host fmaf chain (64 rows x 4 instances, K=%d): %d of 256 differ\n", K, bad);
    return 0;
}
