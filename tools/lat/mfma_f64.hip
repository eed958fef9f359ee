// Numerics + rate of v_mfma_f64_16x16x4_f64 on gfx950: can an f64 panel run the
// reference's fp64 arithmetic (acceldualgrad.m's mat-vecs as sequential fma chains, the oracle's
// orc_solve_f64 / orc_solve_value_f64 order) bit for bit, as the f32 16x16x4 MFMA does for fmaf?
//  (1) D[i][j] = sum_k A[i][k] B[k][j] over K = 200 (50 MFMAs, ascending k), every output compared
//      bitwise with three host models: the sequential fma chain (acc = fma(a_k, b_k, acc), k
//      ascending), a 4-term block with ONE rounding per MFMA (acc + exact(sum of 4 products)), and
//      per-MFMA pairwise sums of rounded products;
//  (2) cycles per MFMA: one dependent chain per wave, two independent chains per wave, 1 and 2
//      waves per SIMD (the f64 matrix rate bounds an f64 panel kernel).
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_f64 mfma_f64.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int kSteps = 2048;

template <int CH>
__global__ void chain(double* out, double s, int active) {
    const int w = threadIdx.x >> 6;
    d4 c0 = {0, 0, 0, 0}, c1 = c0;
    double a = s * (threadIdx.x & 7) * 1e-3, b = s * 1e-3;
    if (w < active) {
        for (int i = 0; i < kSteps; ++i) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            if constexpr (CH == 2) c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        }
    }
    d4 r = c0 + c1;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r.x + r.y + r.z + r.w;
}

// A (16 x K) row-major, B (K x 16) row-major; lane l supplies A[l & 15][4 kb + (l >> 4)] and
// B[4 kb + (l >> 4)][l & 15] for k-block kb; acc[i] = D[(l >> 4) + 4 i][l & 15] (MI355X_MICROARCH:
// the f64 C/D layout is col = lane & 15, row = (lane >> 4) + 4 reg_idx, unlike the f32 form).
__global__ void numerics(const double* A, const double* B, double* D, int K) {
    const int l = threadIdx.x;
    d4 acc = {0, 0, 0, 0};
    for (int kb = 0; kb < K / 4; ++kb) {
        const int k = 4 * kb + (l >> 4);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * K + k], B[k * 16 + (l & 15)], acc, 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i) D[l * 4 + i] = acc[i];
}

template <int CH>
void run(const char* name, double* out, int grid, int threads, int active) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((chain<CH>), dim3(grid), dim3(threads), 0, 0, out, 1.0, active);
    const int reps = 10;
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((chain<CH>), dim3(grid), dim3(threads), 0, 0, out, 1.0, active);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ns = ms / reps * 1e6 / kSteps;
    const double flop = 2.0 * 16 * 16 * 4 * CH * (active / 4.0) * 4 * grid;  // per step, whole chip
    printf("%-36s %7.3f ns/step (%6.2f cyc @2.4GHz), %d MFMA/step/wave, chip %6.1f TF/s\n", name, ns, ns * 2.4, CH,
           flop / (ns * 1e-9) / 1e12);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int grid = p.multiProcessorCount;
    double* out;
    hipMalloc(&out, (size_t)grid * 512 * sizeof(double));
    run<1>("f64 16x16x4 dep chain, 1 wave/SIMD", out, grid, 256, 4);
    run<2>("f64 16x16x4 2 chains, 1 wave/SIMD", out, grid, 256, 4);
    run<1>("f64 16x16x4 dep chain, 2 waves/SIMD", out, grid, 512, 8);
    run<2>("f64 16x16x4 2 chains, 2 waves/SIMD", out, grid, 512, 8);

    const int K = 200;
    std::vector<double> A(16 * K), B(K * 16), D(256);
    srand(1);
    auto rnd = [] {
        const double v = (rand() / (double)RAND_MAX) * 2.0 - 1.0;
        return v * (rand() % 7 == 0 ? 1e-6 : 1.0) * (rand() % 11 == 0 ? 1e5 : 1.0);
    };
    for (auto& v : A) v = rnd();
    for (auto& v : B) v = rnd();
    double *dA, *dB, *dD;
    hipMalloc(&dA, A.size() * 8);
    hipMalloc(&dB, B.size() * 8);
    hipMalloc(&dD, 256 * 8);
    hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(numerics, dim3(1), dim3(64), 0, 0, dA, dB, dD, K);
    hipMemcpy(D.data(), dD, 256 * 8, hipMemcpyDeviceToHost);
    int bad_seq = 0, bad_blk = 0, bad_pair = 0;
    double maxrel = 0.0;
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 4; ++i) {
            const int row = (l >> 4) + 4 * i, col = l & 15;
            double seq = 0.0, blk = 0.0, pair = 0.0;
            for (int k = 0; k < K; ++k) seq = std::fma(A[row * K + k], B[k * 16 + col], seq);
            for (int kb = 0; kb < K / 4; ++kb) {
                long double s4 = 0.0L;  // 4 exact-ish products, one rounding into the accumulator
                double p[4];
                for (int t = 0; t < 4; ++t) {
                    const int k = 4 * kb + t;
                    s4 += (long double)A[row * K + k] * (long double)B[k * 16 + col];
                    p[t] = A[row * K + k] * B[k * 16 + col];
                }
                blk = (double)((long double)blk + s4);
                pair = pair + ((p[0] + p[1]) + (p[2] + p[3]));
            }
            const double g = D[l * 4 + i];
            bad_seq += memcmp(&g, &seq, 8) != 0;
            bad_blk += memcmp(&g, &blk, 8) != 0;
            bad_pair += memcmp(&g, &pair, 8) != 0;
            if (seq != 0.0) maxrel = std::fmax(maxrel, std::fabs(g - seq) / std::fabs(seq));
        }
    printf("f64 16x16x4 chain (16x16 outputs, K=%d) differing from: sequential fma chain %d/256, "
           "4-term block one rounding %d/256, pairwise rounded products %d/256; max rel vs fma chain %.3e\n",
           K, bad_seq, bad_blk, bad_pair, maxrel);
    return 0;
}
