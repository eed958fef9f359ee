// Micro-benchmark for the "W32" pair layout: the 32
// instances of a panel pair as the 32 columns of v_mfma_f32_32x32x2_f32 chains instead of two
// 16-column panels on v_mfma_f32_16x16x4_f32.
//  (1) numerics: a 32x32x2 chain over K = 200 (100 MFMAs, ascending k) bitwise against the host's
//      fmaf chain (A lane l: A[l&31][k = 2s + (l>>5)], B: B[k][l&31], D reg r: row
//      (r&3) + 8(r>>2) + 4(l>>5), col l&31 -- cdna_hip_programming.md);
//  (2) cycles per MFMA of one dependent 32x32x2 chain alone on a SIMD (the 16x16x4 chain needs 40
//      per 32-cycle issue, so a lone 16x16x4 chain runs at 80 %);
//  (3) phases mimicking one GEMM of the C4 pair (n = m = 200, 32 instances), A from an L2-resident
//      image, B from LDS, an epilogue and a barrier per phase:
//      mode 0: today's deal, 16 waves of 16x16x4 chains, 26 chains as 7,7,6,6 (no hand-off)
//      mode 1: W32, 8 waves: tiles 0-3 (32 rows) one chain each on waves 4-7; tiles 4 and 5 split
//              37 / 63 MFMAs between SIMDs 0 -> 2 and 1 -> 3 through an LDS hand-off (waves 0, 1 ->
//              2, 3), rows 192-199 as one 16x16x4 chain per panel on waves 0, 1 after their pieces:
//              6.5 chain units (1600 cycles) on every SIMD
//      mode 2: mode 1 without the hand-off (tile 4, 5 whole on waves 2, 3): 6,6,8,8 units... as a
//              bound on what the hand-off costs
// Build: hipcc --offload-arch=gfx950 -O3 -o w32 w32.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
constexpr int kPhases = 1000;

__global__ void numerics(const float* A, const float* B, float* D, int K) {
    const int l = threadIdx.x;
    f16v acc = {};
    for (int s = 0; s < K / 2; ++s) {
        const int k = 2 * s + (l >> 5);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[(l & 31) * K + k], B[k * 32 + (l & 31)], acc, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) D[l * 16 + r] = acc[r];
}

__global__ void lone_chain(float* out, int steps) {
    f16v acc = {};
    const float a = 1e-3f * (threadIdx.x & 7), b = 1e-3f;
    if ((threadIdx.x >> 6) == 0)
        for (int i = 0; i < steps; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    float s = 0.0f;
    for (int r = 0; r < 16; ++r) s += acc[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---- phase model -----------------------------------------------------------------------------
// 16x16x4 chain: 13 k-blocks (last 2 steps), A one float4 per block from L2 (PD ahead), B from LDS
template <bool DUAL, int PD>
__device__ __forceinline__ void chain16(const float4* __restrict__ A, const float4* Bl, int lane, f4& c0, f4& c1) {
    float4 a[PD + 1], b[2];
#pragma unroll
    for (int p = 0; p < PD; ++p) a[p] = A[(size_t)p * 13 * 64 + lane];
    b[0] = Bl[lane];
#pragma unroll
    for (int kb = 0; kb < 13; ++kb) {
        const int cur = kb & 1, nxt = cur ^ 1;
        if (kb + PD < 13) a[(kb + PD) % (PD + 1)] = A[(size_t)(kb + PD) * 13 * 64 + lane];
        if (kb + 1 < 13) b[nxt] = Bl[(kb + 1) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
        const float4 x = a[kb % (PD + 1)], y = b[cur];
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, y.x, c0, 0, 0, 0);
        if (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, y.w, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, y.y, c0, 0, 0, 0);
        if (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, y.z, c1, 0, 0, 0);
        if (kb + 1 < 13) {
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, y.z, c0, 0, 0, 0);
            if (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, y.y, c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, y.w, c0, 0, 0, 0);
            if (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, y.x, c1, 0, 0, 0);
        }
        asm volatile("" : "+v"(c0), "+v"(c1)::"memory");
    }
}

// 32x32x2 chain piece: MFMAs [S0, S1) of 100 (4 per float4 block of A and of B), A PD blocks ahead
template <int S0, int S1, int PD>
__device__ __forceinline__ void chain32(const float4* __restrict__ A, const float4* Bl, int lane, f16v& acc) {
    constexpr int B0 = S0 / 4, B1 = S1 / 4;
    float4 a[PD + 1], b[2];
#pragma unroll
    for (int p = 0; p < PD; ++p) a[p] = A[(size_t)(B0 + p) * 64 + lane];
    b[0] = Bl[B0 * 64 + lane];
#pragma unroll
    for (int kb = B0; kb < B1; ++kb) {
        const int i = kb - B0, cur = i & 1, nxt = cur ^ 1;
        if (kb + PD < B1) a[(i + PD) % (PD + 1)] = A[(size_t)(kb + PD) * 64 + lane];
        if (kb + 1 < B1) b[nxt] = Bl[(kb + 1) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
        const float4 x = a[i % (PD + 1)], y = b[cur];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x.x, y.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x.y, y.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x.z, y.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x.w, y.w, acc, 0, 0, 0);
        asm volatile("" : "+v"(acc)::"memory");
    }
}

template <int MODE>
__global__ __launch_bounds__(MODE == 0 ? 1024 : 512) void phases(float* out, const float4* amat) {
    __shared__ float4 bl[26 * 64];    // B operands (either layout), fragment order
    __shared__ float4 hand[2][4][64];  // hand-off accumulators (16 floats per lane)
    __shared__ int hflag[2];
    __shared__ float sink[16][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 26 * 64; i += blockDim.x) bl[i] = make_float4(1e-3f, 2e-3f, 3e-3f, 4e-3f);
    if (threadIdx.x < 2) hflag[threadIdx.x] = 0;
    __syncthreads();
    float keep = 0.0f;
    for (int p = 0; p < kPhases; ++p) {
        float e = 0.0f;
        if constexpr (MODE == 0) {  // 26 chains: waves 0-9 double (tiles 0-9), 10-15 single
            f4 c0 = {0, 0, 0, 0}, c1 = c0;
            const float4* A = amat + (size_t)(w % 13) * 64;
            if (w < 10) chain16<true, 1>(A, bl, lane, c0, c1);
            else chain16<false, 2>(A, bl + 13 * 64, lane, c0, c1);
            const f4 s = c0 * 0.5f + c1 * 0.25f;
            e = s.x * s.y + s.z * s.w;
        } else {
            f16v acc = {};
            const int tile = w < 4 ? 4 + (w & 1) : w - 4;  // waves 0,2: tile 4; 1,3: tile 5; 4-7: tiles 0-3
            const float4* A = amat + (size_t)tile * 25 * 64;
            if (w >= 4) {
                chain32<0, 100, 2>(A, bl, lane, acc);
            } else if (MODE == 2) {  // no hand-off: waves 2, 3 run tiles 4, 5 whole; 0, 1 the 16x16 rows
                if (w >= 2) chain32<0, 100, 2>(A, bl, lane, acc);
            } else if (w < 2) {  // first 36 MFMAs of tile 4 (5), then post
                chain32<0, 36, 2>(A, bl, lane, acc);
                for (int q = 0; q < 4; ++q) hand[w][q][lane] = make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(&hflag[w], p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                acc = f16v{};
            } else {  // wait for the piece, continue MFMAs [36, 100)
                while (__hip_atomic_load(&hflag[w - 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != p + 1)
                    __builtin_amdgcn_s_sleep(1);
                for (int q = 0; q < 4; ++q) {
                    const float4 h = hand[w - 2][q][lane];
                    acc[4 * q] = h.x; acc[4 * q + 1] = h.y; acc[4 * q + 2] = h.z; acc[4 * q + 3] = h.w;
                }
                chain32<36, 100, 2>(A, bl, lane, acc);
            }
            if (w < 2) {  // rows 192-199: one 16x16x4 chain per panel
                f4 c0 = {0, 0, 0, 0}, c1 = c0;
                chain16<false, 2>(amat + (size_t)(6 * 25 + w) * 64, bl, lane, c0, c1);
                e += c0.x + c0.y;
            }
            for (int r = 0; r < 16; r += 2) e += acc[r] * acc[r + 1];
        }
        sink[w][lane] = e;
        keep += e * 1e-9f;
        __syncthreads();
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = keep + sink[(w + 1) & 7][lane];
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    // (1) numerics
    const int K = 200;
    std::vector<float> A(32 * K), B(K * 32), D(64 * 16);
    srand(3);
    auto rnd = [] { return (float)((rand() / (double)RAND_MAX) * 2.0 - 1.0) * (rand() % 5 == 0 ? 1e-3f : 1.0f); };
    for (auto& v : A) v = rnd();
    for (auto& v : B) v = rnd();
    float *dA, *dB, *dD, *out;
    hipMalloc(&dA, A.size() * 4);
    hipMalloc(&dB, B.size() * 4);
    hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(numerics, dim3(1), dim3(64), 0, 0, dA, dB, dD, K);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
            float acc = 0.0f;
            for (int k = 0; k < K; ++k) acc = std::fmaf(A[row * K + k], B[k * 32 + col], acc);
            const float g = D[l * 16 + r];
            bad += memcmp(&g, &acc, 4) != 0;
        }
    printf("32x32x2 chain vs host fmaf chain (32x32 outputs, K=%d): %d of 1024 differ\n", K, bad);
    // (2) lone chain
    hipMalloc(&out, sizeof(float) * (size_t)cus * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int steps = 20000;
    for (int k = 0; k < 2; ++k) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(lone_chain, dim3(cus), dim3(64), 0, 0, out, steps);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("lone dependent 32x32x2 chain: %.2f ns per MFMA (%.1f cycles at 2.4 GHz)\n", ms * 1e6 / steps,
           ms * 1e6 / steps * 2.4);
    // (3) phases
    float4* amat;
    hipMalloc(&amat, sizeof(float4) * 13 * 13 * 64 * 2);
    hipMemset(amat, 0, sizeof(float4) * 13 * 13 * 64 * 2);
    const char* names[] = {"16x16x4, 16 waves, 7,7,6,6 chains", "W32, 8 waves, 6.5 units/SIMD (hand-off)",
                           "W32, 8 waves, no hand-off (6,6,8,8)"};
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            for (int k = 0; k < 2; ++k) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL((phases<0>), dim3(cus), dim3(1024), 0, 0, out, amat);
                if (mode == 1) hipLaunchKernelGGL((phases<1>), dim3(cus), dim3(512), 0, 0, out, amat);
                if (mode == 2) hipLaunchKernelGGL((phases<2>), dim3(cus), dim3(512), 0, 0, out, amat);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            hipEventElapsedTime(&ms, e0, e1);
            printf("rep %d mode %d %-42s %.3f us/phase\n", rep, mode, names[mode], 1e3f * ms / kPhases);
        }
    return 0;
}
