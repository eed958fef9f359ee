// Micro-benchmark for DESIGN §10 item 2(b): does splitting the panel pairs' 16-wave workgroup
// into two independent 8-wave workgroups per CU hide the per-GEMM phase boundary (barrier, the
// first LDS operand after it, the epilogue of the last chains)?
// Each "phase" mimics one GEMM of gpad_panel2_kernel: every wave reads its B operand from LDS
// (written by another wave before the barrier), runs its nc chains of 50 dependent
// v_mfma_f32_16x16x4_f32 (interleaved when nc = 2), writes an epilogue result to LDS, barrier.
//   mode 0: 1 x 16 waves, 26 chains (waves 0-9 two chains): SIMD loads 7,7,6,6 (pairs, no hand-off)
//   mode 1: 1 x 16 waves, 24 chains (waves 0-7 two chains): 6,6,6,6
//   mode 2: 2 x 8 waves, 13 chains each (waves 0-4 two chains)
//   mode 3: 2 x 8 waves, 12 chains each (waves 0-3 two chains): 24 per CU as mode 1
//   mode 4: mode 1 with A fragments streamed from an L2-resident image, one block ahead
//   mode 5: mode 4 with B read from LDS in fragment order, one block ahead (panel_gemm3's operands)
//   mode 6, 7: mode 4 with the A ring 2 / 3 blocks ahead
// Prints us per phase; the MFMA bound of a 6-chain SIMD is 6 x 50 x 32 = 9600 cycles.
// Build: hipcc --offload-arch=gfx950 -O3 -o twin twin.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kPhases = 2000;
constexpr int kSteps = 50;

template <int WAVES, bool DUAL, int OPS>
__device__ __forceinline__ void run(float (*lds)[WAVES][64], const float4* __restrict__ amat,
                                    const float4* bl, float* out, int w, int lane) {
    f4 keep = {0, 0, 0, 0};
    for (int p = 0; p < kPhases; ++p) {
        const float b = lds[p & 1][(w + 1) % WAVES][lane];  // operand produced before the last barrier
        const float a = 0.5f + 1e-4f * w;
        const float a1 = a + 1e-3f;  // a distinct second chain (else it folds into the first)
        f4 c0 = {0, 0, 0, 0}, c1 = {1, 1, 1, 1};
        if constexpr (OPS == 0) {
#pragma unroll
            for (int s = 0; s < kSteps; ++s) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
                if constexpr (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b, c1, 0, 0, 0);
            }
        } else {  // 13 blocks of 4 steps (the last 2), A (1 KB per block) from L2 one block ahead,
                  // B from LDS (OPS 2) one block ahead, as panel_gemm3
            const float4* A = amat + (size_t)(w % 13) * 64;
            constexpr int PD = OPS <= 2 ? 1 : OPS - 1;  // A blocks in flight
            float4 ab[PD + 1], bb[2];
#pragma unroll
            for (int p2 = 0; p2 < PD; ++p2) ab[p2] = A[(size_t)p2 * 13 * 64 + lane];
            bb[0] = OPS == 2 ? bl[lane] : make_float4(b, b, b, b);
#pragma unroll
            for (int kb = 0; kb < 13; ++kb) {
                const int cur = kb & 1, nxt = cur ^ 1;
                if (kb + PD < 13) ab[(kb + PD) % (PD + 1)] = A[(size_t)(kb + PD) * 13 * 64 + lane];
                if (kb + 1 < 13) bb[nxt] = OPS == 2 ? bl[(kb + 1) * 64 + lane] : make_float4(b, b, b, b);
                __builtin_amdgcn_sched_barrier(0);
                const float4 x = ab[kb % (PD + 1)], y = bb[cur];
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, y.x, c0, 0, 0, 0);
                if constexpr (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, y.w, c1, 0, 0, 0);
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, y.y, c0, 0, 0, 0);
                if constexpr (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, y.z, c1, 0, 0, 0);
                if (kb + 1 < 13) {
                    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, y.z, c0, 0, 0, 0);
                    if constexpr (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, y.y, c1, 0, 0, 0);
                    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, y.w, c0, 0, 0, 0);
                    if constexpr (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, y.x, c1, 0, 0, 0);
                }
                asm volatile("" : "+v"(c0), "+v"(c1)::"memory");
            }
        }
        // epilogue: a few dependent VALU ops on the chain results, one LDS write (double buffer)
        f4 e = c0 * 0.5f + c1 * 0.25f;
        e = e * e + keep;
        keep = e * 1e-9f;
        lds[(p + 1) & 1][w][lane] = 1.0f + 1e-9f * (e.x + e.y + e.z + e.w);
        __syncthreads();
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = keep.x + keep.y + keep.z + keep.w;
}

template <int WAVES, int OPS>
__global__ __launch_bounds__(WAVES * 64) void phases(float* out, const float4* amat, int dual_waves) {
    __shared__ float lds[2][WAVES][64];
    __shared__ float4 bl[13 * 64];  // B blocks in fragment order (OPS 2)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    lds[0][w][lane] = 1.0f + 1e-3f * lane;
    for (int i = threadIdx.x; i < 13 * 64; i += blockDim.x) bl[i] = make_float4(1e-3f, 2e-3f, 3e-3f, 4e-3f);
    __syncthreads();
    if (w < dual_waves) run<WAVES, true, OPS>(lds, amat, bl, out, w, lane);
    else run<WAVES, false, OPS>(lds, amat, bl, out, w, lane);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, sizeof(float) * 2 * cus * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float4* amat;  // one 13 x 13-block fragment image (170 KB, L2-resident), as the panels' A
    hipMalloc(&amat, sizeof(float4) * 13 * 13 * 64);
    hipMemset(amat, 0, sizeof(float4) * 13 * 13 * 64);
    const char* names[] = {"1x16 waves, 26 chains (7,7,6,6)", "1x16 waves, 24 chains (6,6,6,6)",
                           "2x8 waves, 2x13 chains", "2x8 waves, 2x12 chains",
                           "6,6,6,6 + A from L2", "6,6,6,6 + A from L2 + B from LDS",
                           "6,6,6,6 + A from L2, 2 blocks ahead", "6,6,6,6 + A from L2, 3 blocks ahead"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int mode = 0; mode < 8; ++mode) {
            for (int k = 0; k < 2; ++k) {  // warm-up, then timed
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL((phases<16, 0>), dim3(cus), dim3(1024), 0, 0, out, amat, 10);
                if (mode == 1) hipLaunchKernelGGL((phases<16, 0>), dim3(cus), dim3(1024), 0, 0, out, amat, 8);
                if (mode == 2) hipLaunchKernelGGL((phases<8, 0>), dim3(2 * cus), dim3(512), 0, 0, out, amat, 5);
                if (mode == 3) hipLaunchKernelGGL((phases<8, 0>), dim3(2 * cus), dim3(512), 0, 0, out, amat, 4);
                if (mode == 4) hipLaunchKernelGGL((phases<16, 1>), dim3(cus), dim3(1024), 0, 0, out, amat, 8);
                if (mode == 5) hipLaunchKernelGGL((phases<16, 2>), dim3(cus), dim3(1024), 0, 0, out, amat, 8);
                if (mode == 6) hipLaunchKernelGGL((phases<16, 3>), dim3(cus), dim3(1024), 0, 0, out, amat, 8);
                if (mode == 7) hipLaunchKernelGGL((phases<16, 4>), dim3(cus), dim3(1024), 0, 0, out, amat, 8);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("rep %d mode %d %-38s %.3f us/phase\n", rep, mode, names[mode], 1e3f * ms / kPhases);
        }
    }
    hipFree(amat);
    hipFree(out);
    return 0;
}
