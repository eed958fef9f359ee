// Micro-benchmark for the ONE-PANEL layout of gpad_panel2_kernel (C3: one 16-instance panel per CU,
// n = m = 200, T = 13): phases of one GEMM -- A from an L2-resident fragment image, B from LDS,
// a short epilogue and a barrier per phase -- with different deals of the 13 row-tile chains over
// the 16 waves (wave w on SIMD w % 4; the SIMD issues MFMAs oldest wave first):
//   mode 0: 13 single-chain waves (4,3,3,3), no relay (the pre-r02 layout)
//   mode 1: 12 single-chain waves, 3 per SIMD, tile 12 skipped (the balanced singles' bound)
//   mode 2: 12 tiles as one DOUBLE wave (two tiles' chains interleaved over one B fragment) + one
//           single per SIMD, single older, tile 12 skipped
//   mode 3: mode 2 + tile 12 as a 4-piece relay over the oldest wave of each SIMD (raised priority)
//   mode 4: mode 1 + the same 4-piece relay (singles + relay)
//   mode 5: mode 2 with the double older than the single
//   mode 6: mode 3 with the double older than the single
//   mode 7: mode 2 + tile 12 as a 3-piece relay on the oldest waves of SIMDs 0-2
//   mode 8: mode 2 + tile 12 as a 2-piece relay, [0,7) on SIMD 0 then [7,13) on SIMD 1 (oldest waves)
//   mode 9: mode 2 + tile 12 whole on SIMD 0's oldest wave (no relay: 4 chains there)
//   mode 10: mode 2 + tile 12 as a LAGGED 4-piece relay (r06): in phase p the oldest waves of SIMDs
//           0, 1 run pieces [0,3), [3,6) of chain p while those of SIMDs 2, 3 run pieces [6,9), [9,13)
//           of chain p-1 (the hand-off 1 -> 2 crosses the barrier): a chain's result is due a phase
//           later, so the phase's sequential path is two pieces, not four
//   mode 11: mode 1 (singles 3/SIMD) + the lagged relay of mode 10
//   mode 12: mode 10 without the pieces' raised priority; mode 13: mode 3 without it
//   mode 14: mode 2 + rows 192..199 on the VALU, lagged: the oldest waves of SIMDs 0, 1 each run 100
//           fmaf steps of two interleaved chains per lane per phase (128 outputs x 200 steps over
//           two phases), operands from LDS (A broadcast, B per lane)
//   mode 15: mode 2 + the same work on the oldest wave of every SIMD: 100 steps of one chain per lane
// (relay pieces read their A blocks from registers loaded before the phase's barrier)
// Bound (modes 1-6): 3 chains x 52 MFMAs x 32 cycles = 4992 cycles per SIMD per phase (modes 3, 4, 6
// add 13 relay MFMAs per SIMD: 5408).
// Build: hipcc --offload-arch=gfx950 -O3 -o onepanel onepanel.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kPhases = 2000;
constexpr int T = 13;

// blocks [KB0, KB1) of tile (A image rows) chains; DUAL: two tiles (A0, A1) over one B
template <bool DUAL, int KB0, int KB1>
__device__ __forceinline__ void chain(const float4* __restrict__ A0, const float4* __restrict__ A1, const float4* Bl,
                                      int lane, f4& c0, f4& c1) {
    float4 a0[2], a1[2], b[2];
    a0[0] = A0[(size_t)KB0 * T * 64 + lane];
    if (DUAL) a1[0] = A1[(size_t)KB0 * T * 64 + lane];
    b[0] = Bl[KB0 * 64 + lane];
#pragma unroll
    for (int kb = KB0; kb < KB1; ++kb) {
        const int cur = (kb - KB0) & 1, nxt = cur ^ 1;
        if (kb + 1 < KB1) {
            a0[nxt] = A0[(size_t)(kb + 1) * T * 64 + lane];
            if (DUAL) a1[nxt] = A1[(size_t)(kb + 1) * T * 64 + lane];
            b[nxt] = Bl[(kb + 1) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        const float4 x = a0[cur], z = a1[cur], y = b[cur];
        const int steps = kb + 1 < T ? 4 : 2;  // n = 200: the last block issues 2 steps
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, y.x, c0, 0, 0, 0);
        if (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(z.x, y.x, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, y.y, c0, 0, 0, 0);
        if (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(z.y, y.y, c1, 0, 0, 0);
        if (steps > 2) {
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, y.z, c0, 0, 0, 0);
            if (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(z.z, y.z, c1, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, y.w, c0, 0, 0, 0);
            if (DUAL) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(z.w, y.w, c1, 0, 0, 0);
        }
        asm volatile("" : "+v"(c0), "+v"(c1)::"memory");
    }
}

// a relay piece with its A blocks loaded ahead (before the barrier that precedes the phase)
template <int KB0, int KB1>
__device__ __forceinline__ void piece(const float4 (&pre)[5], const float4* Bl, int lane, f4& c0) {
    float4 b[2];
    b[0] = Bl[KB0 * 64 + lane];
#pragma unroll
    for (int kb = KB0; kb < KB1; ++kb) {
        const int cur = (kb - KB0) & 1, nxt = cur ^ 1;
        if (kb + 1 < KB1) b[nxt] = Bl[(kb + 1) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
        const float4 x = pre[kb - KB0], y = b[cur];
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, y.x, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, y.y, c0, 0, 0, 0);
        if (kb + 1 < T) {
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, y.z, c0, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, y.w, c0, 0, 0, 0);
        }
        asm volatile("" : "+v"(c0)::"memory");
    }
}

// role of wave w: kind 0 idle, 1 single (tile t0), 2 double (t0, t1), 3 relay piece t0 = piece index
struct Role {
    int kind, t0, t1;
};

template <int MODE>
__device__ Role role_of(int w) {
    const int s = w & 3, age = w >> 2;  // age 0 = oldest on its SIMD
    const bool relay = MODE == 3 || MODE == 4 || MODE == 6;
    if (MODE == 14 || MODE == 15) {
        if (age == 0) return (MODE == 15 || s < 2) ? Role{7, s, 0} : Role{0, 0, 0};
        if (age == 1) return Role{1, 8 + s, 0};
        if (age == 2) return Role{2, 2 * s, 2 * s + 1};
        return Role{0, 0, 0};
    }
    if (MODE == 13) {
        if (age == 0) return Role{3, s, 0};
        if (age == 1) return Role{1, 8 + s, 0};
        if (age == 2) return Role{2, 2 * s, 2 * s + 1};
        return Role{0, 0, 0};
    }
    if (MODE == 10 || MODE == 11 || MODE == 12) {
        if (age == 0) return Role{6, s, 0};
        if (MODE == 11) return Role{1, 3 * s + age - 1, 0};
        if (age == 1) return Role{1, 8 + s, 0};
        if (age == 2) return Role{2, 2 * s, 2 * s + 1};
        return Role{0, 0, 0};
    }
    if (MODE == 7) {  // double + single per SIMD, 3-piece relay on the oldest waves of SIMDs 0-2
        if (age == 0) return s < 3 ? Role{4, s, 0} : Role{0, 0, 0};
        if (age == 1) return Role{1, 8 + s, 0};
        if (age == 2) return Role{2, 2 * s, 2 * s + 1};
        return Role{0, 0, 0};
    }
    if (MODE == 8) {  // double + single per SIMD, 2-piece relay [0,7) SIMD 0 -> [7,13) SIMD 1 (oldest)
        if (age == 0) return s < 2 ? Role{5, s, 0} : Role{0, 0, 0};
        if (age == 1) return Role{1, 8 + s, 0};
        if (age == 2) return Role{2, 2 * s, 2 * s + 1};
        return Role{0, 0, 0};
    }
    if (MODE == 9) {  // double + single per SIMD, tile 12 whole on SIMD 0's oldest wave
        if (age == 0) return s == 0 ? Role{1, 12, 0} : Role{0, 0, 0};
        if (age == 1) return Role{1, 8 + s, 0};
        if (age == 2) return Role{2, 2 * s, 2 * s + 1};
        return Role{0, 0, 0};
    }
    if (MODE == 0) return w < 13 ? Role{1, w, 0} : Role{0, 0, 0};
    if (relay && age == 0) return Role{3, s, 0};
    if (MODE == 1 || MODE == 4) return age >= 1 ? Role{1, 3 * s + age - 1, 0} : Role{0, 0, 0};
    // doubles: tiles 2s, 2s+1 (0..7); singles: tile 8 + s
    const bool dbl_older = MODE == 5 || MODE == 6;
    const int single_age = dbl_older ? 2 : 1, double_age = dbl_older ? 1 : 2;
    if (age == single_age) return Role{1, 8 + s, 0};
    if (age == double_age) return Role{2, 2 * s, 2 * s + 1};
    return Role{0, 0, 0};
}

template <int MODE>
__global__ __launch_bounds__(1024) void phases(float* out, const float4* amat) {
    __shared__ float4 bl[T * 64];
    __shared__ float4 hand[4][64];
    __shared__ int hflag[4];
    __shared__ float sink[16][64];
    __shared__ float4 arow[2][64];  // remainder rows' A values (broadcast reads)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < T * 64; i += blockDim.x) bl[i] = make_float4(1e-3f, 2e-3f, 3e-3f, 4e-3f);
    if (threadIdx.x < 4) hflag[threadIdx.x] = 0;
    if (threadIdx.x < 128) arow[threadIdx.x >> 6][threadIdx.x & 63] = make_float4(1e-3f, -2e-3f, 3e-3f, -4e-3f);
    __syncthreads();
    const Role r = role_of<MODE>(__builtin_amdgcn_readfirstlane(w));
    // relay pieces: their A blocks, loaded before the barrier that precedes each phase
    float4 pre[5];
    auto load_pre = [&]() {
        if (r.kind == 3 || r.kind == 4 || r.kind == 6) {
            const int kb0 = r.kind == 4 ? 4 * r.t0 : 3 * r.t0;
#pragma unroll
            for (int i = 0; i < 5; ++i) pre[i] = amat[(size_t)((kb0 + i < T ? kb0 + i : T - 1) * T + 12) * 64 + lane];
        }
    };
    load_pre();
    float keep = 0.0f;
    for (int p = 0; p < kPhases; ++p) {
        float e = 0.0f;
        f4 c0 = {0, 0, 0, 0}, c1 = c0;
        if (r.kind == 1) {
            chain<false, 0, T>(amat + (size_t)r.t0 * 64, amat, bl, lane, c0, c1);
        } else if (r.kind == 2) {
            chain<true, 0, T>(amat + (size_t)r.t0 * 64, amat + (size_t)r.t1 * 64, bl, lane, c0, c1);
        } else if (r.kind == 5) {  // 2-piece relay
            if (r.t0 > 0) {
                while (__hip_atomic_load(&hflag[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != p + 1)
                    __builtin_amdgcn_s_sleep(1);
                const float4 h = hand[0][lane];
                c0 = f4{h.x, h.y, h.z, h.w};
            }
            __builtin_amdgcn_s_setprio(3);
            if (r.t0 == 0) chain<false, 0, 7>(amat + (size_t)12 * 64, amat, bl, lane, c0, c1);
            else chain<false, 7, T>(amat + (size_t)12 * 64, amat, bl, lane, c0, c1);
            __builtin_amdgcn_s_setprio(0);
            if (r.t0 == 0) {
                hand[0][lane] = make_float4(c0.x, c0.y, c0.z, c0.w);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __hip_atomic_store(&hflag[0], p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                c0 = f4{0, 0, 0, 0};
            }
        } else if (r.kind == 7) {  // VALU remainder: 100 steps per phase, 2 chains (mode 14) or 1 (15)
            float x0 = c0.x, x1 = c0.y;
#pragma unroll 5
            for (int k4 = 0; k4 < 25; ++k4) {
                const float4 a0 = arow[0][k4], b0 = bl[k4 * 64 + lane];
                x0 = __builtin_fmaf(a0.x, b0.x, x0);
                x0 = __builtin_fmaf(a0.y, b0.y, x0);
                x0 = __builtin_fmaf(a0.z, b0.z, x0);
                x0 = __builtin_fmaf(a0.w, b0.w, x0);
                if (MODE == 14) {
                    const float4 a1 = arow[1][k4], b1 = bl[(k4 + 25) * 64 + lane];
                    x1 = __builtin_fmaf(a1.x, b1.x, x1);
                    x1 = __builtin_fmaf(a1.y, b1.y, x1);
                    x1 = __builtin_fmaf(a1.z, b1.z, x1);
                    x1 = __builtin_fmaf(a1.w, b1.w, x1);
                }
            }
            c0 = f4{x0, x1, 0.0f, 0.0f};
        } else if (r.kind == 6) {  // lagged relay: pieces 0, 1 of chain p, pieces 2, 3 of chain p - 1
            const int c = r.t0 < 2 ? p : p - 1;  // the chain this piece works on
            if (c >= 0) {
                // slots: 0 (piece 0 -> 1), 1 + (c & 1) (1 -> 2, across the barrier), 3 (2 -> 3)
                const int in = r.t0 == 1 ? 0 : (r.t0 == 2 ? 1 + (c & 1) : 3);
                if (r.t0 > 0) {
                    while (__hip_atomic_load(&hflag[in], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != c + 1)
                        __builtin_amdgcn_s_sleep(1);
                    const float4 h = hand[in][lane];
                    c0 = f4{h.x, h.y, h.z, h.w};
                }
                if (MODE != 12) __builtin_amdgcn_s_setprio(3);
                if (r.t0 == 0) piece<0, 3>(pre, bl, lane, c0);
                if (r.t0 == 1) piece<3, 6>(pre, bl, lane, c0);
                if (r.t0 == 2) piece<6, 9>(pre, bl, lane, c0);
                if (r.t0 == 3) piece<9, T>(pre, bl, lane, c0);
                __builtin_amdgcn_s_setprio(0);
                if (r.t0 < 3) {
                    const int out = r.t0 == 0 ? 0 : (r.t0 == 1 ? 1 + (c & 1) : 3);
                    hand[out][lane] = make_float4(c0.x, c0.y, c0.z, c0.w);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __hip_atomic_store(&hflag[out], c + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    c0 = f4{0, 0, 0, 0};
                }
            }
        } else if (r.kind == 3 || r.kind == 4) {  // tile 12 relayed: 4 pieces [0,3) [3,6) [6,9) [9,13)
            // (kind 3) or 3 pieces [0,4) [4,8) [8,13) (kind 4) on the oldest waves, A loaded ahead
            const int last = r.kind == 3 ? 3 : 2;
            if (r.t0 > 0) {
                while (__hip_atomic_load(&hflag[r.t0 - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != p + 1)
                    __builtin_amdgcn_s_sleep(1);
                const float4 h = hand[r.t0 - 1][lane];
                c0 = f4{h.x, h.y, h.z, h.w};
            }
            if (MODE != 13) __builtin_amdgcn_s_setprio(3);
            if (r.kind == 3) {
                if (r.t0 == 0) piece<0, 3>(pre, bl, lane, c0);
                if (r.t0 == 1) piece<3, 6>(pre, bl, lane, c0);
                if (r.t0 == 2) piece<6, 9>(pre, bl, lane, c0);
                if (r.t0 == 3) piece<9, T>(pre, bl, lane, c0);
            } else {
                if (r.t0 == 0) piece<0, 4>(pre, bl, lane, c0);
                if (r.t0 == 1) piece<4, 8>(pre, bl, lane, c0);
                if (r.t0 == 2) piece<8, T>(pre, bl, lane, c0);
            }
            __builtin_amdgcn_s_setprio(0);
            if (r.t0 < last) {
                hand[r.t0][lane] = make_float4(c0.x, c0.y, c0.z, c0.w);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __hip_atomic_store(&hflag[r.t0], p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                c0 = f4{0, 0, 0, 0};
            }
        }
        const f4 s = c0 * 0.5f + c1 * 0.25f;
        e = s.x * s.y + s.z * s.w;
        sink[w][lane] = e;
        keep += e * 1e-9f;
        load_pre();
        __syncthreads();
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = keep + sink[(w + 1) & 15][lane];
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, sizeof(float) * (size_t)cus * 1024);
    float4* amat;
    hipMalloc(&amat, sizeof(float4) * T * T * 64);
    hipMemset(amat, 0, sizeof(float4) * T * T * 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"13 singles 4,3,3,3, no relay", "12 singles 3/SIMD (tile 12 skipped)",
                           "double+single/SIMD, single older (tile 12 skipped)", "mode 2 + 4-piece relay of tile 12",
                           "singles 3/SIMD + 4-piece relay", "double+single, double older (no tile 12)",
                           "mode 5 + 4-piece relay", "double+single + 3-piece relay (SIMDs 0-2)",
                           "double+single + 2-piece relay [0,7) S0 -> [7,13) S1", "double+single + tile 12 whole on S0",
                           "double+single + LAGGED 4-piece relay", "singles 3/SIMD + LAGGED 4-piece relay",
                           "mode 10, pieces at normal priority", "mode 3, pieces at normal priority",
                           "mode 2 + VALU rows 192..199, 2 waves x 2 chains", "mode 2 + VALU rows 192..199, 4 waves x 1 chain"};
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 16; ++mode) {
            for (int k = 0; k < 2; ++k) {
                hipEventRecord(e0);
                switch (mode) {
                    case 0: hipLaunchKernelGGL((phases<0>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 1: hipLaunchKernelGGL((phases<1>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 2: hipLaunchKernelGGL((phases<2>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 3: hipLaunchKernelGGL((phases<3>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 4: hipLaunchKernelGGL((phases<4>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 5: hipLaunchKernelGGL((phases<5>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 6: hipLaunchKernelGGL((phases<6>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 7: hipLaunchKernelGGL((phases<7>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 8: hipLaunchKernelGGL((phases<8>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 9: hipLaunchKernelGGL((phases<9>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 10: hipLaunchKernelGGL((phases<10>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 11: hipLaunchKernelGGL((phases<11>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 12: hipLaunchKernelGGL((phases<12>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 13: hipLaunchKernelGGL((phases<13>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 14: hipLaunchKernelGGL((phases<14>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                    case 15: hipLaunchKernelGGL((phases<15>), dim3(cus), dim3(1024), 0, 0, out, amat); break;
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            hipEventElapsedTime(&ms, e0, e1);
            printf("rep %d mode %d %-52s %.3f us/phase\n", rep, mode, names[mode], 1e3f * ms / kPhases);
        }
    return 0;
}
