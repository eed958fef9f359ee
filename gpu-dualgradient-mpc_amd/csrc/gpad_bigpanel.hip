// gpad_bigpanel.hip -- shared-matrix batches with n or m beyond the panel kernels' 256 rows
// (gfx950, f32 MFMA).  E.g. the battery MPC at N = 50 (n = 200, m = 900) or N = 200 / m = 800.
//
// Same scheme as gpad_panel.hip -- a workgroup owns a panel of 16 instances for the whole solve,
// the two mat-vecs are skinny GEMMs on v_mfma_f32_16x16x4_f32 with A (the constant matrices) in
// fragment order streamed from L2/MALL and B (w, zhat) in LDS in fragment order, every row chain
// an ascending-k fmaf chain (bit-exact with the reference's sequential steps) -- but the two
// GEMMs have different shapes: GEMM 1 has T1 = ceil(n/16) row tiles and T2 = ceil(m/16) k-blocks,
// GEMM 2 the reverse, and up to 64 tiles of each.  Wave w (of 16) owns
// row tiles w, w+16, ... of both GEMMs (NT1 / NT2 of them, compile-time) and runs their chains
// (GEMM 2: two tiles interleaved, sharing the B fragments) one after another; the
// per-row state of its tiles (z, g_P; y, w, u, p_D) lives in its registers.  The Algorithm-1 test
// partials are reduced per wave over its tiles, then across the 16 waves in LDS.
//
// Fragment images (built by launch_pack_bigpanel): PA1[b][t] = -ML tile t (16 rows), k-block b
// (b < T2, t < T1); PA2[b][t] = G/L tile t, k-block b (b < T1, t < T2); each a float4 per lane,
// lane (j, c) holding A[16t + pi(c)][16b + 4q + j] as in gpad_panel.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>

#include "gpad_internal.h"

namespace gpad {

typedef float bf32x4 __attribute__((ext_vector_type(4)));
constexpr int kBigMaxTiles = 64;  // n, m <= 1024 (4 tiles per wave and GEMM)
constexpr int kBigWaves = 16;

__device__ __forceinline__ int bpi16(int rho) { return 4 * (rho & 3) + (rho >> 2); }

__global__ void pack_bigpanel_kernel(const float* __restrict__ src, int rows, int cols, double scale, int Tr,
                                     int Tk, float4* __restrict__ dst) {
    // dst[(b * Tr + t) * 64 + lane]: k-block b < Tk (16 columns), row tile t < Tr
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= Tr * Tk * 64) return;
    const int lane = idx & 63, t = (idx >> 6) % Tr, b = (idx >> 6) / Tr;
    const int row = 16 * t + bpi16(lane & 15);
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int col = 16 * b + 4 * q + (lane >> 4);
        v[q] = (row < rows && col < cols) ? (float)(scale * (double)src[(size_t)row * cols + col]) : 0.0f;
    }
    dst[idx] = make_float4(v[0], v[1], v[2], v[3]);
}

__host__ __device__ inline int big_tiles(int x) { return (x + 15) / 16; }

struct BigSlot {  // per wave: its tiles' partials of the test, per column
    float violz[16], violh[16], wmin[16];
    double gap[16];
    float magh[16];  // max(|G_L zhat| + |pD|); with violz reused by the verification of test (A)
};

// LDS: w and p_D per GEMM-2 row tile, zhat per GEMM-1 row tile (1 KiB each), 16 test slots
static size_t big_lds_bytes(int n, int m) {
    return (size_t)(big_tiles(n) + 2 * big_tiles(m)) * 64 * sizeof(float4) + kBigWaves * sizeof(BigSlot);
}

bool bigpanel_supported(int n, int m) {
    const int t1 = big_tiles(n), t2 = big_tiles(m);
    return (t1 > 16 || t2 > 16) && t1 <= kBigMaxTiles && t2 <= kBigMaxTiles && n > 0 && m > 0 &&
           big_lds_bytes(n, m) <= 160 * 1024;
}

size_t bigpanel_frag_bytes(int n, int m) {
    return bigpanel_supported(n, m) ? (size_t)2 * big_tiles(n) * big_tiles(m) * 64 * sizeof(float4) : 0;
}

hipError_t launch_pack_bigpanel(const float* ML, const float* G, int n, int m, float mg_sign, double g_scale,
                                void* frag, hipStream_t s) {
    const int T1 = big_tiles(n), T2 = big_tiles(m);
    float4* pa1 = reinterpret_cast<float4*>(frag);
    float4* pa2 = pa1 + (size_t)T1 * T2 * 64;
    const int tot = T1 * T2 * 64;
    // PA1 = sign * ML (n x m): row tiles T1, k-blocks T2;  PA2 = g_scale * G (m x n): T2 tiles, T1 blocks
    hipLaunchKernelGGL(pack_bigpanel_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, ML, n, m, (double)mg_sign,
                       T1, T2, pa1);
    hipLaunchKernelGGL(pack_bigpanel_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, G, m, n, g_scale, T2, T1,
                       pa2);
    return hipGetLastError();
}

__device__ __forceinline__ float4 bas_float4(__attribute__((ext_vector_type(4))) unsigned v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// acc = sum over k-blocks b < nkb (the last one only its kq 4-steps) of A[b][t] x B[b]:
// A by buffer loads (byte offset (b * Tr + t) KiB + lane 16 B) two k-blocks ahead, B from LDS
// one block ahead.  Unrolled by two with fixed register roles and unconditional (clamped) loads
// so that each block waits only for its own operands (see panel_gemm_rt in gpad_panel.hip).
__device__ __forceinline__ void big_blk(bf32x4& acc, const float4& a, const float4& b, int steps) {
    __builtin_amdgcn_sched_barrier(0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
    if (steps > 1) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
    if (steps > 2) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
    if (steps > 3) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void big_blk2(bf32x4& acc0, bf32x4& acc1, const float4& a, const float4& c,
                                         const float4& b, int steps) {
    __builtin_amdgcn_sched_barrier(0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(c.x, b.x, acc1, 0, 0, 0);
    if (steps > 1) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(c.y, b.y, acc1, 0, 0, 0);
    }
    if (steps > 2) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(c.z, b.z, acc1, 0, 0, 0);
    }
    if (steps > 3) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(c.w, b.w, acc1, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ bf32x4 big_gemm(__amdgpu_buffer_rsrc_t PA, const float4* B, int t, int Tr, int nkb,
                                           int kq, int lane) {
    bf32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const int voff = t * 1024 + lane * 16, stride = Tr * 1024, last = nkb - 1;
    auto lda = [&](int kb) -> float4 {
        return bas_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb < last ? kb : last) * stride, 0));
    };
    float4 a0 = lda(0), a1 = lda(1), b0 = B[lane], b1;
    int kb = 0;  // pairs of full blocks, then the rest (the last block with its kq steps)
    for (; kb + 2 <= last; kb += 2) {
        b1 = B[(kb + 1) * 64 + lane];
        big_blk(acc, a0, b0, 4);
        a0 = lda(kb + 2);
        b0 = B[(kb + 2) * 64 + lane];
        big_blk(acc, a1, b1, 4);
        a1 = lda(kb + 3);
    }
    if (kb < last) {
        b1 = B[last * 64 + lane];
        big_blk(acc, a0, b0, 4);
        a0 = a1;
        b0 = b1;
    }
    big_blk(acc, a0, b0, kq);
    asm volatile("" : "+v"(acc)::"memory");
    return acc;
}

// two row tiles t0, t1 of the same GEMM in one pass: the chains interleave (hiding the 40-cycle
// MFMA dependency of each other) and share every B fragment (one LDS read for both)
__device__ __forceinline__ void big_gemm2(__amdgpu_buffer_rsrc_t PA, const float4* B, int t0, int t1, int Tr,
                                          int nkb, int kq, int lane, bf32x4& acc0, bf32x4& acc1) {
    acc0 = bf32x4{0.0f, 0.0f, 0.0f, 0.0f};
    acc1 = bf32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int v0 = t0 * 1024 + lane * 16, v1 = t1 * 1024 + lane * 16, stride = Tr * 1024, last = nkb - 1;
    auto lda = [&](int voff, int kb) -> float4 {
        return bas_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb < last ? kb : last) * stride, 0));
    };
    float4 a0 = lda(v0, 0), c0 = lda(v1, 0), a1 = lda(v0, 1), c1 = lda(v1, 1), b0 = B[lane], b1;
    int kb = 0;  // pairs of full blocks, then the rest (the last block with its kq steps)
    for (; kb + 2 <= last; kb += 2) {
        b1 = B[(kb + 1) * 64 + lane];
        big_blk2(acc0, acc1, a0, c0, b0, 4);
        a0 = lda(v0, kb + 2);
        c0 = lda(v1, kb + 2);
        b0 = B[(kb + 2) * 64 + lane];
        big_blk2(acc0, acc1, a1, c1, b1, 4);
        a1 = lda(v0, kb + 3);
        c1 = lda(v1, kb + 3);
    }
    if (kb < last) {
        b1 = B[last * 64 + lane];
        big_blk2(acc0, acc1, a0, c0, b0, 4);
        a0 = a1;
        c0 = c1;
        b0 = b1;
    }
    big_blk2(acc0, acc1, a0, c0, b0, kq);
    asm volatile("" : "+v"(acc0), "+v"(acc1)::"memory");
}

template <int NT1, int NT2>
__global__ __launch_bounds__(64 * kBigWaves) void gpad_bigpanel_kernel(SolveArgs<float> a) {
    extern __shared__ __attribute__((aligned(16))) float4 big_lds[];
    const int n = a.n, m = a.m, N = a.N, K = a.check_every;
    const int T1 = big_tiles(n), T2 = big_tiles(m);
    float4* Wl = big_lds;           // [T2][64] w in fragment order (B of GEMM 1)
    float4* Zh = big_lds + T2 * 64;  // [T1][64] zhat (B of GEMM 2)
    float4* Pd = Zh + T1 * 64;       // [T2][64] p_D rows
    BigSlot* slots = reinterpret_cast<BigSlot*>(Pd + T2 * 64);

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = lane >> 4, c = lane & 15;
    const size_t abytes = (size_t)T1 * T2 * 1024;
    const __amdgpu_buffer_rsrc_t PA1 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.frag), 0, (int)abytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t PA2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)a.frag + abytes), 0, (int)abytes, 0x00020000);
    const bool use_tol = a.tol > 0.0;
    const bool fresh = a.v_begin == 0;
    const bool carry = a.v_end < N;
    // GEMM 1: K = m over T2 k-blocks (the last kq1 4-steps), GEMM 2: K = n over T1 k-blocks
    const int kq1 = (m - 16 * (T2 - 1) + 3) / 4, kq2 = (n - 16 * (T1 - 1) + 3) / 4;
    const int count = a.count_in ? __builtin_amdgcn_readfirstlane(*a.count_in) : a.batch;
    if (a.count_in && count <= a.fin_thresh) return;
    const int panels = (count + 15) / 16;

    for (int p = blockIdx.x; p < panels; p += gridDim.x) {
        const int k = 16 * p + c;
        bool active = k < count;
        const int inst = active ? (a.idx_in ? a.idx_in[k] : k) : 0;
        const size_t bi = (size_t)inst;
        unsigned live = 0u;  // columns still running (uniform)
        {
            const int left = count - 16 * p;
            live = left >= 16 ? 0xFFFFu : ((1u << left) - 1u);
        }
        float z[NT1][4], gp[NT1][4];
        float y[NT2][4], u[NT2][4];
#pragma unroll
        for (int q = 0; q < NT1; ++q) {
            const int t = w + kBigWaves * q;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * t + 4 * r + j;
                const bool ok = active && t < T1 && i < n;
                z[q][r] = ok ? a.z[bi * n + i] : 0.0f;
                gp[q][r] = ok ? a.gP[bi * a.ld_gP + i] : 0.0f;
            }
            if (t < T1 && fresh && use_tol) Zh[t * 64 + lane] = make_float4(z[q][0], z[q][1], z[q][2], z[q][3]);
        }
#pragma unroll
        for (int q = 0; q < NT2; ++q) {
            const int t = w + kBigWaves * q;
            float wv[4], pd[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * t + 4 * r + j;
                const bool ok = active && t < T2 && i < m;
                y[q][r] = ok ? a.y[bi * m + i] : 0.0f;
                pd[r] = ok ? (float)(a.gscale * (double)a.g[bi * a.ld_g + i]) : 0.0f;
                if (fresh) {
                    wv[r] = __builtin_fmaf(a.beta[0], y[q][r] - y[q][r], y[q][r]);
                    u[q][r] = 0.0f;
                } else {
                    wv[r] = ok ? a.wc[bi * m + i] : 0.0f;
                    u[q][r] = ok && use_tol ? a.uc[bi * m + i] : 0.0f;
                }
            }
            if (t < T2) {
                Wl[t * 64 + lane] = make_float4(wv[0], wv[1], wv[2], wv[3]);
                Pd[t * 64 + lane] = make_float4(pd[0], pd[1], pd[2], pd[3]);
            }
        }
        if (fresh && use_tol) {  // u = G_L z_{-1}, then the 8c recursion
            __syncthreads();
#pragma unroll
            for (int q = 0; q < NT2; ++q) {
                const int t = w + kBigWaves * q;
                if (t < T2) {
                    const bf32x4 cz = big_gemm(PA2, Zh, t, T2, T1, kq2, lane);
#pragma unroll
                    for (int r = 0; r < 4; ++r) u[q][r] = cz[r];
                }
            }
        }
        __syncthreads();

        int v = a.v_begin;
        float th = a.theta[v], bn = a.beta[v + 1];
        while (true) {
            const float th_next = a.theta[v + 1], bn_next = a.beta[v + 2];
            ++v;
            const bool chk = use_tol && (v % K) == 0;
            const float omt = 1.0f - th;
            // ---- GEMM 1 + epilogue: zhat = -ML w - g_P (8b), z (8c) ---------------------------
#pragma unroll
            for (int q = 0; q < NT1; ++q) {
                const int t = w + kBigWaves * q;
                if (t < T1) {
                    const bf32x4 acc = big_gemm(PA1, Wl, t, T1, T2, kq1, lane);
                    float zh[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        zh[r] = acc[r] - gp[q][r];
                        const float zn = __builtin_fmaf(omt, z[q][r], th * zh[r]);
                        if (active) z[q][r] = zn;
                    }
                    Zh[t * 64 + lane] = make_float4(zh[0], zh[1], zh[2], zh[3]);
                }
            }
            __syncthreads();
            // ---- GEMM 2 + epilogue: y+ (8d), next w (8a), test partials ----------------------------
            float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
            double gap = 0.0;
            bf32x4 acc_next = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int q = 0; q < NT2; ++q) {
                const int t = w + kBigWaves * q;
                // tiles q, q + 1 of this wave in one interleaved pass (acc of q + 1 kept for the next q)
                bf32x4 acc;
                constexpr bool kPair = NT2 > 1;
                if constexpr (kPair) {
                    if ((q & 1) == 0) {
                        if (t + kBigWaves < T2) {
                            big_gemm2(PA2, Zh, t, t + kBigWaves, T2, T1, kq2, lane, acc, acc_next);
                        } else if (t < T2) {
                            acc = big_gemm(PA2, Zh, t, T2, T1, kq2, lane);
                        }
                    } else {
                        acc = acc_next;
                    }
                } else {
                    if (t < T2) acc = big_gemm(PA2, Zh, t, T2, T1, kq2, lane);
                }
                if (t < T2) {
                    const float4 w4 = Wl[t * 64 + lane];
                    const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
                    const float4 p4 = Pd[t * 64 + lane];
                    const float pdq[4] = {p4.x, p4.y, p4.z, p4.w};
                    float wn[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float cv = acc[r];
                        const float sv = (wv[r] + pdq[r]) + cv;               // seq_functions.cpp:84
                        const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;   // seq_functions.cpp:85
                        wn[r] = __builtin_fmaf(bn, yp - y[q][r], yp);
                        if (use_tol) {
                            const float un = __builtin_fmaf(omt, u[q][r], th * cv);
                            if (active) u[q][r] = un;
                            if (chk && active && (16 * t + 4 * r + j) < m) {
                                const float tt = cv + pdq[r];
                                violh = fmaxf(violh, tt);
                                magh = fmaxf(magh, __builtin_fabsf(cv) + __builtin_fabsf(pdq[r]));
                                wmin = fminf(wmin, wv[r]);
                                gap -= (double)wv[r] * (double)tt;
                                violz = fmaxf(violz, u[q][r] + pdq[r]);
                            }
                        }
                        if (active) y[q][r] = yp;
                    }
                    if (active) Wl[t * 64 + lane] = make_float4(wn[0], wn[1], wn[2], wn[3]);
                }
            }
            if (chk) {  // this wave's partials per column -> its slot
#pragma unroll
                for (int o = 16; o < 64; o <<= 1) {
                    violz = fmaxf(violz, __shfl_xor(violz, o, 64));
                    violh = fmaxf(violh, __shfl_xor(violh, o, 64));
                    magh = fmaxf(magh, __shfl_xor(magh, o, 64));
                    wmin = fminf(wmin, __shfl_xor(wmin, o, 64));
                    gap += __shfl_xor(gap, o, 64);
                }
                if (j == 0) {
                    slots[w].violz[c] = violz;
                    slots[w].violh[c] = violh;
                    slots[w].magh[c] = magh;
                    slots[w].wmin[c] = wmin;
                    slots[w].gap[c] = gap;
                }
            }
            th = th_next;
            bn = bn_next;
            __syncthreads();
            if (!chk && v < a.v_end) continue;

            // ---- Algorithm 1 test: every wave reduces the wave slots for the 16 columns, ballot ---
            unsigned m1 = 0u, m2 = 0u;
            bool zh_out = true;  // this iteration's zhat still in Zh (no verification GEMM ran)
            if (chk) {
                int st1 = 0;
                if (lane < 16 && ((live >> lane) & 1u)) {
                    double vz = -INFINITY, vh = -INFINITY, wm = INFINITY, gq = 0.0, mh = 0.0;
#pragma unroll
                    for (int s2 = 0; s2 < kBigWaves; ++s2) {
                        vz = fmax(vz, (double)slots[s2].violz[lane]);
                        vh = fmax(vh, (double)slots[s2].violh[lane]);
                        mh = fmax(mh, (double)slots[s2].magh[lane]);
                        wm = fmin(wm, (double)slots[s2].wmin[lane]);
                        gq += slots[s2].gap[lane];
                    }
                    st1 = (vz * a.L <= a.tol ? 1 : 0) |
                          ((viol_ok(vh, mh, a.L, a.tol, ViolMargin<float>::value) && (wm >= 0.0) &&
                            (gq * a.L <= a.tol_gap)) ? 2 : 0);
                }
                const unsigned mA = (unsigned)__ballot(st1 & 1);
                m2 = (unsigned)__ballot(st1 & 2);
                if (mA) {  // (A) nominated for some column: G_L z for the panel
                    zh_out = false;
#pragma unroll
                    for (int q = 0; q < NT1; ++q) {
                        const int t = w + kBigWaves * q;
                        if (t < T1) {
                            if (active && ((m2 >> c) & 1u)) {  // test (B)'s zhat out before z replaces it
                                const float4 h4 = Zh[t * 64 + lane];
                                const float zh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    const int i = 16 * t + 4 * r + j;
                                    if (i < n) a.z[bi * n + i] = zh[r];
                                }
                            }
                            Zh[t * 64 + lane] = make_float4(z[q][0], z[q][1], z[q][2], z[q][3]);
                        }
                    }
                    __syncthreads();
                    const bool nom = active && ((mA >> c) & 1u);
                    float vc = -INFINITY, mc = 0.0f;
#pragma unroll
                    for (int q = 0; q < NT2; ++q) {
                        const int t = w + kBigWaves * q;
                        if (t < T2) {
                            const bf32x4 cz = big_gemm(PA2, Zh, t, T2, T1, kq2, lane);
                            const float4 p4 = Pd[t * 64 + lane];
                            const float pdq[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                if (nom && (16 * t + 4 * r + j) < m) {
                                    u[q][r] = cz[r];  // the recursion restarts from the direct value
                                    vc = fmaxf(vc, cz[r] + pdq[r]);
                                    mc = fmaxf(mc, __builtin_fabsf(cz[r]) + __builtin_fabsf(pdq[r]));
                                }
                            }
                        }
                    }
#pragma unroll
                    for (int o = 16; o < 64; o <<= 1) {
                        vc = fmaxf(vc, __shfl_xor(vc, o, 64));
                        mc = fmaxf(mc, __shfl_xor(mc, o, 64));
                    }
                    if (j == 0) {  // every wave's stage-1 reads precede the barrier above
                        slots[w].violz[c] = vc;
                        slots[w].magh[c] = mc;
                    }
                    __syncthreads();
                    bool ver = false;
                    if (lane < 16 && ((mA >> lane) & 1u)) {
                        double vcc = -INFINITY, mcc = 0.0;
#pragma unroll
                        for (int s2 = 0; s2 < kBigWaves; ++s2) {
                            vcc = fmax(vcc, (double)slots[s2].violz[lane]);
                            mcc = fmax(mcc, (double)slots[s2].magh[lane]);
                        }
                        ver = viol_ok(vcc, mcc, a.L, a.tol, ViolMargin<float>::value);
                    }
                    m1 = (unsigned)__ballot(ver);
                    m2 &= ~m1;
                }
            }
            const int cdc = ((m1 >> c) & 1u) ? 1 : (((m2 >> c) & 1u) ? 2 : 0);
            if (active && (cdc != 0 || v >= N)) {  // finished column: results out
#pragma unroll
                for (int q = 0; q < NT1; ++q) {
                    const int t = w + kBigWaves * q;
                    if (t < T1) {
                        const float4 h4 = Zh[t * 64 + lane];  // this iteration's zhat (own slot)
                        const float zh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i = 16 * t + 4 * r + j;
                            if (i < n && (cdc != 2 || zh_out)) a.z[bi * n + i] = cdc == 2 ? zh[r] : z[q][r];
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < NT2; ++q) {
                    const int t = w + kBigWaves * q;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * t + 4 * r + j;
                        if (t < T2 && i < m) a.y[bi * m + i] = y[q][r];
                    }
                }
                if (w == 0 && j == 0) {
                    a.iters[inst] = v;
                    a.conv[inst] = cdc;
                }
                active = false;
            }
            live &= ~(m1 | m2);
            if (v >= N) live = 0u;
            if (v >= a.v_end || live == 0u) break;
        }
        // ---- phase end: park the survivors -----------------------------------------------------
        if (carry) {
            const bool park = active && v >= a.v_end;
            if (park) {
#pragma unroll
                for (int q = 0; q < NT1; ++q) {
                    const int t = w + kBigWaves * q;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * t + 4 * r + j;
                        if (t < T1 && i < n) a.z[bi * n + i] = z[q][r];
                    }
                }
#pragma unroll
                for (int q = 0; q < NT2; ++q) {
                    const int t = w + kBigWaves * q;
                    if (t < T2) {
                        const float4 w4 = Wl[t * 64 + lane];  // w of iteration v + 1 (own slot)
                        const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i = 16 * t + 4 * r + j;
                            if (i < m) {
                                a.y[bi * m + i] = y[q][r];
                                a.wc[bi * m + i] = wv[r];
                                if (use_tol) a.uc[bi * m + i] = u[q][r];
                            }
                        }
                    }
                }
            }
            if (w == 0) list_survivors(a, p, park, inst, lane, j);  // lanes 0..15 speak for the columns
        }
        __syncthreads();  // the next panel reuses the LDS tiles
    }
}

template <int NT1, int NT2>
static hipError_t launch_big_nt(const SolveArgs<float>& a, int grid, hipStream_t s) {
    const size_t lds = big_lds_bytes(a.n, a.m);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)gpad_bigpanel_kernel<NT1, NT2>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((gpad_bigpanel_kernel<NT1, NT2>), dim3(grid), dim3(64 * kBigWaves), lds, s, a);
    return hipGetLastError();
}

static int nt_of(int tiles) {  // row tiles per wave, rounded up to 1, 2 or 4
    const int q = (tiles + kBigWaves - 1) / kBigWaves;
    return q <= 1 ? 1 : (q <= 2 ? 2 : 4);
}

// one phase launch of the big-panel kernel (the phase loop is launch_panel's)
hipError_t launch_bigpanel(const SolveArgs<float>& a, int grid, hipStream_t s) {
    const int q1 = nt_of(big_tiles(a.n)), q2 = nt_of(big_tiles(a.m));
#define BIG_CASE(A, B) \
    case A * 8 + B: return launch_big_nt<A, B>(a, grid, s);
    switch (q1 * 8 + q2) {
        BIG_CASE(1, 1) BIG_CASE(1, 2) BIG_CASE(1, 4)
        BIG_CASE(2, 1) BIG_CASE(2, 2) BIG_CASE(2, 4)
        BIG_CASE(4, 1) BIG_CASE(4, 2)
        default: return launch_big_nt<4, 4>(a, grid, s);
    }
#undef BIG_CASE
}

}  // namespace gpad
