// gpad_cpanel.hip -- GPAD_KERNEL_CONDENSED for shared-matrix batches: the condensed operator on
// the f32 MFMA pipe (opt-in; NOT the reference's arithmetic, see gpad_condensed.hip / gpad.h).
//
// The panel kernels (gpad_panel.hip) run the reference's two skinny GEMMs per iteration,
// Zhat = (-ML) W and Y' = G_L Zhat.  With zhat eliminated (G_L zhat = H w + c, H = G_L (-ML),
// m x m) an iteration is ONE GEMM  S[m x 16] = H W[m x 16]  plus the 8d/8c epilogue on the dual
// side (wbar = theta-average of w, so z = -ML wbar - g_P is formed only when Algorithm 1 decides
// and at the end): half the MFMA work at n = m, one barrier per iteration.
//
// Layout: a workgroup owns a group of P panels (P = 2: 32 instances beyond 16 per CU, else 1) at a
// time, grid-stride over groups.  Default: 16 waves (4 per SIMD), wave w owns the single
// (panel, row tile) chains w and w + 16 (T = 13, P = 2: 7,7,6,6 chains per SIMD); option: 8 waves
// owning tiles w, w + 8 of all P panels, both panels' chains on one A stream.  A unit's row state
// (y, u, c) stays in the owning wave's registers, p_D and wbar in LDS.  W is double buffered in
// LDS in MFMA B-fragment order (the accumulator layout of the fragment-permuted A images equals
// the next B fragment, see gpad_panel.hip), so an iteration reads W[v & 1] and writes
// W[(v+1) & 1]: one barrier per iteration.
// The direct GEMMs of a decided test -- X = (-ML) V (V = wbar for test A, w for test B) and
// G_L X -- reuse the panel kernels' packed -ML / G_L images; the H image is packed the same way.
// Bit-exact against oracle/gpad_oracle.c orc_solve_condensed_f32 (each output row one
// ascending-k fmaf chain, as the MFMA computes it).
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "gpad_internal.h"

namespace gpad {

typedef float cf32x4 __attribute__((ext_vector_type(4)));
typedef unsigned cu32x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ int cp_pi16(int rho) { return 4 * (rho & 3) + (rho >> 2); }

// H image from the k-major Ht (Ht[k][ldm] = H[i][k]): PH[b][t][lane][q] = H[16t + pi(lane&15)][16b + 4q + (lane>>4)]
__global__ void pack_cpanel_kernel(const float* __restrict__ Ht, int m, int ldm, int T, float4* __restrict__ dst) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= T * T * 64) return;
    const int lane = idx & 63, t = (idx >> 6) % T, b = (idx >> 6) / T;
    const int row = 16 * t + cp_pi16(lane & 15);
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int col = 16 * b + 4 * q + (lane >> 4);
        v[q] = (row < m && col < m) ? Ht[(size_t)col * ldm + row] : 0.0f;
    }
    dst[idx] = make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float4 cp_f4(cu32x4 v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// acc = A[tile] (T k-blocks from L2, one block ahead) x B (LDS fragment order), ascending k
template <int T>
__device__ __forceinline__ cf32x4 cp_gemm(__amdgpu_buffer_rsrc_t PA, const float4* B, int voff, int lane) {
    cf32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    float4 a[2], b[2];
    a[0] = cp_f4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, 0, 0));
    b[0] = B[lane];
#pragma unroll
    for (int kb = 0; kb < T; ++kb) {
        const int cur = kb & 1, nxt = cur ^ 1;
        if (kb + 1 < T) {
            a[nxt] = cp_f4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb + 1) * T * 1024, 0));
            b[nxt] = B[(kb + 1) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].x, b[cur].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].y, b[cur].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].z, b[cur].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].w, b[cur].w, acc, 0, 0, 0);
        asm volatile("" ::: "memory");
    }
    return acc;
}

struct CpSlot {  // per unit: per column partials of the Algorithm-1 test
    float violz[16], violh[16], wmin[16], magh[16];
    double gap[16];
};

template <int T, int P>
struct CpLds {
    float4 W[P][2][T * 64];  // w, double buffered (B of the H GEMM)
    float4 WB[P][T * 64];    // wbar (B of test A's direct GEMM and of the final z)
    float4 Z[P][T * 64];     // X = -ML V - g_P (B of the direct G_L GEMM); g_P at group start
    float4 PD[P][T * 64];    // p_D of the unit rows (parked in LDS, not VGPRs)
    CpSlot slots[P * T];
};
constexpr int kCpMaxTiles = 14;  // LDS: 6 T KiB per panel + slots <= 160 KiB

// 16 waves: wave w owns the single (panel, tile) units w, w+16 (unit u = panel u / T, tile u % T),
// 4 waves per SIMD, every chain its own A stream -- at P = 2, T = 13 the SIMDs carry 7,7,6,6
// chains.  (An 8-wave deal with both panels' chains on one A stream measured slower, 2.68 vs
// 2.43 ms at the C4 shard, profiles/r02_condensed_panel_waves.txt, and was removed in round 3.)
template <int T, int P>
__global__ __launch_bounds__(1024) void gpad_cpanel_kernel(SolveArgs<float> a) {
    constexpr int kCpPanels = P;  // panels per group: 2 (32 instances) or 1 (16)
    constexpr int WV = 16;
    constexpr int NU = (P * T + WV - 1) / WV;  // units per wave
    constexpr int PU = 1;  // panels per unit
    extern __shared__ __attribute__((aligned(16))) float4 cp_lds[];
    CpLds<T, P>* Lp = reinterpret_cast<CpLds<T, P>*>(cp_lds);
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = lane >> 4, c = lane & 15;
    const int n = a.n, m = a.m, N = a.N, K = a.check_every;
    const int abytes = T * T * 1024;
    const __amdgpu_buffer_rsrc_t PA1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.frag), 0, abytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t PA2 =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)a.frag + abytes), 0, abytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t PH = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.hfrag), 0, abytes, 0x00020000);
    const bool use_tol = a.tol > 0.0;
    const int count = a.batch;
    const int groups = (count + 16 * kCpPanels - 1) / (16 * kCpPanels);
    auto uid = [&](int q) { return w + WV * q; };
    auto tile = [&](int q) { return uid(q) % T; };
    auto uvalid = [&](int q) { return uid(q) < P * T; };
    auto upan = [&](int q, int) { return uid(q) / T; };  // panel of unit q
    // acc[0] = A (tile of unit q) x B of the unit's panel
    auto gemm = [&](int q, __amdgpu_buffer_rsrc_t PA, const float4* B0, const float4* B1, cf32x4 (&acc)[2]) {
        acc[0] = cp_gemm<T>(PA, upan(q, 0) ? B1 : B0, tile(q) * 1024 + lane * 16, lane);
    };

    for (int grp = blockIdx.x; grp < groups; grp += gridDim.x) {
        const int k0 = 16 * kCpPanels * grp;
        unsigned live = 0u;  // bit 16 pp + c: column c of panel pp holds an unfinished instance
        for (int pp = 0; pp < kCpPanels; ++pp) {
            const int left = count - k0 - 16 * pp;
            live |= (left >= 16 ? 0xFFFFu : (left > 0 ? (1u << left) - 1u : 0u)) << (16 * pp);
        }
        // ---- unit state (y, u, c in registers; p_D, wbar, w in LDS); g_P into Z -----------------
        float y[NU][PU][4], u[NU][PU][4], cv[NU][PU][4];
#pragma unroll
        for (int q = 0; q < NU; ++q) {
            const int t = tile(q), fo = t * 64 + lane;
#pragma unroll
            for (int k = 0; k < PU; ++k) {
                const int pp = upan(q, k);
                const int col = k0 + 16 * pp + c;
                const bool act = uvalid(q) && col < count;
                float gp[4], wv[4], pdv[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * t + 4 * r + j;
                    const bool okm = act && i < m, okn = act && i < n;
                    y[q][k][r] = okm ? a.y[(size_t)col * m + i] : 0.0f;
                    pdv[r] = okm ? (float)(a.gscale * (double)a.g[(size_t)col * a.ld_g + i]) : 0.0f;
                    gp[r] = okn ? a.gP[(size_t)col * a.ld_gP + i] : 0.0f;
                    wv[r] = __builtin_fmaf(a.beta[0], y[q][k][r] - y[q][k][r], y[q][k][r]);
                    u[q][k][r] = 0.0f;  // theta_0 = 1: u_0 = s whatever the seed
                }
                if (uvalid(q)) {
                    Lp->Z[pp][fo] = make_float4(gp[0], gp[1], gp[2], gp[3]);
                    Lp->W[pp][0][fo] = make_float4(wv[0], wv[1], wv[2], wv[3]);
                    Lp->WB[pp][fo] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    Lp->PD[pp][fo] = make_float4(pdv[0], pdv[1], pdv[2], pdv[3]);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NU; ++q) {  // c = -G_L g_P (one chain per row, as orc_chain)
            cf32x4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
            if (uvalid(q)) gemm(q, PA2, Lp->Z[0], Lp->Z[P - 1], acc);
#pragma unroll
            for (int k = 0; k < PU; ++k)
#pragma unroll
                for (int r = 0; r < 4; ++r) cv[q][k][r] = -acc[k][r];
        }
        __syncthreads();  // Z is rewritten by the tests

        // X = -ML V - g_P (V: B0 / B1, fragment order) into Z; all threads call it (barrier after);
        // the caller then runs G_L X per unit (gemm(q, PA2, Z...)) and reads X back from Z
        auto direct_x = [&](const float4* B0, const float4* B1) {
#pragma unroll
            for (int q = 0; q < NU; ++q) {
                const int t = tile(q);
                if (uvalid(q)) {
                    cf32x4 acc[2];
                    gemm(q, PA1, B0, B1, acc);
#pragma unroll
                    for (int k = 0; k < PU; ++k) {
                const int pp = upan(q, k);
                        const int col = k0 + 16 * pp + c;
                        float xo[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i = 16 * t + 4 * r + j;
                            const float gpi = (i < n && col < count) ? a.gP[(size_t)col * a.ld_gP + i] : 0.0f;
                            xo[r] = i < n ? acc[k][r] - gpi : 0.0f;  // seq_functions.cpp:61-62 order
                        }
                        Lp->Z[pp][t * 64 + lane] = make_float4(xo[0], xo[1], xo[2], xo[3]);
                    }
                }
            }
            __syncthreads();
        };
        // per-column reduction of a panel's tile slots (lane = 16 pp + c, lane < 32)
        auto reduce = [&](double& vz, double& vh, double& mh, double& wm, double& gq) {
            vz = -INFINITY;
            vh = -INFINITY;
            mh = 0.0;
            wm = INFINITY;
            gq = 0.0;
            const int pp = lane >> 4;
            if (pp < kCpPanels)
                for (int s2 = pp * T; s2 < (pp + 1) * T; ++s2) {
                    vz = fmax(vz, (double)Lp->slots[s2].violz[c]);
                    vh = fmax(vh, (double)Lp->slots[s2].violh[c]);
                    mh = fmax(mh, (double)Lp->slots[s2].magh[c]);
                    wm = fmin(wm, (double)Lp->slots[s2].wmin[c]);
                    gq += Lp->slots[s2].gap[c];
                }
        };
        auto publish = [&](int pp, int t, float vz, float vh, float mh, float wm, double gp) {
#pragma unroll
            for (int o = 16; o < 64; o <<= 1) {
                vz = fmaxf(vz, __shfl_xor(vz, o, 64));
                vh = fmaxf(vh, __shfl_xor(vh, o, 64));
                mh = fmaxf(mh, __shfl_xor(mh, o, 64));
                wm = fminf(wm, __shfl_xor(wm, o, 64));
                gp += __shfl_xor(gp, o, 64);
            }
            if (j == 0) {
                CpSlot& sl = Lp->slots[pp * T + t];
                sl.violz[c] = vz;
                sl.violh[c] = vh;
                sl.magh[c] = mh;
                sl.wmin[c] = wm;
                sl.gap[c] = gp;
            }
        };
        // results of the columns in `done`: z rows from Z (the last direct_x), y from the registers
        auto put_out = [&](unsigned done, int v, int code) {
#pragma unroll
            for (int q = 0; q < NU; ++q) {
                const int t = tile(q);
                if (uvalid(q)) {
#pragma unroll
                    for (int k = 0; k < PU; ++k) {
                const int pp = upan(q, k);
                        const int bit = 16 * pp + c;
                        if ((done >> bit) & 1u) {
                            const size_t col = (size_t)(k0 + bit);
                            const float4 x4 = Lp->Z[pp][t * 64 + lane];
                            const float xo[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int i = 16 * t + 4 * r + j;
                                if (i < n) a.z[col * n + i] = xo[r];
                                if (i < m) a.y[col * m + i] = y[q][k][r];
                            }
                        }
                    }
                }
            }
            if (w == 0 && lane < 32 && ((done >> lane) & 1u)) {
                a.iters[k0 + lane] = v;
                a.conv[k0 + lane] = code;
            }
        };

        int v = 0;
        float th = a.theta[0], bn = a.beta[1];
        while (true) {
            const float th_next = a.theta[v + 1], bn_next = a.beta[v + 2];
            const int rb = v & 1;
            ++v;
            const bool chk = use_tol && (v % K) == 0;
            const float omt = 1.0f - th;
            {
#pragma unroll
                for (int q = 0; q < NU; ++q) {
                    const int t = tile(q), fo = t * 64 + lane;
                    if (uvalid(q)) {
                        cf32x4 acc[2];
                        gemm(q, PH, Lp->W[0][rb], Lp->W[P - 1][rb], acc);
#pragma unroll
                        for (int k = 0; k < PU; ++k) {
                const int pp = upan(q, k);
                            const bool act = (live >> (16 * pp + c)) & 1u;
                            const float4 w4 = Lp->W[pp][rb][fo], b4 = Lp->WB[pp][fo], p4 = Lp->PD[pp][fo];
                            const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
                            const float wbv[4] = {b4.x, b4.y, b4.z, b4.w};
                            const float pdv[4] = {p4.x, p4.y, p4.z, p4.w};
                            float wn[4], wbn[4];
                            float vz = -INFINITY, vh = -INFINITY, mh = 0.0f, wm = INFINITY;
                            double gp = 0.0;
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const float sc = acc[k][r] + cv[q][k][r];  // G_L zhat, condensed
                                wbn[r] = __builtin_fmaf(omt, wbv[r], th * wv[r]);
                                const float sv = (wv[r] + pdv[r]) + sc;
                                const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;
                                const float un2 = __builtin_fmaf(omt, u[q][k][r], th * sc);
                                wn[r] = __builtin_fmaf(bn, yp - y[q][k][r], yp);
                                if (act) {
                                    if (use_tol) u[q][k][r] = un2;
                                    y[q][k][r] = yp;
                                }
                                if (chk && act && 16 * t + 4 * r + j < m) {
                                    const float tt = sc + pdv[r];
                                    vz = fmaxf(vz, u[q][k][r] + pdv[r]);
                                    vh = fmaxf(vh, tt);
                                    mh = fmaxf(mh, __builtin_fabsf(sc) + __builtin_fabsf(pdv[r]));
                                    wm = fminf(wm, wv[r]);
                                    gp -= (double)wv[r] * (double)tt;
                                }
                            }
                            if (act) {
                                Lp->W[pp][rb ^ 1][fo] = make_float4(wn[0], wn[1], wn[2], wn[3]);
                                Lp->WB[pp][fo] = make_float4(wbn[0], wbn[1], wbn[2], wbn[3]);
                            } else {
                                Lp->W[pp][rb ^ 1][fo] = w4;
                            }
                            if (chk) publish(pp, t, vz, vh, mh, wm, gp);
                        }
                    }
                }
            }
            th = th_next;
            bn = bn_next;
            __syncthreads();
            if (!chk && v < a.v_end) continue;

            if (chk) {
                double vz, vh, mh, wm, gq;
                reduce(vz, vh, mh, wm, gq);
                const bool mine = lane < 16 * kCpPanels && ((live >> (lane & 31)) & 1u);
                const bool nomA = mine && vz * a.L <= a.tol;
                const bool nomB = mine && viol_ok(vh, mh, a.L, a.tol, ViolMargin<float>::value) && wm >= 0.0 &&
                                  gq * a.L <= a.tol_gap;
                const unsigned mA = (unsigned)__ballot(nomA);
                const unsigned mB = (unsigned)__ballot(nomB);
                __syncthreads();  // every wave's slot reads precede the rewrites below
                if (mA) {  // (A): decide on G_L z of z = -ML wbar - g_P, u reset to it
                    direct_x(Lp->WB[0], Lp->WB[P - 1]);
#pragma unroll
                    for (int q = 0; q < NU; ++q) {
                        const int t = tile(q);
                        if (uvalid(q)) {
                            cf32x4 gz[2];
                            gemm(q, PA2, Lp->Z[0], Lp->Z[P - 1], gz);
#pragma unroll
                            for (int k = 0; k < PU; ++k) {
                const int pp = upan(q, k);
                                const bool nom = (mA >> (16 * pp + c)) & 1u;
                                const float4 p4 = Lp->PD[pp][t * 64 + lane];
                                const float pdv[4] = {p4.x, p4.y, p4.z, p4.w};
                                float vc = -INFINITY, mc = 0.0f;
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    if (nom) u[q][k][r] = gz[k][r];
                                    if (nom && 16 * t + 4 * r + j < m) {
                                        vc = fmaxf(vc, gz[k][r] + pdv[r]);
                                        mc = fmaxf(mc, __builtin_fabsf(gz[k][r]) + __builtin_fabsf(pdv[r]));
                                    }
                                }
                                publish(pp, t, vc, -INFINITY, mc, INFINITY, 0.0);
                            }
                        }
                    }
                    __syncthreads();
                    reduce(vz, vh, mh, wm, gq);
                    const unsigned m1 = (unsigned)__ballot(lane < 32 && ((mA >> (lane & 31)) & 1u) &&
                                                           viol_ok(vz, mh, a.L, a.tol, ViolMargin<float>::value)) &
                                        live;
                    if (m1) put_out(m1, v, 1);
                    live &= ~m1;
                    __syncthreads();  // slot reads before the (B) rewrites
                }
                const unsigned mBv = mB & live;
                if (mBv) {  // (B): decide on G_L zhat of zhat = -ML w - g_P (w: W[rb], intact)
                    direct_x(Lp->W[0][rb], Lp->W[P - 1][rb]);
#pragma unroll
                    for (int q = 0; q < NU; ++q) {
                        const int t = tile(q);
                        if (uvalid(q)) {
                            cf32x4 gh[2];
                            gemm(q, PA2, Lp->Z[0], Lp->Z[P - 1], gh);
#pragma unroll
                            for (int k = 0; k < PU; ++k) {
                const int pp = upan(q, k);
                                const bool nom = (mBv >> (16 * pp + c)) & 1u;
                                const float4 w4 = Lp->W[pp][rb][t * 64 + lane], p4 = Lp->PD[pp][t * 64 + lane];
                                const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
                                const float pdv[4] = {p4.x, p4.y, p4.z, p4.w};
                                float vh2 = -INFINITY, mh2 = 0.0f, wm2 = INFINITY;
                                double gp2 = 0.0;
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    if (nom && 16 * t + 4 * r + j < m) {
                                        const float tt = gh[k][r] + pdv[r];
                                        vh2 = fmaxf(vh2, tt);
                                        mh2 = fmaxf(mh2, __builtin_fabsf(gh[k][r]) + __builtin_fabsf(pdv[r]));
                                        wm2 = fminf(wm2, wv[r]);
                                        gp2 -= (double)wv[r] * (double)tt;
                                    }
                                }
                                publish(pp, t, -INFINITY, vh2, mh2, wm2, gp2);
                            }
                        }
                    }
                    __syncthreads();
                    reduce(vz, vh, mh, wm, gq);
                    const unsigned m2 = (unsigned)__ballot(lane < 32 && ((mBv >> (lane & 31)) & 1u) &&
                                                           viol_ok(vh, mh, a.L, a.tol, ViolMargin<float>::value) &&
                                                           wm >= 0.0 && gq * a.L <= a.tol_gap) &
                                        live;
                    if (m2) put_out(m2, v, 2);
                    live &= ~m2;
                }
            }
            if (v >= N && live) {  // the rest ran out of iterations: z = -ML wbar - g_P
                __syncthreads();
                direct_x(Lp->WB[0], Lp->WB[P - 1]);
                put_out(live, v, 0);
                live = 0u;
            }
            if (live == 0u || v >= a.v_end) break;
            if (chk) __syncthreads();  // the tests' LDS traffic precedes the next iteration
        }
        // ---- phase end (a.v_end < N): park the survivors for the latency finisher ----------------
        // y in place; the next w, wbar and u in the carry buffers; ids appended to idx_out
        if (a.v_end < N && live) {
#pragma unroll
            for (int q = 0; q < NU; ++q) {
                const int t = tile(q), fo = t * 64 + lane;
                if (uvalid(q)) {
#pragma unroll
                    for (int k = 0; k < PU; ++k) {
                const int pp = upan(q, k);
                        const int bit = 16 * pp + c;
                        if ((live >> bit) & 1u) {
                            const size_t col = (size_t)(k0 + bit);
                            const float4 w4 = Lp->W[pp][v & 1][fo], b4 = Lp->WB[pp][fo];
                            const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
                            const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int i = 16 * t + 4 * r + j;
                                if (i < m) {
                                    a.y[col * m + i] = y[q][k][r];
                                    a.wc[col * m + i] = wv[r];
                                    a.wbc[col * m + i] = bv[r];
                                    a.uc[col * m + i] = u[q][k][r];
                                    a.cc[col * m + i] = cv[q][k][r];
                                }
                            }
                        }
                    }
                }
            }
            if (w == 0) {
                const bool mine = lane < 32 && ((live >> (lane & 31)) & 1u);
                int base = 0;
                if (lane == 0) base = atomicAdd(a.count_out, (int)__popc(live));
                base = __shfl(base, 0, 64);
                if (mine) a.idx_out[base + (int)__popc(live & ((1u << lane) - 1u))] = k0 + lane;
            }
        }
        __syncthreads();  // the next group reuses the LDS arrays
    }
}

bool cpanel_supported(int n, int m) {
    const int T = ((n > m ? n : m) + 15) / 16;
    return T >= 1 && T <= kCpMaxTiles;
}

size_t cpanel_frag_bytes(int n, int m) {
    const int T = ((n > m ? n : m) + 15) / 16;
    return (size_t)T * T * 1024;
}

hipError_t launch_pack_cpanel(const float* Ht, int n, int m, int ldm, void* hfrag, hipStream_t s) {
    const int T = ((n > m ? n : m) + 15) / 16;
    const int tot = T * T * 64;
    hipLaunchKernelGGL(pack_cpanel_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, Ht, m, ldm, T,
                       reinterpret_cast<float4*>(hfrag));
    return hipGetLastError();
}

template <int T, int P>
static hipError_t launch_cp_tp(const SolveArgs<float>& a, hipStream_t s) {
    const size_t lds = sizeof(CpLds<T, P>);
    hipError_t e = hipFuncSetAttribute((const void*)gpad_cpanel_kernel<T, P>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    const int groups = (a.batch + 16 * P - 1) / (16 * P);
    const int grid = groups < a.num_cus ? groups : a.num_cus;
    hipLaunchKernelGGL((gpad_cpanel_kernel<T, P>), dim3(grid), dim3(1024), lds, s, a);
    return hipGetLastError();
}
// two panels per group once single panels outnumber the CUs (a group's iteration is latency-bound:
// one panel per CU halves it while the batch fits one round)
static int cp_panels(int batch, int num_cus) { return batch > 16 * num_cus ? 2 : 1; }
template <int T>
static hipError_t launch_cp_t(const SolveArgs<float>& a, hipStream_t s) {
    return cp_panels(a.batch, a.num_cus) == 2 ? launch_cp_tp<T, 2>(a, s) : launch_cp_tp<T, 1>(a, s);
}

// Takeover iteration of an eps-mode condensed batch from the previous solve's counts: the panels
// cost ~t_p per iteration while any group is alive (each CU runs its group at the group's
// latency); the latency kernel finishes the survivors two per CU (DPP issue shared, ~1.6 us per
// iteration each) after a ~25 us start (H rows and c per workgroup).  Pick the test iteration v
// minimising  v t_p + 25 + max(max_i (it_i - v) 1.6, sum_i (it_i - v)+ 1.6 / CUs)  [us].
// t_p: the busiest SIMD's MFMA chains (ceil(P T / 4)) at 32 cycles per MFMA + ~1.5 us.  Calibrated
// on the C4 shard (tools/cond_take_sweep.py, profiles/r02_cond_takeover.jsonl: t_p = 6.8 us;
// forced takeovers 260 / 280 / 300 / 330 / none: 2.69 / 2.32 / 2.25 / 2.37 / 2.58 ms).
int cpanel_takeover(const int* iters, int batch, int n, int m, int N, int check_every, int num_cus) {
    const int T = ((n > m ? n : m) + 15) / 16;
    const int chains_simd = (cp_panels(batch, num_cus) * T + 3) / 4;  // 16-wave single-chain deal
    const double tp = chains_simd * T * 4 * 32 / 2.2e3 + 1.5;        // us
    const double tl = 1.6 * (m / 200.0 > 0.25 ? m / 200.0 : 0.25);   // us per iteration, 2 per CU
    const int K = check_every > 0 ? check_every : 10;
    int mx = 0;
    for (int b = 0; b < batch; ++b) mx = iters[b] > mx ? iters[b] : mx;
    // survivors and remaining work past every v from one histogram of the counts: O(batch + mx)
    std::vector<long long> cnt((size_t)mx + 2, 0);
    for (int b = 0; b < batch; ++b) cnt[iters[b] > 0 ? iters[b] : 0]++;
    std::vector<long long> above((size_t)mx + 2, 0), rem((size_t)mx + 2, 0);  // #(it > v), sum (it - v)+
    for (int v = mx - 1; v >= 0; --v) {
        above[v] = above[v + 1] + cnt[v + 1];
        rem[v] = rem[v + 1] + above[v];
    }
    int best_v = N;
    double best = 1e300;
    for (int v = K; v < mx && v < N; v += K) {
        const double lat = (mx - v) * tl, thr = rem[v] * tl / num_cus;
        const double cost = v * tp + 25.0 + (lat > thr ? lat : thr);
        if (cost < best) {
            best = cost;
            best_v = v;
        }
    }
    const double none = mx * tp;  // panels to the end
    return none <= best ? 0 : best_v;
}

hipError_t launch_cpanel(const SolveArgs<float>& a, hipStream_t s, bool* supported) {
    const int T = ((a.n > a.m ? a.n : a.m) + 15) / 16;
    *supported = cpanel_supported(a.n, a.m) && a.frag && a.hfrag && a.frag_tiles == T && a.strideA == 0 &&
                 a.strideB == 0;
    if (!*supported) return hipSuccess;
    switch (T) {
        case 1: return launch_cp_t<1>(a, s);
        case 2: return launch_cp_t<2>(a, s);
        case 3: return launch_cp_t<3>(a, s);
        case 4: return launch_cp_t<4>(a, s);
        case 5: return launch_cp_t<5>(a, s);
        case 6: return launch_cp_t<6>(a, s);
        case 7: return launch_cp_t<7>(a, s);
        case 8: return launch_cp_t<8>(a, s);
        case 9: return launch_cp_t<9>(a, s);
        case 10: return launch_cp_t<10>(a, s);
        case 11: return launch_cp_t<11>(a, s);
        case 12: return launch_cp_t<12>(a, s);
        case 13: return launch_cp_t<13>(a, s);
        default: return launch_cp_t<14>(a, s);
    }
}

}  // namespace gpad
