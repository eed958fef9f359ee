// gpad_quad.hip -- the four-column ping-pong finisher (shared matrices): the duo kernel's layout
// (gpad_duo.hip) with four instances per slot on the matrix core.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <utility>

#include "gpad_chain.h"
#include "gpad_internal.h"

namespace gpad {

// =========================================================================================
// gpad_quad_kernel: shared matrices, two slots of FOUR instances per workgroup, fed by a queue.
// =========================================================================================
// The duo finisher (gpad_duo.hip) runs one instance per slot as a DPP fmac chain: a lane holds one
// matrix row in VGPRs and the vector element of step k arrives by a row broadcast.  Two slots per
// CU already saturate the SIMD's DPP issue (10.2 cycles per step with two waves), so the duo's
// throughput is ~0.8 instance-iterations per us per CU -- a fifth of a panel's.
//
// Here each slot holds four instances and the 8b / 8d chains run on the matrix core:
// v_mfma_f32_4x4x1_16b_f32 with the instance vectors in A, broadcast from one block (cbsz:4
// abid:t), and the register-resident matrix rows in B:
//     D_b[i][j] += x_i[k] * M[4b + j][k]      (lane 4b + j = row, VGPR i = instance)
// so lane l accumulates row l of all four instances, in ascending k, each step one fused
// multiply-add with one rounding -- bitwise the reference's sequential fmaf chain
// (tools/lat/quad_bcast.hip: 0 of 256 differ) -- and the per-row state (z, y, u) keeps the duo's
// lane = row layout, one VGPR per instance.  Lane 4t + i of a ring register holds x_i[64h + 4t + c]
// in component c: one ds_read_b128 per lane feeds 64 chain steps.  A dependent 4x4x1 step costs 15
// cycles (20.5 with the partner slot's chain on the same SIMD) against the DPP step's 5.9 (10.2),
// for four instances instead of one.
//
// A slot with a single live instance runs it as the duo's DPP chain instead (lower latency), so a
// CU whose queue has drained finishes its last instances at the duo's speed.  The LDS vectors are
// instance-major ([column][k], padded to 64), which both chains read directly.
//
// Columns are refilled one by one from the work list as their instances finish (the duo's queue:
// list positions g + c G first, c = 4 slot + column, then claims from a.qctr one ahead).  Every
// column runs its own iteration index (theta / beta per column); instances only finish at tests
// or at N, and a refilled column starts at the list's v_begin, so the columns of a slot normally
// test together -- the code does not rely on it (per-column test flags).
//
// The arithmetic per instance is exactly the duo's / resident kernel's (same chains, same
// epilogues, same test with the same wave reductions), hence bit-identical results and
// iteration counts with the oracle whichever engine (MFMA or DPP) ran which iteration.
typedef float qf4 __attribute__((ext_vector_type(4)));

template <int S>
__device__ __forceinline__ float comp4(const float4& x) {
    if constexpr ((S & 3) == 0) return x.x;
    else if constexpr ((S & 3) == 1) return x.y;
    else if constexpr ((S & 3) == 2) return x.z;
    else return x.w;
}

// steps 64 H + S .. of the chain (S < 64, k < KLEN)
template <int KLEN, int K, int H, int S>
__device__ __forceinline__ void quad_steps(qf4& acc, const float4& x, const float (&r)[K]) {
    if constexpr (S < 64 && 64 * H + S < KLEN) {
        acc = __builtin_amdgcn_mfma_f32_4x4x1f32(comp4<S>(x), r[64 * H + S], acc, 4, S >> 2, 0);
        quad_steps<KLEN, K, H, S + 1>(acc, x, r);
    }
}

template <int KLEN, int K, int H>
__device__ __forceinline__ void quad_groups(qf4& acc, float4 (&ring)[2], const float (&r)[K], const float* xb) {
    constexpr int NH = (KLEN + 63) / 64;
    if constexpr (H < NH) {
        if constexpr (H + 1 < NH) ring[(H + 1) & 1] = *reinterpret_cast<const float4*>(xb + 64 * (H + 1));
        quad_steps<KLEN, K, H, 0>(acc, ring[H & 1], r);
        quad_groups<KLEN, K, H + 1>(acc, ring, r, xb);
    }
}

// acc[i] = sum_k x_i[k] r[k], k = 0..KLEN-1 in ascending order, for the four columns of x (LDS,
// [4][P], P a multiple of 64): this lane's row of four instances
template <int KLEN, int K, int P>
__device__ __forceinline__ qf4 quad_chain(const float (&r)[K], const float* x) {
    static_assert(KLEN % 8 == 0 && KLEN <= K && KLEN <= P && P % 64 == 0, "bad quad chain");
    const int l = threadIdx.x & 63;
    const float* xb = x + (l & 3) * P + 4 * (l >> 2);
    float4 ring[2];
    ring[0] = *reinterpret_cast<const float4*>(xb);
    qf4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    quad_groups<KLEN, K, 0>(acc, ring, r, xb);
    return acc;
}

// either engine for the live columns of a slot (mask, uniform): four on the matrix core, or the
// one live column i0 on the DPP chain (its result in component i0, the others zero)
template <int KLEN, int K, int P>
__device__ __forceinline__ qf4 slot_chain(const float (&r)[K], const float* x, unsigned mask) {
    if (__builtin_popcount(mask) >= 2) return quad_chain<KLEN, K, P>(r, x);
    const int i0 = __builtin_ctz(mask);
    const float d = chain_regs<KLEN, K>(r, x + i0 * P);
    qf4 acc;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = i == i0 ? d : 0.0f;
    return acc;
}

struct QuadSlot {       // bookkeeping uniform (scalar); x0, x1: this lane's row of the 4 instances
    int pos[4];         // list position per column (>= count: empty)
    int vs[4];          // iterations done
    int nextp[4];       // pre-claimed next position
    float th[4], bn[4]; // theta_vs, beta_{vs+1}
    bool need8d;        // 8b done, 8d pending
    qf4 x0;             // -ML lanes: z;  G/L lanes: y  (u = G_L z in LDS: the rows take 200 VGPRs)
};
struct QuadCtx {
    int tid, count, G, v0, n, m, N, Kc, nA, nwaves, row, claim_base;
    bool fresh, use_tol, isA, live;
};

template <int PA, int PB>
struct QuadLds {
    float xw[2][4][PA];    // w per slot and column (broadcast to the -ML rows)
    float xz[2][4][PB];    // zhat per slot and column (to the G/L rows)
    float zl[4][PB];       // z of a slot's columns: verification chains and fresh u seeds
    float gp[2][4][PB];    // g_P of the -ML rows
    float pd[2][4][PA];    // p_D of the G/L rows
    float ul[2][4][PA];    // u = G_L z of the G/L rows (the 8c recursion of test (A))
    CheckSlot slots[2][4][kResidentMaxThreads / 64];
    CheckSlot vslots[4][kResidentMaxThreads / 64];
    int claim[2][4];
};

__device__ __forceinline__ unsigned live_mask(const QuadSlot& s, int count) {
    unsigned m = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) m |= (s.pos[i] < count ? 1u : 0u) << i;
    return m;
}

// columns `mask` of slot SL take their pre-claimed positions (claiming the next ones); uniform,
// contains barriers.  Loads as gpad_duo.hip duo_refill; a fresh start with a tolerance seeds
// u = G_L z_{-1} by one chain over the refilled columns' z.
template <int SL, int KB, int K, int PA, int PB>
__device__ __forceinline__ void quad_refill(const SolveArgs<float>& a, const QuadCtx& c, QuadSlot& s, unsigned mask,
                                            QuadLds<PA, PB>& L, const float (&r)[K]) {
    unsigned seeded = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (!((mask >> i) & 1u)) continue;
        const int p = s.nextp[i];
        if (c.tid == 0 && p < c.count) L.claim[SL][i] = c.claim_base + atomicAdd(a.qctr, 1);
        s.pos[i] = __builtin_amdgcn_readfirstlane(p);
        s.vs[i] = c.v0;
        s.th[i] = a.theta[c.v0];
        s.bn[i] = a.beta[c.v0 + 1];
        s.x0[i] = 0.0f;
        if (p < c.count) {
            const size_t b = (size_t)(a.idx_in ? a.idx_in[p] : p);
            if (c.isA) {
                if (c.live) {
                    const float zv = a.z[b * c.n + c.row];
                    s.x0[i] = zv;
                    L.gp[SL][i][c.row] = a.gP[b * a.ld_gP + c.row];
                    if (c.fresh && c.use_tol) L.zl[i][c.row] = zv;
                }
            } else if (c.live) {
                const float yv = a.y[b * c.m + c.row];
                s.x0[i] = yv;
                L.pd[SL][i][c.row] = (float)(a.gscale * (double)a.g[b * a.ld_g + c.row]);
                L.xw[SL][i][c.row] = c.fresh ? __builtin_fmaf(a.beta[0], yv - yv, yv) : a.wc[b * c.m + c.row];
                L.ul[SL][i][c.row] = (c.use_tol && !c.fresh) ? a.uc[b * c.m + c.row] : 0.0f;
            }
            seeded |= 1u << i;
        }
        asm volatile("" ::: "memory");  // one column's loads at a time (hoisted together they spill the rows)
    }
    __syncthreads();  // (publishes the claims)
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if ((mask >> i) & 1u)
            s.nextp[i] = s.pos[i] < c.count ? __builtin_amdgcn_readfirstlane(L.claim[SL][i]) : c.count;
    if (seeded && c.fresh && c.use_tol) {  // u = G_L z_{-1}, then the 8c recursion
        if (!c.isA) {
            const qf4 us = slot_chain<KB, K, PB>(r, &L.zl[0][0], seeded);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (((seeded >> i) & 1u) && c.live) L.ul[SL][i][c.row] = us[i];
        }
        __syncthreads();  // zl free again
    }
}

// one step: -ML waves run 8b+8c of slot SA, G/L waves 8d+8a (+ test) of slot SB
template <int SA, int SB, int KA, int KB, int K, int PA, int PB>
__device__ __forceinline__ void quad_step(const SolveArgs<float>& a, const QuadCtx& c, QuadSlot& sa, QuadSlot& sb,
                                          QuadLds<PA, PB>& L, const float (&r)[K]) {
    const unsigned ma = __builtin_amdgcn_readfirstlane(live_mask(sa, c.count));
    const unsigned mb = __builtin_amdgcn_readfirstlane(live_mask(sb, c.count));
    const bool runA = ma && !sa.need8d;
    const bool runB = sb.need8d;  // (a slot with 8d pending has live columns)
    unsigned chk = 0u;            // columns of SB whose test falls on this iteration
    if (runB && c.use_tol) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (((mb >> i) & 1u) && ((sb.vs[i] + 1) % c.Kc) == 0) chk |= 1u << i;
    }
    if (c.isA) {
        if (runA) {
            const qf4 acc = slot_chain<KA, K, PA>(r, &L.xw[SA][0][0], ma);
            if (c.live) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float th = sa.th[i];
                    const float zhv = acc[i] - L.gp[SA][i][c.row];
                    sa.x0[i] = __builtin_fmaf(1.0f - th, sa.x0[i], th * zhv);
                    L.xz[SA][i][c.row] = ((ma >> i) & 1u) ? zhv : 0.0f;
                }
            }
        }
    } else if (runB) {
        const qf4 cv = slot_chain<KB, K, PB>(r, &L.xz[SB][0][0], mb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float th = sb.th[i], bn = sb.bn[i];
            float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
            double gap = 0.0;
            const bool ck = (chk >> i) & 1u;
            if (c.live) {
                const float pdi = L.pd[SB][i][c.row], wi = L.xw[SB][i][c.row], ci = cv[i];
                const float sv = (wi + pdi) + ci;                     // seq_functions.cpp:84
                const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;   // seq_functions.cpp:85
                float ui = 0.0f;
                if (c.use_tol) {
                    ui = __builtin_fmaf(1.0f - th, L.ul[SB][i][c.row], th * ci);
                    L.ul[SB][i][c.row] = ui;
                }
                if (ck) {
                    const float t = ci + pdi;
                    violh = t;
                    magh = __builtin_fabsf(ci) + __builtin_fabsf(pdi);
                    wmin = wi;
                    gap = -((double)wi * (double)t);
                    violz = ui + pdi;
                }
                const float wn = __builtin_fmaf(bn, yp - sb.x0[i], yp);
                sb.x0[i] = yp;
                L.xw[SB][i][c.row] = ((mb >> i) & 1u) ? wn : 0.0f;
            }
            if (ck) check_publish<float>(L.slots[SB][i], violz, violh, wmin, gap, magh);
        }
    }
    __syncthreads();
    if (runA) sa.need8d = true;
    if (!runB) return;
    sb.need8d = false;
    unsigned nom = 0u, pass2 = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (!((mb >> i) & 1u)) continue;
        const int v = ++sb.vs[i];
        sb.th[i] = a.theta[v];  // next iteration's schedule (tables hold N + 2 entries)
        sb.bn[i] = a.beta[v + 1];
        if ((chk >> i) & 1u) {
            const int st1 = check_stage1<float>(L.slots[SB][i] + c.nA, c.nwaves - c.nA, a.L, a.tol, a.tol_gap);
            if (st1 & 1) nom |= 1u << i;
            if (st1 & 2) pass2 |= 1u << i;
        }
    }
    // the decisions come from LDS words every lane reads alike: keep them scalar, so the column
    // bookkeeping (and the control flow around the chains and barriers) stays uniform
    nom = __builtin_amdgcn_readfirstlane(nom);
    pass2 = __builtin_amdgcn_readfirstlane(pass2);
    unsigned ver = 0u;
    if (nom) {  // (A) nominated: decide on the direct chain G_L z, reset u to it
        if (c.isA && c.live) {
#pragma unroll
            for (int i = 0; i < 4; ++i) L.zl[i][c.row] = sb.x0[i];
        }
        __syncthreads();
        if (!c.isA) {
            const qf4 cz = slot_chain<KB, K, PB>(r, &L.zl[0][0], nom);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (!((nom >> i) & 1u)) continue;
                float vc = -INFINITY, mc = 0.0f;
                if (c.live) {
                    const float pdi = L.pd[SB][i][c.row];
                    L.ul[SB][i][c.row] = cz[i];
                    vc = cz[i] + pdi;
                    mc = __builtin_fabsf(cz[i]) + __builtin_fabsf(pdi);
                }
                check_publish<float>(L.vslots[i], vc, vc, vc, 0.0, mc);
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (((nom >> i) & 1u) && check_verify<float>(L.vslots[i] + c.nA, c.nwaves - c.nA, a.L, a.tol))
                ver |= 1u << i;
        ver = __builtin_amdgcn_readfirstlane(ver);
    }
    unsigned fin = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (!((mb >> i) & 1u)) continue;
        const int done = check_code(((nom >> i) & 1u) | (((pass2 >> i) & 1u) << 1), (ver >> i) & 1u);
        if (done || sb.vs[i] >= c.N) {
            const size_t b = (size_t)(a.idx_in ? a.idx_in[sb.pos[i]] : sb.pos[i]);
            if (c.live) {
                if (c.isA) a.z[b * c.n + c.row] = done == 2 ? L.xz[SB][i][c.row] : sb.x0[i];  // (B) certifies zhat
                else a.y[b * c.m + c.row] = sb.x0[i];
            }
            if (c.tid == 0) {
                a.iters[b] = sb.vs[i];
                a.conv[b] = done;
            }
            fin |= 1u << i;
        }
    }
    if (fin) quad_refill<SB, KB, K, PA, PB>(a, c, sb, fin, L, r);
}

template <int KA, int KB>
__global__ __launch_bounds__(kResidentMaxThreads) void gpad_quad_kernel(SolveArgs<float> a) {
    constexpr int K = KA > KB ? KA : KB;
    constexpr int PA = (KA + 63) / 64 * 64, PB = (KB + 63) / 64 * 64;
    __shared__ __attribute__((aligned(16))) QuadLds<PA, PB> L;

    QuadCtx c;
    c.tid = threadIdx.x;
    c.count = a.count_in ? __builtin_amdgcn_readfirstlane(*a.count_in) : a.batch;
    if (a.count_in && c.count > a.fin_thresh) return;  // the panel phase has them
    c.G = gridDim.x;
    if ((int)blockIdx.x >= c.count) return;
    c.v0 = a.v_begin;
    c.fresh = c.v0 == 0;
    c.use_tol = a.tol > 0.0;
    c.n = a.n;
    c.m = a.m;
    c.N = a.N;
    c.Kc = a.check_every;
    c.nA = (c.n + 63) >> 6;
    c.nwaves = blockDim.x >> 6;
    c.isA = (c.tid >> 6) < c.nA;
    c.row = c.isA ? c.tid : c.tid - 64 * c.nA;
    c.live = c.isA ? c.row < c.n : c.row < c.m;

    float r[K];
    {
        const int len = c.isA ? c.m : c.n;
        const float* __restrict__ Mt = c.isA ? a.MGt : a.GLt;
        const int ld = c.isA ? a.ldn : a.ldm;
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = (c.live && k < len) ? Mt[(size_t)k * ld + c.row] : 0.0f;
    }
    {
        float* f = reinterpret_cast<float*>(&L);
        using Lds = QuadLds<PA, PB>;
        for (int i = c.tid; i < (int)(offsetof(Lds, slots) / sizeof(float)); i += blockDim.x) f[i] = 0.0f;
    }
    // Static start: column q = 4 slot + i of workgroup g takes list position q G + g (the list is
    // sorted longest-predicted-first); later positions are claimed from the counter.
    c.claim_base = 8 * c.G;
    __syncthreads();  // (LDS zeroed before the refills write it)
    QuadSlot s0, s1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s0.nextp[i] = (int)blockIdx.x + i * c.G;
        s1.nextp[i] = (int)blockIdx.x + (4 + i) * c.G;
    }
    s0.need8d = s1.need8d = false;
    quad_refill<0, KB, K, PA, PB>(a, c, s0, 0xFu, L, r);
    quad_refill<1, KB, K, PA, PB>(a, c, s1, 0xFu, L, r);
    while (__builtin_amdgcn_readfirstlane(live_mask(s0, c.count) | live_mask(s1, c.count))) {
        quad_step<0, 1, KA, KB, K, PA, PB>(a, c, s0, s1, L, r);
        quad_step<1, 0, KA, KB, K, PA, PB>(a, c, s1, s0, L, r);
    }
}

template <int KA>
static void launch_quad_b(int kb, dim3 g, dim3 bl, hipStream_t st, const SolveArgs<float>& a) {
    switch (kb) {
        case 32: hipLaunchKernelGGL((gpad_quad_kernel<KA, 32>), g, bl, 0, st, a); break;
        case 64: hipLaunchKernelGGL((gpad_quad_kernel<KA, 64>), g, bl, 0, st, a); break;
        case 96: hipLaunchKernelGGL((gpad_quad_kernel<KA, 96>), g, bl, 0, st, a); break;
        case 128: hipLaunchKernelGGL((gpad_quad_kernel<KA, 128>), g, bl, 0, st, a); break;
        case 160: hipLaunchKernelGGL((gpad_quad_kernel<KA, 160>), g, bl, 0, st, a); break;
        case 192: hipLaunchKernelGGL((gpad_quad_kernel<KA, 192>), g, bl, 0, st, a); break;
        case 200: hipLaunchKernelGGL((gpad_quad_kernel<KA, 200>), g, bl, 0, st, a); break;
        default: hipLaunchKernelGGL((gpad_quad_kernel<KA, 208>), g, bl, 0, st, a); break;
    }
}

hipError_t launch_quad(const SolveArgs<float>& a, int grid, hipStream_t st) {
    if (!resident_supported(a.n, a.m) || a.strideA || a.strideB || !a.qctr || grid < 1)
        return hipErrorInvalidValue;
    const int threads = 64 * (((a.n + 63) >> 6) + ((a.m + 63) >> 6));
    const dim3 g(grid), bl(threads);
    const int ka = res_bucket(a.m), kb = res_bucket(a.n);
    switch (ka) {
        case 32: launch_quad_b<32>(kb, g, bl, st, a); break;
        case 64: launch_quad_b<64>(kb, g, bl, st, a); break;
        case 96: launch_quad_b<96>(kb, g, bl, st, a); break;
        case 128: launch_quad_b<128>(kb, g, bl, st, a); break;
        case 160: launch_quad_b<160>(kb, g, bl, st, a); break;
        case 192: launch_quad_b<192>(kb, g, bl, st, a); break;
        case 200: launch_quad_b<200>(kb, g, bl, st, a); break;
        default: launch_quad_b<208>(kb, g, bl, st, a); break;
    }
    return hipGetLastError();
}

}  // namespace gpad
