// gpad_flatpanel.hip -- the flat (equal-cell) battery path on the f32 MFMA pipe (gfx950).
//
// The flat data (ENABLE_FLATTEN_MATRICES, seq_functions.cpp:5-43; gpad_flat.hip header) define
// the two mat-vecs by their structural nonzeros only.  Over a panel of 16 instances they are
// n_u + n_u + 1 skinny GEMMs, each output row still ONE ascending-k fmaf chain in the
// reference's order (bit-exact with StepTwo/StepFourGPADFlatSequential):
//   8b, cell j (j < n_u):  zhat[i n_u + j] = A1_j[i][:] . B1_j - g_P, i < Nh, K1 = 4 Nh + E
//        A1_j[i][s] = MGf[i][j + n_u s] (s < 4 Nh), MGf[i][mc + s - 4 Nh] (the E coupling terms)
//        B1_j[s]    = w[j + n_u s],                 w[mc + s - 4 Nh]
//   8d, cell c:  constraint rows r = c + n_u s (s < 4 Nh): A2_c[s][t] = GLf[r][t], K2 = Nh,
//        B2_c[t] = zhat[t n_u + c]
//   8d, coupling rows r = mc + e (e < E): A3[e][q] = GLf[r][q / n_u], K3 = n, B3 = zhat
// (mc = 4 n_u Nh, E = m - mc).  ~3x fewer MFMAs than the full matrices at the battery shapes.
// The epilogues scatter: zhat of row (i, j) goes to B2_j[i] and B3[i n_u + j]; w of a cell row
// to B1_c[s], of a coupling row to every B1_j[4 Nh + e]; y+ = (s + w) + p_D, y+ < 0 -> 0 (the
// flat steps' order).  A workgroup (16 waves) owns a panel of 16 instances for the whole solve;
// the GEMM units (sub-GEMM, row tile) are dealt to the waves round-robin, each unit's row state
// in the owning wave's registers.  Fragment images are packed at gpad_setup_flat.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "gpad_internal.h"

namespace gpad {

typedef float ff32x4 __attribute__((ext_vector_type(4)));
constexpr int kFlatPanelWaves = 16;
constexpr int kFlatPanelWavesMax = 16;

struct FlatGeom {  // sizes in tiles / k-blocks of 16 rows; image offsets in float4s
    int n_u, Nh, n, m, mc, E;
    int KBc, KBe, KB1, kq1;  // 8b per cell: K = 16 KBc (4 Nh cell terms, zero-padded) + the E coupling terms
    int T1;                  // 8b row tiles per cell (= the k-blocks of the 8d cell GEMMs, K = Nh)
    int kq2;                 // 8d per cell: T2 = KBc row tiles, KB2 = T1 k-blocks
    int KB3, kq3;            // 8d coupling: KBe row tiles, K = n
    int U1, U2;              // units (sub-GEMM, row tile) of the two phases
    int off1c, off2, off3, total;  // images [n_u][KBc][T1] + [KBe][T1] (the coupling blocks, shared
                                   // by every cell's chain), [n_u][T1][KBc], [KB3][KBe] of 64 float4
    int PB;                  // LDS blocks per panel
    int P;                   // panels per workgroup (set by the launcher)
    // unit descriptors (set by the launcher): pp << 16 | (cell + 1) << 8 | t
    int d1[4 * kFlatPanelWavesMax];
    int d2[4 * kFlatPanelWavesMax];
};

__host__ __device__ inline int fp_ceil16(int x) { return (x + 15) / 16; }
__host__ __device__ inline int fp_kq(int K, int KB) { return (K - 16 * (KB - 1) + 3) / 4; }

__host__ __device__ inline FlatGeom flat_geom(int n, int m, int n_u) {
    FlatGeom g;
    g.n_u = n_u;
    g.Nh = n / n_u;
    g.n = n;
    g.m = m;
    g.mc = 4 * n_u * g.Nh;
    g.E = m - g.mc;
    g.KBc = fp_ceil16(4 * g.Nh);
    g.KBe = fp_ceil16(g.E);
    g.KB1 = g.KBc + g.KBe;
    g.kq1 = fp_kq(g.E, g.KBe);
    g.T1 = fp_ceil16(g.Nh);
    g.kq2 = fp_kq(g.Nh, g.T1);
    g.KB3 = fp_ceil16(n);
    g.kq3 = fp_kq(n, g.KB3);
    g.U1 = n_u * g.T1;
    g.U2 = g.KBe + n_u * g.KBc;
    g.off1c = n_u * g.KBc * g.T1 * 64;
    g.off2 = g.off1c + g.KBe * g.T1 * 64;
    g.off3 = g.off2 + n_u * g.T1 * g.KBc * 64;
    g.total = g.off3 + g.KB3 * g.KBe * 64;
    g.PB = n_u * (g.KBc + g.T1) + g.KBe + g.KB3;
    g.P = 1;
    return g;
}

// LDS, 1 KiB per block of 16 rows x 16 instances (MFMA B-fragment order):
//   W  [n_u][KBc]  w of each cell's constraint rows (row s of cell c = constraint c + n_u s)
//   We [KBe]       w of the coupling rows (one copy, the tail of every cell's 8b chain)
//   Zc [n_u][T1]   zhat per cell (row i of cell j = zhat[i n_u + j])
//   Zn [KB3]       zhat in natural order (the coupling rows' operand)
// test partials: one slot per phase-2 unit (its 16 columns, reduced over the unit's rows)
struct FlatPanelSlot {
    float violz[16], violh[16], wmin[16];
    double gap[16];
    float magh[16];  // max(|G_L zhat| + |pD|); with violz reused by the verification of test (A)
};
static size_t flatpanel_lds_bytes(const FlatGeom& g, int P) {
    return (size_t)P * g.PB * 1024 + (size_t)P * g.U2 * sizeof(FlatPanelSlot);
}

__device__ __forceinline__ int fp_pi16(int rho) { return 4 * (rho & 3) + (rho >> 2); }

// A values from the flat data as the setup stores it: MGf row-major Nh x m (sign-folded -ML),
// GLT t-major Nh x m (GLT[t][r] = GLf[r][t])
__device__ __forceinline__ float flat_a1(const FlatGeom& g, const float* MGf, int j, int i, int s) {
    if (i >= g.Nh) return 0.0f;
    if (s < 16 * g.KBc) return s < 4 * g.Nh ? MGf[(size_t)i * g.m + j + g.n_u * s] : 0.0f;
    const int e = s - 16 * g.KBc;
    return e < g.E ? MGf[(size_t)i * g.m + g.mc + e] : 0.0f;
}
__device__ __forceinline__ float flat_a2(const FlatGeom& g, const float* GLT, int c, int s, int t) {
    if (s >= 4 * g.Nh || t >= g.Nh) return 0.0f;
    return GLT[(size_t)t * g.m + c + g.n_u * s];
}
__device__ __forceinline__ float flat_a3(const FlatGeom& g, const float* GLT, int e, int q) {
    if (e >= g.E || q >= g.n) return 0.0f;
    return GLT[(size_t)(q / g.n_u) * g.m + g.mc + e];
}

__global__ void pack_flatpanel_kernel(FlatGeom g, const float* __restrict__ MGf, const float* __restrict__ GLT,
                                      float4* __restrict__ dst) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= g.total) return;
    const int lane = idx & 63;
    const int rrow = fp_pi16(lane & 15);  // row inside the tile (fragment-order permutation)
    float v[4];
    if (idx < g.off1c) {  // [n_u][KBc][T1]: the cell blocks of each cell's 8b chains
        const int blk = idx >> 6;
        const int t = blk % g.T1, b = (blk / g.T1) % g.KBc, j = blk / (g.T1 * g.KBc);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = flat_a1(g, MGf, j, 16 * t + rrow, 16 * b + 4 * q + (lane >> 4));
    } else if (idx < g.off2) {  // [KBe][T1]: the coupling blocks (the same for every cell)
        const int blk = (idx - g.off1c) >> 6;
        const int t = blk % g.T1, b = g.KBc + blk / g.T1, j = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = flat_a1(g, MGf, j, 16 * t + rrow, 16 * b + 4 * q + (lane >> 4));
    } else if (idx < g.off3) {  // [n_u][T1 k-blocks][KBc tiles]
        const int blk = (idx - g.off2) >> 6;
        const int t = blk % g.KBc, b = (blk / g.KBc) % g.T1, c = blk / (g.KBc * g.T1);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = flat_a2(g, GLT, c, 16 * t + rrow, 16 * b + 4 * q + (lane >> 4));
    } else {  // [KB3 k-blocks][KBe tiles]
        const int blk = (idx - g.off3) >> 6;
        const int t = blk % g.KBe, b = blk / g.KBe;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = flat_a3(g, GLT, 16 * t + rrow, 16 * b + 4 * q + (lane >> 4));
    }
    dst[idx] = make_float4(v[0], v[1], v[2], v[3]);
}

bool flatpanel_supported(int n, int m, int n_u) {
    if (n_u <= 0 || n % n_u || m <= 4 * n) return false;
    const FlatGeom g = flat_geom(n, m, n_u);
    return flatpanel_lds_bytes(g, 1) <= 160 * 1024 && g.U1 <= 4 * kFlatPanelWaves && g.U2 <= 4 * kFlatPanelWaves &&
           (long long)g.total * 16 < (1LL << 31) && n_u < 255 && g.KBc < 256 && g.T1 < 256;
}

size_t flatpanel_frag_bytes(int n, int m, int n_u) {
    return flatpanel_supported(n, m, n_u) ? (size_t)flat_geom(n, m, n_u).total * sizeof(float4) : 0;
}

hipError_t launch_pack_flatpanel(const float* MGf, const float* GLT, int n, int m, int n_u, void* frag,
                                 hipStream_t s) {
    const FlatGeom g = flat_geom(n, m, n_u);
    hipLaunchKernelGGL(pack_flatpanel_kernel, dim3((unsigned)((g.total + 255) / 256)), dim3(256), 0, s, g, MGf, GLT,
                       reinterpret_cast<float4*>(frag));
    return hipGetLastError();
}

__device__ __forceinline__ float4 fas_float4(__attribute__((ext_vector_type(4))) unsigned v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

// one unit's chain over nkb k-blocks (the last only its kq 4-steps): A by buffer loads at byte
// offset voff + b * stride, two k-blocks in flight; B block b from Ba (b < kbs) or Bb (b >= kbs)
__device__ __forceinline__ ff32x4 fp_gemm(__amdgpu_buffer_rsrc_t PA, int voff, int stride, int nkb, int kq,
                                          const float4* Ba, int kbs, const float4* Bb, int lane) {
    ff32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    float4 a0 = fas_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, 0, 0));
    float4 a1 = nkb > 1 ? fas_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, stride, 0)) : a0;
    float4 b0 = kbs > 0 ? Ba[lane] : Bb[lane];
    for (int kb = 0; kb < nkb; ++kb) {
        const float4 ak = a0, bk = b0;
        a0 = a1;
        if (kb + 2 < nkb) a1 = fas_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb + 2) * stride, 0));
        if (kb + 1 < nkb) b0 = kb + 1 < kbs ? Ba[(kb + 1) * 64 + lane] : Bb[(kb + 1 - kbs) * 64 + lane];
        const int steps = kb + 1 < nkb ? 4 : kq;
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.x, bk.x, acc, 0, 0, 0);
        if (steps > 1) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.y, bk.y, acc, 0, 0, 0);
        if (steps > 2) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.z, bk.z, acc, 0, 0, 0);
        if (steps > 3) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.w, bk.w, acc, 0, 0, 0);
        asm volatile("" : "+v"(acc)::"memory");
    }
    return acc;
}

// a phase-2 unit: the coupling tile t (u < KBe) or tile t of cell c's constraint rows
struct FpUnit2 {
    int cell, t;
};
__device__ __forceinline__ FpUnit2 fp_unit2(const FlatGeom& g, int u) {
    FpUnit2 x;
    if (u < g.KBe) {
        x.cell = -1;
        x.t = u;
    } else {
        x.cell = (u - g.KBe) / g.KBc;
        x.t = (u - g.KBe) - x.cell * g.KBc;
    }
    return x;
}
// constraint row of output row rr of a phase-2 unit (-1: padding)
__device__ __forceinline__ int fp_row2(const FlatGeom& g, FpUnit2 x, int rr) {
    if (x.cell < 0) return rr < g.E ? g.mc + rr : -1;
    return rr < 4 * g.Nh ? x.cell + g.n_u * rr : -1;
}

// A fragment prefetch of a unit's first two k-blocks (issued before the barrier that precedes
// its chain: the L2 latency overlaps the barrier and the epilogue)
struct FpPre {
    float4 a0, a1;
};
// A operand source: the fragment image in global memory (L2-resident, buffer loads) or a copy
// of it in LDS (ALDS: when it fits beside the panels' vectors)
template <bool ALDS>
__device__ __forceinline__ float4 fp_lda(__amdgpu_buffer_rsrc_t PA, const float4* As, int voff, int off) {
    if constexpr (ALDS) return As[(voff + off) >> 4];
    else return fas_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, off, 0));
}
// A block kb of a chain sits at byte offset voff + kb * stride (+ ajump from block akbs on: the
// 8b chains continue in the shared coupling image)
__device__ __forceinline__ int fp_aoff(int kb, int stride, int akbs, int ajump) {
    return kb * stride + (kb >= akbs ? ajump : 0);
}
template <bool ALDS>
__device__ __forceinline__ FpPre fp_pre(__amdgpu_buffer_rsrc_t PA, const float4* As, int voff, int stride, int nkb,
                                        int akbs = 1 << 30, int ajump = 0) {
    FpPre f;
    f.a0 = fp_lda<ALDS>(PA, As, voff, fp_aoff(0, stride, akbs, ajump));
    f.a1 = fp_lda<ALDS>(PA, As, voff, fp_aoff(nkb > 1 ? 1 : 0, stride, akbs, ajump));
    return f;
}
// one unit's chain over nkb k-blocks (the last only its kq 4-steps): A two blocks ahead (the
// first two prefetched by fp_pre), B one block ahead, block b of B from Ba (b < kbs) or Bb.
// Unrolled by two with fixed register roles and every load unconditional (indices clamped to
// the last block): the waitcnt for a block's operands then counts only the loads issued after
// them, instead of draining the queue at every conditional load or register rotation.
template <bool ALDS>
__device__ __forceinline__ ff32x4 fp_chain(__amdgpu_buffer_rsrc_t PA, const float4* As, FpPre f, int voff, int stride,
                                           int nkb, int kq, const float4* Ba, int kbs, const float4* Bb, int lane,
                                           int akbs = 1 << 30, int ajump = 0) {
    ff32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    const int last = nkb - 1;
    auto ldb = [&](int kb) -> float4 { return kb < kbs ? Ba[kb * 64 + lane] : Bb[(kb - kbs) * 64 + lane]; };
    float4 a0 = f.a0, a1 = f.a1;
    float4 b0 = ldb(0), b1;
    auto full = [&](const float4& ak, const float4& bk) {
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.x, bk.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.y, bk.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.z, bk.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.w, bk.w, acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // pairs of full blocks (four MFMA steps each, no branch in between), then the rest: the last
    // block alone (its kq steps), or one full block and the last
    int kb = 0;
    for (; kb + 2 <= last; kb += 2) {
        b1 = ldb(kb + 1);
        full(a0, b0);
        a0 = fp_lda<ALDS>(PA, As, voff, fp_aoff(kb + 2, stride, akbs, ajump));
        b0 = ldb(kb + 2);
        full(a1, b1);
        a1 = fp_lda<ALDS>(PA, As, voff, fp_aoff(kb + 3 < last ? kb + 3 : last, stride, akbs, ajump));
    }
    if (kb < last) {
        b1 = ldb(last);
        full(a0, b0);
        a0 = a1;
        b0 = b1;
    }
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc, 0, 0, 0);
    if (kq > 1) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc, 0, 0, 0);
    if (kq > 2) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc, 0, 0, 0);
    if (kq > 3) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc, 0, 0, 0);
    asm volatile("" : "+v"(acc)::"memory");
    return acc;
}

// unit geometry (uniform), from the launcher's descriptor tables.  The unit index goes through an
// empty asm so that nothing derived from it is hoisted out of the iteration loop (the derived
// offsets are a few scalar ops; holding them across the loop would spill).
__device__ __forceinline__ int fp_opq(int x) {
    asm volatile("" : "+s"(x));
    return x;
}
struct FpU1 {
    int pp, j, t;
};
__device__ __forceinline__ FpU1 fp_u1(const FlatGeom& g, int un) {
    const int d = g.d1[fp_opq(un)];
    FpU1 x;
    x.pp = d >> 16;
    x.j = ((d >> 8) & 0xFF) - 1;
    x.t = d & 0xFF;
    return x;
}
struct FpU2 {
    int pp, cell, t;
};
__device__ __forceinline__ FpU2 fp_u2(const FlatGeom& g, int un) {
    const int d = g.d2[fp_opq(un)];
    FpU2 x;
    x.pp = d >> 16;
    x.cell = ((d >> 8) & 0xFF) - 1;
    x.t = d & 0xFF;
    return x;
}
__device__ __forceinline__ int fp_voff1(const FlatGeom& g, FpU1 x, int lane) {
    return (x.j * g.KBc * g.T1 + x.t) * 1024 + lane * 16;
}
__device__ __forceinline__ int fp_ajump1(const FlatGeom& g, FpU1 x) {  // cell image -> coupling image
    return g.off1c * 16 - (x.j + 1) * g.KBc * g.T1 * 1024;
}
__device__ __forceinline__ int fp_voff2(const FlatGeom& g, FpU2 x, int lane) {
    return (x.cell < 0 ? g.off3 + x.t * 64 : g.off2 + (x.cell * g.T1 * g.KBc + x.t) * 64) * 16 + lane * 16;
}

template <int NU1, int NU2, bool ALDS, int W>
__global__ __launch_bounds__(64 * W, 4) void gpad_flatpanel_kernel(SolveArgs<float> a, FlatGeom g) {
    extern __shared__ __attribute__((aligned(16))) float4 fp_lds[];
    const int P = g.P;
    // per panel pp at fp_lds + pp * PB * 64:  Wc [n_u][KBc] | We [KBe] | Zc [n_u][T1] | Zn [KB3]
    const int oWe = g.n_u * g.KBc * 64, oZc = oWe + g.KBe * 64, oZn = oZc + g.n_u * g.T1 * 64;
    const int PBf = g.PB * 64;
    FlatPanelSlot* slots = reinterpret_cast<FlatPanelSlot*>(fp_lds + P * PBf);  // [P * U2]
    float4* As = fp_lds + P * PBf + (P * g.U2 * (int)sizeof(FlatPanelSlot)) / 16;  // ALDS: the A image

    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int jl = lane >> 4, c = lane & 15;
    const int n = a.n, m = a.m, N = a.N, K = a.check_every;
    const __amdgpu_buffer_rsrc_t PA =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.frag), 0, g.total * 16, 0x00020000);
    const bool use_tol = a.tol > 0.0;
    // phased compaction (as gpad_panel.hip): a phase runs iterations [v_begin, v_end) over the
    // instances idx_in[0 .. *count_in) (null: all), parks the survivors and lists them
    const bool fresh = a.v_begin == 0;
    const bool carry = a.v_end < N;
    const int count = a.count_in ? __builtin_amdgcn_readfirstlane(*a.count_in) : a.batch;
    const int groups = (count + 16 * P - 1) / (16 * P);
    const int nu1 = P * g.U1, nu2 = P * g.U2;
    if constexpr (ALDS) {
        const float4* src = reinterpret_cast<const float4*>(a.frag);
        for (int e = threadIdx.x; e < g.total; e += 64 * W) As[e] = src[e];
    }
    // Zn's rows past n are read by the last k-block of the coupling chains: zero once
    for (int pp = 0; pp < P; ++pp)
        for (int e = threadIdx.x; e < g.KB3 * 64; e += 64 * W)
            fp_lds[pp * PBf + oZn + e] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);

    for (int grp = blockIdx.x; grp < groups; grp += gridDim.x) {
        const int k0 = 16 * P * grp;  // first column of the group; column (pp, c) = k0 + 16 pp + c
        // the instance of column `bit` (= 16 pp + c) of this group
        auto inst_of = [&](int bit) -> size_t {
            const int k = k0 + bit;
            return (size_t)(a.idx_in ? a.idx_in[k] : k);
        };
        unsigned long long live = 0ull;
        for (int pp = 0; pp < P; ++pp) {
            const int left = count - k0 - 16 * pp;
            const unsigned msk = left >= 16 ? 0xFFFFu : (left > 0 ? ((1u << left) - 1u) : 0u);
            live |= (unsigned long long)msk << (16 * pp);
        }
        // ---- this wave's rows: z, g_P (phase 1), y, p_D (phase 2); w (and z_{-1}) into LDS --------
        float z[NU1][4], gp[NU1][4];
        float y[NU2][4], u[NU2][4], pd[NU2][4];
#pragma unroll
        for (int q = 0; q < NU1; ++q) {
            const int un = w + W * q;
            const FpU1 x = fp_u1(g, un < nu1 ? un : 0);
            const int col = k0 + 16 * x.pp + c;
            const bool act = un < nu1 && col < count;
            const size_t bi = act ? inst_of(16 * x.pp + c) : 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * x.t + 4 * r + jl;
                const bool ok = act && i < g.Nh;
                z[q][r] = ok ? a.z[bi * n + i * g.n_u + x.j] : 0.0f;
                gp[q][r] = ok ? a.gP[bi * a.ld_gP + i * g.n_u + x.j] : 0.0f;
            }
            if (un < nu1 && use_tol && fresh) {  // z_{-1} as the B operand of u = G_L z_{-1}
                float4* L = fp_lds + x.pp * PBf;
                L[oZc + (x.j * g.T1 + x.t) * 64 + lane] = make_float4(z[q][0], z[q][1], z[q][2], z[q][3]);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * x.t + 4 * r + jl, kk = i * g.n_u + x.j;
                    if (i < g.Nh)
                        reinterpret_cast<float*>(&L[oZn + (kk >> 4) * 64 + (kk & 3) * 16 + c])[(kk >> 2) & 3] = z[q][r];
                }
            }
        }
#pragma unroll
        for (int q = 0; q < NU2; ++q) {
            const int un = w + W * q;
            const FpU2 x = fp_u2(g, un < nu2 ? un : 0);
            const int col = k0 + 16 * x.pp + c;
            const bool act = un < nu2 && col < count;
            const size_t bi = act ? inst_of(16 * x.pp + c) : 0;
            float wv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = fp_row2(g, FpUnit2{x.cell, x.t}, 16 * x.t + 4 * r + jl);
                const bool ok = row >= 0 && act;
                y[q][r] = ok ? a.y[bi * m + row] : 0.0f;
                pd[q][r] = ok ? (float)(a.gscale * (double)a.g[bi * a.ld_g + row]) : 0.0f;
                if (fresh) {  // w_0 = y_0 + beta_0 (y_0 - y_{-1}), y_{-1} = y_0; u below
                    u[q][r] = 0.0f;
                    wv[r] = __builtin_fmaf(a.beta[0], y[q][r] - y[q][r], y[q][r]);
                } else {  // carried from the previous phase
                    u[q][r] = ok && use_tol ? a.uc[bi * m + row] : 0.0f;
                    wv[r] = ok ? a.wc[bi * m + row] : 0.0f;
                }
            }
            if (un < nu2) {
                float4* L = fp_lds + x.pp * PBf;
                L[(x.cell < 0 ? oWe + x.t * 64 : (x.cell * g.KBc + x.t) * 64) + lane] =
                    make_float4(wv[0], wv[1], wv[2], wv[3]);
            }
        }
        __syncthreads();
        if (use_tol && fresh) {  // u = G_L z_{-1}
#pragma unroll
            for (int q = 0; q < NU2; ++q) {
                const int un = w + W * q;
                if (un < nu2) {
                    const FpU2 x = fp_u2(g, un);
                    const bool cp = x.cell < 0;
                    const float4* L = fp_lds + x.pp * PBf;
                    const int voff = fp_voff2(g, x, lane), stride = (cp ? g.KBe : g.KBc) * 1024;
                    const int nkb = cp ? g.KB3 : g.T1;
                    const ff32x4 cz = fp_chain<ALDS>(PA, As, fp_pre<ALDS>(PA, As, voff, stride, nkb), voff, stride, nkb,
                                               cp ? g.kq3 : g.kq2, cp ? L + oZn : L + oZc + x.cell * g.T1 * 64,
                                               nkb, L + oZn, lane);
#pragma unroll
                    for (int r = 0; r < 4; ++r) u[q][r] = cz[r];
                }
            }
            __syncthreads();  // the zhat arrays are rewritten by the first iteration
        }

        // first units' A fragments, one barrier ahead
        FpPre pre1{}, pre2{};
        if (w < nu1) {
            const FpU1 x = fp_u1(g, w);
            pre1 = fp_pre<ALDS>(PA, As, fp_voff1(g, x, lane), g.T1 * 1024, g.KB1, g.KBc, fp_ajump1(g, x));
        }
        int v = a.v_begin;
        float th = a.theta[v], bn = a.beta[v + 1];
        while (true) {
            const float th_next = a.theta[v + 1], bn_next = a.beta[v + 2];
            ++v;
            const bool chk = use_tol && (v % K) == 0;
            const float omt = 1.0f - th;
            // ---- 8b + 8c: per-cell chains over (cell w, coupling w) ---------------------------------
#pragma unroll
            for (int q = 0; q < NU1; ++q) {
                const int un = w + W * q;
                if (un < nu1) {
                    const FpU1 x = fp_u1(g, un);
                    const bool act = (live >> (16 * x.pp + c)) & 1ull;
                    float4* L = fp_lds + x.pp * PBf;
                    const int voff = fp_voff1(g, x, lane);
                    const int ajump = fp_ajump1(g, x);
                    const FpPre f = q == 0 ? pre1 : fp_pre<ALDS>(PA, As, voff, g.T1 * 1024, g.KB1, g.KBc, ajump);
                    const ff32x4 acc = fp_chain<ALDS>(PA, As, f, voff, g.T1 * 1024, g.KB1, g.kq1, L + x.j * g.KBc * 64, g.KBc,
                                                      L + oWe, lane, g.KBc, ajump);
                    float zh[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        zh[r] = acc[r] - gp[q][r];  // seq_functions.cpp:18
                        const float zn = __builtin_fmaf(omt, z[q][r], th * zh[r]);
                        if (act) z[q][r] = zn;
                    }
                    L[oZc + (x.j * g.T1 + x.t) * 64 + lane] = make_float4(zh[0], zh[1], zh[2], zh[3]);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = 16 * x.t + 4 * r + jl, kk = i * g.n_u + x.j;
                        if (i < g.Nh)
                            reinterpret_cast<float*>(&L[oZn + (kk >> 4) * 64 + (kk & 3) * 16 + c])[(kk >> 2) & 3] =
                                zh[r];
                    }
                }
            }
            if (w < nu2) {
                const FpU2 x = fp_u2(g, w);
                pre2 = fp_pre<ALDS>(PA, As, fp_voff2(g, x, lane), (x.cell < 0 ? g.KBe : g.KBc) * 1024,
                              x.cell < 0 ? g.KB3 : g.T1);
            }
            __syncthreads();
            // ---- 8d + next 8a: cell and coupling chains; w back to LDS; test partials per unit -------
#pragma unroll
            for (int q = 0; q < NU2; ++q) {
                const int un = w + W * q;
                if (un < nu2) {
                    const FpU2 x = fp_u2(g, un);
                    const bool act = (live >> (16 * x.pp + c)) & 1ull;
                    const bool cp = x.cell < 0;
                    float4* L = fp_lds + x.pp * PBf;
                    const int voff = fp_voff2(g, x, lane), stride = (cp ? g.KBe : g.KBc) * 1024;
                    const int nkb = cp ? g.KB3 : g.T1;
                    const FpPre f = q == 0 ? pre2 : fp_pre<ALDS>(PA, As, voff, stride, nkb);
                    const ff32x4 acc = fp_chain<ALDS>(PA, As, f, voff, stride, nkb, cp ? g.kq3 : g.kq2,
                                                cp ? L + oZn : L + oZc + x.cell * g.T1 * 64, nkb, L + oZn, lane);
                    float4* wp = L + (cp ? oWe + x.t * 64 : (x.cell * g.KBc + x.t) * 64) + lane;
                    const float4 w4 = *wp;
                    const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
                    const int lim = cp ? g.E : 4 * g.Nh;
                    float wn[4];
                    float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
                    double gap = 0.0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float cv = acc[r], wi = wv[r], pdi = pd[q][r];
                        const float sv = (cv + wi) + pdi;        // seq_functions.cpp:37
                        const float yp = sv < 0.0f ? 0.0f : sv;  // seq_functions.cpp:40-42
                        if (use_tol) {
                            const float un2 = __builtin_fmaf(omt, u[q][r], th * cv);
                            if (act) u[q][r] = un2;
                            if (chk && act && 16 * x.t + 4 * r + jl < lim) {
                                const float tt = cv + pdi;
                                violh = fmaxf(violh, tt);
                                magh = fmaxf(magh, __builtin_fabsf(cv) + __builtin_fabsf(pdi));
                                wmin = fminf(wmin, wi);
                                gap -= (double)wi * (double)tt;
                                violz = fmaxf(violz, u[q][r] + pdi);
                            }
                        }
                        wn[r] = __builtin_fmaf(bn, yp - y[q][r], yp);
                        if (act) y[q][r] = yp;
                    }
                    if (act) *wp = make_float4(wn[0], wn[1], wn[2], wn[3]);
                    if (chk) {  // this unit's partials per column -> its slot
#pragma unroll
                        for (int o = 16; o < 64; o <<= 1) {
                            violz = fmaxf(violz, __shfl_xor(violz, o, 64));
                            violh = fmaxf(violh, __shfl_xor(violh, o, 64));
                            magh = fmaxf(magh, __shfl_xor(magh, o, 64));
                            wmin = fminf(wmin, __shfl_xor(wmin, o, 64));
                            gap += __shfl_xor(gap, o, 64);
                        }
                        if (jl == 0) {
                            slots[un].violz[c] = violz;
                            slots[un].violh[c] = violh;
                            slots[un].magh[c] = magh;
                            slots[un].wmin[c] = wmin;
                            slots[un].gap[c] = gap;
                        }
                    }
                }
            }
            if (w < nu1) {
                const FpU1 x = fp_u1(g, w);
                pre1 = fp_pre<ALDS>(PA, As, fp_voff1(g, x, lane), g.T1 * 1024, g.KB1, g.KBc, fp_ajump1(g, x));
            }
            th = th_next;
            bn = bn_next;
            __syncthreads();
            if (!chk && v < a.v_end) continue;

            unsigned long long m1 = 0ull, m2 = 0ull;
            bool zh_out = true;  // this iteration's zhat still in Zc (no verification chains ran)
            if (chk) {  // lane = (panel lane >> 4, column lane & 15): reduce that panel's unit slots
                int st1 = 0;
                const int pp = lane >> 4;
                if (pp < P && ((live >> lane) & 1ull)) {
                    double vz = -INFINITY, vh = -INFINITY, wm = INFINITY, gq = 0.0, mh = 0.0;
                    for (int s2 = pp * g.U2; s2 < (pp + 1) * g.U2; ++s2) {
                        vz = fmax(vz, (double)slots[s2].violz[c]);
                        vh = fmax(vh, (double)slots[s2].violh[c]);
                        mh = fmax(mh, (double)slots[s2].magh[c]);
                        wm = fmin(wm, (double)slots[s2].wmin[c]);
                        gq += slots[s2].gap[c];
                    }
                    st1 = (vz * a.L <= a.tol ? 1 : 0) |
                          ((viol_ok(vh, mh, a.L, a.tol, ViolMargin<float>::value) && (wm >= 0.0) &&
                            (gq * a.L <= a.tol_gap)) ? 2 : 0);
                }
                const unsigned long long mA = __ballot(st1 & 1);
                m2 = __ballot(st1 & 2);
                if (mA) {  // (A) nominated for some column: the flat G_L z chains of the group
                    zh_out = false;
#pragma unroll
                    for (int q = 0; q < NU1; ++q) {
                        const int un = w + W * q;
                        if (un < nu1) {
                            const FpU1 x = fp_u1(g, un);
                            const int bit = 16 * x.pp + c;
                            float4* L = fp_lds + x.pp * PBf;
                            float4* zc = &L[oZc + (x.j * g.T1 + x.t) * 64 + lane];
                            if ((m2 >> bit) & 1ull) {  // test (B)'s zhat out before z replaces it
                                const float4 zh4 = *zc;
                                const float zhv[4] = {zh4.x, zh4.y, zh4.z, zh4.w};
                                const size_t bi = inst_of(bit);
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    const int i = 16 * x.t + 4 * r + jl;
                                    if (i < g.Nh) a.z[bi * n + i * g.n_u + x.j] = zhv[r];
                                }
                            }
                            *zc = make_float4(z[q][0], z[q][1], z[q][2], z[q][3]);
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int i = 16 * x.t + 4 * r + jl, kk = i * g.n_u + x.j;
                                if (i < g.Nh)
                                    reinterpret_cast<float*>(&L[oZn + (kk >> 4) * 64 + (kk & 3) * 16 + c])[(kk >> 2) & 3] =
                                        z[q][r];
                            }
                        }
                    }
                    __syncthreads();
#pragma unroll
                    for (int q = 0; q < NU2; ++q) {
                        const int un = w + W * q;
                        if (un < nu2) {
                            const FpU2 x = fp_u2(g, un);
                            const bool nom = (mA >> (16 * x.pp + c)) & 1ull;
                            const bool cp = x.cell < 0;
                            const float4* L = fp_lds + x.pp * PBf;
                            const int voff = fp_voff2(g, x, lane), stride = (cp ? g.KBe : g.KBc) * 1024;
                            const int nkb = cp ? g.KB3 : g.T1;
                            const ff32x4 cz = fp_chain<ALDS>(PA, As, fp_pre<ALDS>(PA, As, voff, stride, nkb), voff,
                                                             stride, nkb, cp ? g.kq3 : g.kq2,
                                                             cp ? L + oZn : L + oZc + x.cell * g.T1 * 64, nkb,
                                                             L + oZn, lane);
                            const int lim = cp ? g.E : 4 * g.Nh;
                            float vc = -INFINITY, mc = 0.0f;
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                if (nom) u[q][r] = cz[r];  // the recursion restarts from the direct value
                                if (nom && 16 * x.t + 4 * r + jl < lim) {
                                    vc = fmaxf(vc, cz[r] + pd[q][r]);
                                    mc = fmaxf(mc, __builtin_fabsf(cz[r]) + __builtin_fabsf(pd[q][r]));
                                }
                            }
#pragma unroll
                            for (int o = 16; o < 64; o <<= 1) {
                                vc = fmaxf(vc, __shfl_xor(vc, o, 64));
                                mc = fmaxf(mc, __shfl_xor(mc, o, 64));
                            }
                            if (jl == 0) {  // every wave's stage-1 reads precede the barrier above
                                slots[un].violz[c] = vc;
                                slots[un].magh[c] = mc;
                            }
                        }
                    }
                    __syncthreads();
                    bool ver = false;
                    if (pp < P && ((mA >> lane) & 1ull)) {
                        double vcc = -INFINITY, mcc = 0.0;
                        for (int s2 = pp * g.U2; s2 < (pp + 1) * g.U2; ++s2) {
                            vcc = fmax(vcc, (double)slots[s2].violz[c]);
                            mcc = fmax(mcc, (double)slots[s2].magh[c]);
                        }
                        ver = viol_ok(vcc, mcc, a.L, a.tol, ViolMargin<float>::value);
                    }
                    m1 = __ballot(ver);
                    m2 &= ~m1;
                }
            }
            const unsigned long long fin = v >= N ? live : (live & (m1 | m2));
            if (fin) {  // finished columns: results out
#pragma unroll
                for (int q = 0; q < NU1; ++q) {
                    const int un = w + W * q;
                    if (un < nu1) {
                        const FpU1 x = fp_u1(g, un);
                        const int bit = 16 * x.pp + c;
                        const bool tb = (m2 >> bit) & 1ull;  // test (B): zhat (pre-written when verified over)
                        if (((fin >> bit) & 1ull) && (!tb || zh_out)) {
                            const size_t bi = inst_of(bit);
                            const float4 zh4 = fp_lds[x.pp * PBf + oZc + (x.j * g.T1 + x.t) * 64 + lane];
                            const float zhv[4] = {zh4.x, zh4.y, zh4.z, zh4.w};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int i = 16 * x.t + 4 * r + jl;
                                if (i < g.Nh) a.z[bi * n + i * g.n_u + x.j] = tb ? zhv[r] : z[q][r];
                            }
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < NU2; ++q) {
                    const int un = w + W * q;
                    if (un < nu2) {
                        const FpU2 x = fp_u2(g, un);
                        const int bit = 16 * x.pp + c;
                        if ((fin >> bit) & 1ull) {
                            const size_t bi = inst_of(bit);
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const int row = fp_row2(g, FpUnit2{x.cell, x.t}, 16 * x.t + 4 * r + jl);
                                if (row >= 0) a.y[bi * m + row] = y[q][r];
                            }
                        }
                    }
                }
                if (w == 0 && ((fin >> lane) & 1ull)) {
                    const size_t bi = inst_of(lane);
                    a.iters[bi] = v;
                    a.conv[bi] = (m1 >> lane) & 1ull ? 1 : ((m2 >> lane) & 1ull ? 2 : 0);
                }
            }
            live &= ~fin;
            if (live == 0ull || v >= a.v_end) break;
        }
        // ---- phase end: park the survivors (z, y in place; w, u carried) and list them ------------
        if (carry && live) {
#pragma unroll
            for (int q = 0; q < NU1; ++q) {
                const int un = w + W * q;
                if (un < nu1) {
                    const FpU1 x = fp_u1(g, un);
                    const int bit = 16 * x.pp + c;
                    if ((live >> bit) & 1ull) {
                        const size_t bi = inst_of(bit);
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i = 16 * x.t + 4 * r + jl;
                            if (i < g.Nh) a.z[bi * n + i * g.n_u + x.j] = z[q][r];
                        }
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < NU2; ++q) {
                const int un = w + W * q;
                if (un < nu2) {
                    const FpU2 x = fp_u2(g, un);
                    const int bit = 16 * x.pp + c;
                    if ((live >> bit) & 1ull) {
                        const size_t bi = inst_of(bit);
                        const float4 w4 = fp_lds[x.pp * PBf + (x.cell < 0 ? oWe + x.t * 64 : (x.cell * g.KBc + x.t) * 64) +
                                                 lane];  // w of iteration v (this unit's own rows)
                        const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = fp_row2(g, FpUnit2{x.cell, x.t}, 16 * x.t + 4 * r + jl);
                            if (row >= 0) {
                                a.y[bi * m + row] = y[q][r];
                                a.wc[bi * m + row] = wv[r];
                                if (use_tol) a.uc[bi * m + row] = u[q][r];
                            }
                        }
                    }
                }
            }
            if (w == 0) {  // lanes 0 .. 16 P - 1 speak for the group's columns
                const bool mine = (live >> lane) & 1ull;
                int base = 0;
                if (lane == 0) base = atomicAdd(a.count_out, (int)__popcll(live));
                base = __shfl(base, 0, 64);
                if (mine) a.idx_out[base + (int)__popcll(live & ((1ull << lane) - 1ull))] = (int)inst_of(lane);
            }
        }
        __syncthreads();  // the next group reuses the LDS arrays
    }
}

template <int NU1, int NU2, bool ALDS, int W>
static hipError_t launch_fp_k(const SolveArgs<float>& a, const FlatGeom& g, size_t lds, int grid, hipStream_t s) {
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)gpad_flatpanel_kernel<NU1, NU2, ALDS, W>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((gpad_flatpanel_kernel<NU1, NU2, ALDS, W>), dim3(grid), dim3(64 * W), lds, s, a, g);
    return hipGetLastError();
}
template <int NU1, int NU2, int W = kFlatPanelWaves>
static hipError_t launch_fp_nt(const SolveArgs<float>& a, const FlatGeom& g, size_t lds, bool alds, int grid,
                               hipStream_t s) {
    return alds ? launch_fp_k<NU1, NU2, true, W>(a, g, lds, grid, s)
                : launch_fp_k<NU1, NU2, false, W>(a, g, lds, grid, s);
}

static int fp_nt(int units, int W = kFlatPanelWaves) {
    const int q = (units + W - 1) / W;
    return q <= 1 ? 1 : (q <= 2 ? 2 : 4);
}

// 8-wave workgroups, two per CU: the same waves per CU as one 16-wave workgroup, but two
// independent barrier domains, so one workgroup's barrier waits overlap the other's chains.
// Only for shapes whose units fit (phase 1 one per wave, phase 2 at most four per wave) with
// the LDS of two workgroups; chosen with GPAD_FLAT_WAVES=8 or by the default rule below.
static hipError_t launch_flatpanel_w8(const SolveArgs<float>& a, FlatGeom g, int panels, hipStream_t s,
                                      bool force, bool* taken) {
    *taken = false;
    int P = 0;
    for (int q = 2; q >= 1 && !P; --q)
        if (q * g.U1 <= 8 && q * g.U2 <= 32 && 2 * flatpanel_lds_bytes(g, q) <= 160 * 1024 &&
            (force ? q == 1 || (panels + q - 1) / q >= 2 * a.num_cus : q == 2 && (panels + q - 1) / q >= 2 * a.num_cus))
            P = q;
    if (!P) return hipSuccess;
    g.P = P;
    for (int un = 0; un < 4 * kFlatPanelWavesMax; ++un) {
        const int pp = un / g.U1, uu = un % g.U1;
        g.d1[un] = un < P * g.U1 ? (pp << 16) | ((uu / g.T1 + 1) << 8) | (uu % g.T1) : 0;
        const int qq = un / g.U2, vv = un % g.U2;
        const int cell = vv < g.KBe ? -1 : (vv - g.KBe) / g.KBc;
        const int t = vv < g.KBe ? vv : (vv - g.KBe) % g.KBc;
        g.d2[un] = un < P * g.U2 ? (qq << 16) | ((cell + 1) << 8) | t : 0;
    }
    size_t lds = flatpanel_lds_bytes(g, P);
    const size_t abytes = (size_t)g.total * 16;
    const bool alds = 2 * (lds + abytes) <= 160 * 1024 && (!a.tune || a.tune->flat_a_lds);
    if (alds) lds += abytes;
    const int groups = (panels + P - 1) / P;
    const int grid = std::min(groups, 2 * a.num_cus);
    *taken = true;
    switch (fp_nt(P * g.U2, 8)) {
        case 1: return launch_fp_nt<1, 1, 8>(a, g, lds, alds, grid, s);
        case 2: return launch_fp_nt<1, 2, 8>(a, g, lds, alds, grid, s);
        default: return launch_fp_nt<1, 4, 8>(a, g, lds, alds, grid, s);
    }
}

// one launch over a.batch instances, or over the phase's list (a.count_in; the geometry and grid
// are sized for a.batch, extra workgroups find no group); a.frag = the flat fragment images.
// P panels per workgroup: as many as keep every CU busy (groups >= CUs), the phase-1 units within
// one per wave and the phase-2 units within 4 per wave, and the LDS within 160 KiB.
static hipError_t launch_flatpanel_once(const SolveArgs<float>& a, hipStream_t s) {
    if (!flatpanel_supported(a.n, a.m, a.n_u) || !a.frag) return hipErrorInvalidValue;
    FlatGeom g = flat_geom(a.n, a.m, a.n_u);
    const int panels = (a.batch + 15) / 16;
    const Tuning tn = a.tune ? *a.tune : Tuning{};
    if (tn.flat_waves == 8) {  // forced 8-wave workgroups
        bool taken = false;
        const hipError_t e = launch_flatpanel_w8(a, g, panels, s, true, &taken);
        if (taken || e != hipSuccess) return e;
    } else if (tn.flat_waves == 0) {
        // default: two 8-wave workgroups per CU when each can hold two panels (C1 packs from 16384:
        // 5.41 -> 5.23 us per batch-iteration); at one panel each they lose to one 16-wave
        // workgroup of two panels (8192: 3.03 vs 3.28 us)
        bool taken = false;
        const hipError_t e = launch_flatpanel_w8(a, g, panels, s, false, &taken);
        if (taken || e != hipSuccess) return e;
    }
    int P = 1;
    for (int q = 4; q > 1; --q) {
        if (q * g.U1 <= kFlatPanelWaves && q * g.U2 <= 4 * kFlatPanelWaves &&
            flatpanel_lds_bytes(g, q) <= 160 * 1024 && (panels + q - 1) / q >= a.num_cus) {
            P = q;
            break;
        }
    }
    if (tn.flat_panels > 0) P = std::min(4, tn.flat_panels);
    while (P > 1 && (P * g.U1 > 4 * kFlatPanelWaves || P * g.U2 > 4 * kFlatPanelWaves ||
                     flatpanel_lds_bytes(g, P) > 160 * 1024))
        --P;
    g.P = P;
    for (int un = 0; un < 4 * kFlatPanelWavesMax; ++un) {
        const int pp = un / g.U1, uu = un % g.U1;
        g.d1[un] = un < P * g.U1 ? (pp << 16) | ((uu / g.T1 + 1) << 8) | (uu % g.T1) : 0;
        const int qq = un / g.U2, vv = un % g.U2;
        const int cell = vv < g.KBe ? -1 : (vv - g.KBe) / g.KBc;
        const int t = vv < g.KBe ? vv : (vv - g.KBe) % g.KBc;
        g.d2[un] = un < P * g.U2 ? (qq << 16) | ((cell + 1) << 8) | t : 0;
    }
    size_t lds = flatpanel_lds_bytes(g, P);
    const size_t abytes = (size_t)g.total * 16;
    const bool alds = lds + abytes <= 160 * 1024 && tn.flat_a_lds;  // A image in LDS
    if (alds) lds += abytes;
    const int groups = (panels + P - 1) / P;
    int grid = a.num_cus * (lds * 2 <= 160 * 1024 ? 2 : 1);
    if (grid > groups) grid = groups;
    const int q1 = fp_nt(P * g.U1), q2 = fp_nt(P * g.U2);
#define FP_CASE(A, B) \
    case A * 8 + B: return launch_fp_nt<A, B>(a, g, lds, alds, grid, s);
    switch (q1 * 8 + q2) {
        FP_CASE(1, 1) FP_CASE(1, 2) FP_CASE(1, 4)
        FP_CASE(2, 1) FP_CASE(2, 2) FP_CASE(2, 4)
        FP_CASE(4, 1) FP_CASE(4, 2)
        default: return launch_fp_nt<4, 4>(a, g, lds, alds, grid, s);
    }
#undef FP_CASE
}

// Phase schedule of a phased flat solve: 2K iterations, then a quarter of the iterations done so
// far (rounded to the test period K), so phases stay short while most columns are alive and grow
// geometrically in a long tail (O(log N) launches); past the previous solve's last iteration
// (v_pred) one phase runs to N, so an unused tail costs no empty launches.  Estimated on battery
// tol-mode batches of 8192: column utilisation ~0.9-0.96 vs 0.61-0.70 in one launch.
int flat_phase_len(int v0, int check_every, const Tuning* t) {
    const int K = check_every > 0 ? check_every : 10;
    const int base = (t && t->phase_len > 0) ? t->phase_len : 2 * K;
    const int grow = (v0 / 4) / K * K;
    return grow > base ? grow : base;
}

hipError_t launch_flatpanel(const SolveArgs<float>& a0, hipStream_t s) {
    if (!flatpanel_supported(a0.n, a0.m, a0.n_u) || !a0.frag) return hipErrorInvalidValue;
    SolveArgs<float> a = a0;
    const Tuning tn = a.tune ? *a.tune : Tuning{};
    a.v_begin = 0;
    a.v_end = a.N;
    a.idx_in = nullptr;
    a.count_in = nullptr;
    // phases pay when the batch is several resident rounds of groups (the time of a resident round
    // is its slowest column either way; compaction shortens the queue of rounds): measured on
    // battery packs, eps mode, phased vs one launch -- C1 8192: 1.91 vs 1.63 ms, 65536: 8.8 vs
    // 10.0 ms; N = 50 4096: 25.1 vs 23.9 ms, 16384: 67.7 vs 87.2 ms (profiles/r02_flat_phased.txt).
    // GPAD_OPT_PHASED: 0 never, 1 (default) from 4 panels per CU, 2 always.
    const int panels = (a.batch + 15) / 16;
    const bool phased = a.tol > 0.0 && a.pwork != nullptr &&
                        (tn.phased == 2 || (tn.phased == 1 && panels >= 4 * a.num_cus));
    if (!phased) return launch_flatpanel_once(a, s);
    // workspace as the panel path's (panel_work_bytes): idx ping-pong, phase counts, carried w, u
    int* idx0 = reinterpret_cast<int*>(a.pwork);
    int* idx1 = idx0 + a.batch;
    int* counts = idx1 + a.batch;
    float* wc = reinterpret_cast<float*>(counts + 2 * kPanelMaxPhases);
    a.wc = wc;
    a.uc = wc + (size_t)a.batch * a.m;
    hipError_t e = hipMemsetAsync(counts, 0, sizeof(int) * kPanelMaxPhases, s);
    if (e != hipSuccess) return e;
    int v0 = 0;
    for (int ph = 0; v0 < a.N; ++ph) {
        int plen = ph >= kPanelMaxPhases - 1 ? a.N : flat_phase_len(v0, a.check_every, &tn);
        if (a0.v_pred > 0 && v0 >= a0.v_pred) plen = a.N;  // beyond the prediction: one last phase
        const int v1 = (a.N - v0 <= plen) ? a.N : v0 + plen;
        a.v_begin = v0;
        a.v_end = v1;
        a.idx_in = ph ? ((ph & 1) ? idx0 : idx1) : nullptr;
        a.count_in = ph ? counts + ph - 1 : nullptr;
        a.idx_out = (ph & 1) ? idx1 : idx0;
        a.count_out = counts + ph;
        if ((e = launch_flatpanel_once(a, s)) != hipSuccess) return e;
        v0 = v1;
    }
    return hipSuccess;
}

}  // namespace gpad
