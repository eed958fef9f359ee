// gpad_pair32.hip -- the C3/C4 shape (n = m = 200) panel pairs on v_mfma_f32_32x32x2_f32 ("W32").
//
// gpad_panel2_kernel runs a pair of 16-instance panels as 26 chains of v_mfma_f32_16x16x4_f32 per
// GEMM (13 row tiles x 2 panels, tile 12 half padding) on 16 waves.  A 16x16x4 chain has a 40-cycle
// dependent latency against a 32-cycle issue, so a chain that runs alone -- the youngest waves of
// each SIMD at the end of a GEMM under oldest-first MFMA arbitration -- issues at 80 %, and its
// A fragments, one block ahead, wait on L2 then; measured MFMA busy 0.82.
//
// Here the 32 instances of the pair are the 32 columns of one 32x32x2 chain (64-cycle issue AND
// 64-cycle dependent latency: a lone chain issues at full rate; exact f32, bitwise the ascending-k
// fmaf chain -- tools/lat/w32.hip).  Rows 0..191 are six 32-row tiles, rows 192..199 one
// v_mfma_f32_16x16x4_f32 chain per panel (8 real rows of 16).  Per GEMM that is 6 x 100 x 64 +
// 2 x 50 x 32 cycles = 41600 = 6.5 chain units of 1600 per SIMD, dealt to 8 waves (2 per SIMD,
// SIMD = wave & 3) with one cross-SIMD chain hand-off per SIMD pair:
//   waves 4..7 ("full"): tile w - 4 (tiles 0..3), whole chains;
//   waves 0, 1 ("head"): MFMAs [0, S) of tile 4 + w, parked in LDS for wave w + 2, then the
//                         remainder chain of panel w (rows 192..199);
//   waves 2, 3 ("tail"): tile 4 + (w - 2) from MFMA S on (the hand-off), its epilogue and state.
// S = 36 MFMAs: SIMDs 0, 1 carry 36 x 64 + 1600 + 6400 = 10304 cycles, SIMDs 2, 3 64 x 64 + 6400 =
// 10496.  The head / tail waves are the older wave of their SIMD, so the head piece runs first and
// the tail continues it as soon as it lands.  A chain cut between MFMAs and continued elsewhere from
// the parked accumulator is the same ascending-k sequence: bit-identical.
//
// Layouts.  32x32x2: lane l supplies A[i = l&31][k = 2s + (l>>5)] and B[k][l&31] to MFMA s and holds
// D[(r&3) + 8(r>>2) + 4(l>>5)][l&31] in accumulator register r (cdna_hip_programming.md).  Vectors
// (w, zhat; z for the verification GEMM) live in LDS in the B order of the NEXT GEMM:
//   V[kb][lane][q] = x[8 kb + 2q + (lane>>5)] of column lane&31,   kb < 25
// and the A images pack the rows of tile t so that accumulator register r of lane l is original row
// 32t + 8(r>>2) + 2(r&3) + (l>>5) -- exactly V[4t + (r>>2)][l][r&3] of the next GEMM:
//   PT[t][kb][lane][q] = M[32t + o(lane&31)][8 kb + 2q + (lane>>5)],  o(i) = 8(i>>3) + 2(i&3) + ((i>>2)&1)
// The remainder chain (16x16x4: lane l supplies A[l&15][k = 4s + (l>>4)], B[k][l&15], holds rows
// 4(l>>4) + r) packs row 192 + 2r + j at packed row 4j + r (j < 2; packed rows 8..15 zero):
//   PR[b][lane][q] = M[192 + 2((lane&15)&3) + ((lane&15)>>2)][16 b + 4q + (lane>>4)]   (zero for lane&15 >= 8)
// so its lanes j = 0, 1 hold rows 192 + 2r + j, i.e. V[24][j*32 + col][r]: one float4 store each; its
// B (k = 4s + j of column c of panel p) is element 2(s&1) + (j>>1) of V[s>>1][(j&1)*32 + 16p + c].
//
// Everything else -- phases (v_begin / v_end, compaction lists, carried w, u), Algorithm 1 with the
// (A) nomination verified on a direct G_L z GEMM, the certification-floor max |g| fold, the hand-off
// failure report -- follows gpad_panel2_kernel, with the same per-element arithmetic, so results are
// bit-identical to it (tests/test_pair32.py) and to the oracle.
#include <hip/hip_runtime.h>

#include <cmath>

#include "gpad_internal.h"

namespace gpad {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kN = 200;      // the shape (n = m = 200)
constexpr int kKB = 25;      // 8-k blocks of K = 200
constexpr int kTiles = 6;    // 32-row tiles (rows 0..191)
constexpr int kMf = 100;     // 32x32x2 MFMAs per full chain
constexpr int kSplit = 36;   // MFMAs of tiles 4, 5 on the head waves (multiple of 4)
constexpr int kRemB = 13;    // 16-k blocks of the remainder chain (the last: 2 steps)
constexpr size_t kPTBytes = (size_t)kTiles * kKB * 64 * 16;  // 153600
constexpr size_t kPRBytes = (size_t)kRemB * 64 * 16;         // 13312
constexpr size_t kImgBytes = kPTBytes + kPRBytes;             // one operand

__device__ __forceinline__ float4 as_f4(u32x4 v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}

__global__ void pack_pair32_kernel(const float* __restrict__ src, double scale, float4* __restrict__ dst) {
    // full tiles: idx < 6*25*64; remainder after
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int nfull = kTiles * kKB * 64;
    if (idx < nfull) {
        const int lane = idx & 63, kb = (idx >> 6) % kKB, t = (idx >> 6) / kKB;
        const int i = lane & 31, h = lane >> 5;
        const int row = 32 * t + 8 * (i >> 3) + 2 * (i & 3) + ((i >> 2) & 1);
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = (float)(scale * (double)src[(size_t)row * kN + 8 * kb + 2 * q + h]);
        dst[idx] = make_float4(v[0], v[1], v[2], v[3]);
    } else if (idx < nfull + kRemB * 64) {
        const int e = idx - nfull, lane = e & 63, b = e >> 6;
        const int rho = lane & 15;
        float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (rho < 8) {
            const int row = 192 + 2 * (rho & 3) + (rho >> 2);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = 16 * b + 4 * q + (lane >> 4);
                v[q] = k < kN ? (float)(scale * (double)src[(size_t)row * kN + k]) : 0.0f;
            }
        }
        dst[idx] = make_float4(v[0], v[1], v[2], v[3]);
    }
}

struct W32Slot {    // per row group and column: (violz, violh, magh, wmin) and the fp64 gap
    float4 f[32];
    double gap[32];
};

struct W32Lds {
    float4 Wl[kKB * 64];    // w (B of GEMM 1)
    float4 Zh[kKB * 64];    // zhat (B of GEMM 2); z during the (A) verification / the u seed
    float4 Gp[kKB * 64];    // g_P per row, same layout (the remainder's rows in block 24)
    float4 Pd[kKB * 64];    // p_D per row
    float4 hand[2][4][64];  // hand-off accumulators (tiles 4, 5)
    W32Slot slots[7];       // row groups: tiles 0..5, the remainder
    int hflag[2];
    int herr;
    int znz[8];
    float gred[8];
};

// A pass over one GEMM for this wave's role.  Full / tail: acc (16 registers) for its tile.  Head:
// the piece [0, S) of tile 4 + p parked for the tail, then the remainder chain of panel p into racc.
template <int S0, int S1>
__device__ __forceinline__ void chain32(const char* __restrict__ PT, const float4* __restrict__ Bl, int lane, int t,
                                        f32x16& acc) {
    // MFMAs [S0, S1) (multiples of 4) of tile t, A two blocks ahead, B one; unrolled so every wait
    // count is static
    const float4* A = reinterpret_cast<const float4*>(PT) + (size_t)t * kKB * 64 + lane;
    constexpr int b0 = S0 >> 2, b1 = S1 >> 2;
    float4 a0 = A[(size_t)b0 * 64], a1 = A[(size_t)(b0 + 1 < b1 ? b0 + 1 : b0) * 64], a2;
    float4 bb = Bl[b0 * 64 + lane], bn;
#pragma unroll
    for (int kb = b0; kb < b1; ++kb) {
        const int k2 = kb + 2 < b1 ? kb + 2 : b1 - 1;
        a2 = A[(size_t)k2 * 64];
        bn = Bl[(kb + 1 < b1 ? kb + 1 : kb) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, bb.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, bb.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, bb.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, bb.w, acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        a0 = a1;
        a1 = a2;
        bb = bn;
    }
}

// the remainder chain of panel p: 16x16x4 over K = 200 (12 blocks of 16 k + 2 steps)
__device__ __forceinline__ f32x4 chain_rem(const char* __restrict__ PR, const float4* __restrict__ Bl, int lane,
                                          int p) {
    const float4* A = reinterpret_cast<const float4*>(PR) + lane;
    const int j = lane >> 4, c = lane & 15, sel = j >> 1;
    const int bidx = (j & 1) * 32 + 16 * p + c;
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    float4 a0 = A[0], a1 = A[64];
    float4 x0 = Bl[bidx], x1 = Bl[64 + bidx];
#pragma unroll
    for (int b = 0; b < kRemB - 1; ++b) {
        const float4 an = A[(size_t)(b + 2 < kRemB ? b + 2 : kRemB - 1) * 64];
        const float4 y0 = Bl[(2 * b + 2) * 64 + bidx];
        const float4 y1 = Bl[(2 * b + 3 < kKB ? 2 * b + 3 : kKB - 1) * 64 + bidx];
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, sel ? x0.y : x0.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, sel ? x0.w : x0.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, sel ? x1.y : x1.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, sel ? x1.w : x1.z, acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        a0 = a1;
        a1 = an;
        x0 = y0;
        x1 = y1;
    }
    // block 12: k = 192..199, two steps, B from V block 24
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, sel ? x0.y : x0.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, sel ? x0.w : x0.z, acc, 0, 0, 0);
    return acc;
}

__device__ __forceinline__ f32x16 handoff_wait32(W32Lds& L, int slot, int gen, int lane) {
    for (int s = 0;; ++s) {
        if (__hip_atomic_load(&L.hflag[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == gen) break;
        if (s == (1 << 20)) {
            L.herr = 1;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    f32x16 h;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 v = L.hand[slot][q][lane];
        h[4 * q] = v.x;
        h[4 * q + 1] = v.y;
        h[4 * q + 2] = v.z;
        h[4 * q + 3] = v.w;
    }
    return h;
}

__device__ __forceinline__ void handoff_post32(W32Lds& L, int slot, int gen, int lane, const f32x16& h) {
#pragma unroll
    for (int q = 0; q < 4; ++q) L.hand[slot][q][lane] = make_float4(h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __hip_atomic_store(&L.hflag[slot], gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// one GEMM pass of the wave's role over B = Bl with the image at img (PT | PR).
// ROLE 0 full (tile t), 1 head (piece of tile 4 + p, then the remainder of panel p), 2 tail (tile 4 + p)
template <int ROLE>
__device__ __forceinline__ void w32_gemm(W32Lds& L, const char* img, const float4* Bl, int lane, int t, int p, int gen,
                                         f32x16& acc, f32x4& racc) {
    if constexpr (ROLE == 0) {
        acc = f32x16{};
        chain32<0, kMf>(img, Bl, lane, t, acc);
    } else if constexpr (ROLE == 1) {
        f32x16 h = {};
        chain32<0, kSplit>(img, Bl, lane, 4 + p, h);
        handoff_post32(L, p, gen, lane, h);
        racc = chain_rem(img + kPTBytes, Bl, lane, p);
    } else {
        acc = handoff_wait32(L, p, gen, lane);
        chain32<kSplit, kMf>(img, Bl, lane, 4 + p, acc);
    }
}

// the rows this lane holds: full / tail, register r -> row 32t + 8(r>>2) + 2(r&3) + h of column
// lane&31; head (remainder), lanes j < 2, register r -> row 192 + 2r + j of column 16p + c
__device__ __forceinline__ int row_of(int t, int r, int h) { return 32 * t + 8 * (r >> 2) + 2 * (r & 3) + h; }

template <int ROLE>
__device__ void w32_run(const SolveArgs<float>& a, W32Lds& L, int t, int p, int items, int count) {
    constexpr int NR = ROLE == 1 ? 4 : 16;  // rows held per lane
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, col = lane & 31;  // full / tail
    const int j = lane >> 4, c = lane & 15;    // head
    const bool rl = ROLE != 1 || j < 2;        // this lane holds real rows
    const int N = a.N, K = a.check_every;
    const char* IM1 = reinterpret_cast<const char*>(a.frag32);
    const char* IM2 = IM1 + kImgBytes;
    const bool use_tol = a.tol > 0.0;
    const bool fresh = a.v_begin == 0;
    const bool carry = a.v_end < N;
    const int mycol = ROLE == 1 ? 16 * p + c : col;  // this lane's column (0..31 of the item)
    const int tb = ROLE == 0 ? t : 4 + p;            // full / tail tile
    int gen = 0;
    float gmx = 0.0f;

    for (int it = blockIdx.x; it < items; it += gridDim.x) {
        // columns still running (bit = column), uniform
        unsigned live = 0u;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            const int left = count - 16 * (2 * it + pp);
            const int cnt = left < 0 ? 0 : (left > 16 ? 16 : left);
            live |= ((1u << cnt) - 1u) << (16 * pp);
        }
        const int kpos = 16 * (2 * it + (mycol >> 4)) + (mycol & 15);
        bool act = kpos < count && rl;
        const int inst = act ? (a.idx_in ? a.idx_in[kpos] : kpos) : 0;
        // ---- state of this lane's rows ----------------------------------------------------------
        float z[NR], y[NR], u[NR];
        {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int i = ROLE == 1 ? 192 + 2 * r + j : row_of(tb, r, h);
                const size_t b = (size_t)inst;
                z[r] = act ? a.z[b * kN + i] : 0.0f;
                y[r] = act ? a.y[b * kN + i] : 0.0f;
                const float gr = act ? a.g[b * a.ld_g + i] : 0.0f;
                gmx = absmax_nan(gmx, gr);
                u[r] = (!fresh && act && use_tol) ? a.uc[b * kN + i] : 0.0f;
            }
            float gp[NR], pd[NR], wv[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int i = ROLE == 1 ? 192 + 2 * r + j : row_of(tb, r, h);
                const size_t b = (size_t)inst;
                gp[r] = act ? a.gP[b * a.ld_gP + i] : 0.0f;
                pd[r] = (float)(a.gscale * (double)(act ? a.g[b * a.ld_g + i] : 0.0f));
                wv[r] = fresh ? __builtin_fmaf(a.beta[0], y[r] - y[r], y[r]) : (act ? a.wc[b * kN + i] : 0.0f);
            }
            if constexpr (ROLE == 1) {
                if (j < 2) {
                    const int o = 24 * 64 + j * 32 + 16 * p + c;
                    L.Gp[o] = make_float4(gp[0], gp[1], gp[2], gp[3]);
                    L.Pd[o] = make_float4(pd[0], pd[1], pd[2], pd[3]);
                    L.Wl[o] = make_float4(wv[0], wv[1], wv[2], wv[3]);
                    if (fresh && use_tol) L.Zh[o] = make_float4(z[0], z[1], z[2], z[3]);
                }
            } else {
#pragma unroll
                for (int b4 = 0; b4 < 4; ++b4) {
                    const int o = (4 * tb + b4) * 64 + lane;
                    L.Gp[o] = make_float4(gp[4 * b4], gp[4 * b4 + 1], gp[4 * b4 + 2], gp[4 * b4 + 3]);
                    L.Pd[o] = make_float4(pd[4 * b4], pd[4 * b4 + 1], pd[4 * b4 + 2], pd[4 * b4 + 3]);
                    L.Wl[o] = make_float4(wv[4 * b4], wv[4 * b4 + 1], wv[4 * b4 + 2], wv[4 * b4 + 3]);
                    if (fresh && use_tol) L.Zh[o] = make_float4(z[4 * b4], z[4 * b4 + 1], z[4 * b4 + 2], z[4 * b4 + 3]);
                }
            }
        }
        if (fresh && use_tol) {  // u = G_L z_{-1}: +0 exactly, and no GEMM, when every z_{-1} is zero
            bool nz = false;
#pragma unroll
            for (int r = 0; r < NR; ++r) nz = nz || z[r] != 0.0f;
            const bool wnz = __ballot(nz) != 0ull;
            if (lane == 0) L.znz[threadIdx.x >> 6] = wnz ? 1 : 0;
            __syncthreads();
            int anynz = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) anynz |= L.znz[i];
            if (anynz) {
                f32x16 acc;
                f32x4 racc;
                w32_gemm<ROLE>(L, IM2, L.Zh, lane, t, p, ++gen, acc, racc);
#pragma unroll
                for (int r = 0; r < NR; ++r) u[r] = ROLE == 1 ? racc[r] : acc[r];
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
            // ---- GEMM 1 + epilogue: zhat = -ML w - g_P (8b), z = (1-th) z + th zhat (8c) ----------
            {
                f32x16 acc;
                f32x4 racc;
                w32_gemm<ROLE>(L, IM1, L.Wl, lane, t, p, ++gen, acc, racc);
                if constexpr (ROLE == 1) {
                    if (j < 2) {
                        const int o = 24 * 64 + j * 32 + 16 * p + c;
                        const float4 g4 = L.Gp[o];
                        const float gp[4] = {g4.x, g4.y, g4.z, g4.w};
                        float zh[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            zh[r] = racc[r] - gp[r];
                            z[r] = __builtin_fmaf(omt, z[r], th * zh[r]);
                        }
                        L.Zh[o] = make_float4(zh[0], zh[1], zh[2], zh[3]);
                    }
                } else {
#pragma unroll
                    for (int b4 = 0; b4 < 4; ++b4) {
                        const int o = (4 * tb + b4) * 64 + lane;
                        const float4 g4 = L.Gp[o];
                        const float gp[4] = {g4.x, g4.y, g4.z, g4.w};
                        float zh[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int r = 4 * b4 + q;
                            zh[q] = acc[r] - gp[q];
                            z[r] = __builtin_fmaf(omt, z[r], th * zh[q]);
                        }
                        L.Zh[o] = make_float4(zh[0], zh[1], zh[2], zh[3]);
                    }
                }
            }
            __syncthreads();
            // ---- GEMM 2 + epilogue: y+ = [w + G_L zhat + p_D]+ (8d), next w (8a), test partials ----
            float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
            double gap = 0.0;
            {
                f32x16 acc;
                f32x4 racc;
                w32_gemm<ROLE>(L, IM2, L.Zh, lane, t, p, ++gen, acc, racc);
                constexpr int NB = ROLE == 1 ? 1 : 4;
#pragma unroll
                for (int b4 = 0; b4 < NB; ++b4) {
                    if (ROLE == 1 && j >= 2) break;
                    const int o = ROLE == 1 ? 24 * 64 + j * 32 + 16 * p + c : (4 * tb + b4) * 64 + lane;
                    const float4 w4 = L.Wl[o], p4 = L.Pd[o];
                    const float wv[4] = {w4.x, w4.y, w4.z, w4.w}, pd[4] = {p4.x, p4.y, p4.z, p4.w};
                    float wn[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int r = 4 * b4 + q;
                        const float cv = ROLE == 1 ? racc[q] : acc[r];
                        const float sv = (wv[q] + pd[q]) + cv;                  // seq_functions.cpp:84
                        const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;     // seq_functions.cpp:85
                        wn[q] = __builtin_fmaf(bn, yp - y[r], yp);
                        y[r] = yp;
                        if (use_tol) {
                            u[r] = __builtin_fmaf(omt, u[r], th * cv);
                            if (chk && act) {
                                const float tt = cv + pd[q];
                                violh = fmaxf(violh, tt);
                                magh = fmaxf(magh, __builtin_fabsf(cv) + __builtin_fabsf(pd[q]));
                                wmin = fminf(wmin, wv[q]);
                                gap -= (double)wv[q] * (double)tt;
                                violz = fmaxf(violz, u[r] + pd[q]);
                            }
                        }
                    }
                    L.Wl[o] = make_float4(wn[0], wn[1], wn[2], wn[3]);
                }
                if (chk) {  // per column: the lane pair (h = 0, 1) / (j = 0, 1), then the slot
                    const int o = ROLE == 1 ? 16 : 32;
                    violz = fmaxf(violz, __shfl_xor(violz, o, 64));
                    violh = fmaxf(violh, __shfl_xor(violh, o, 64));
                    magh = fmaxf(magh, __shfl_xor(magh, o, 64));
                    wmin = fminf(wmin, __shfl_xor(wmin, o, 64));
                    const double go = __shfl_xor(gap, o, 64);
                    gap = (ROLE == 1 ? j == 0 : h == 0) ? gap + go : go + gap;
                    if (ROLE == 1 ? j == 0 : h == 0) {
                        W32Slot& S = L.slots[ROLE == 1 ? 6 : tb];
                        S.f[mycol] = make_float4(violz, violh, magh, wmin);
                        S.gap[mycol] = gap;
                    }
                }
            }
            th = th_next;
            bn = bn_next;
            __syncthreads();
            if (!chk && v < a.v_end) continue;

            // ---- Algorithm 1, per column: lane l < 32 <-> column l; every wave reduces alike ----------
            unsigned m1 = 0u, m2 = 0u;
            bool zh_out = true;
            if (chk) {
                int st1 = 0;
                if (lane < 32 && ((live >> lane) & 1u)) {
                    float4 f = make_float4(-INFINITY, -INFINITY, 0.0f, INFINITY);
                    double gq = 0.0;
#pragma unroll
                    for (int g = 0; g < 7; ++g) {
                        const float4 e = L.slots[g].f[lane];
                        f.x = fmaxf(f.x, e.x);
                        f.y = fmaxf(f.y, e.y);
                        f.z = fmaxf(f.z, e.z);
                        f.w = fminf(f.w, e.w);
                        gq += L.slots[g].gap[lane];
                    }
                    st1 = ((double)f.x * a.L <= a.tol ? 1 : 0) |
                          ((viol_ok((double)f.y, (double)f.z, a.L, a.tol, ViolMargin<float>::value) && (f.w >= 0.0f) &&
                            (gq * a.L <= a.tol_gap)) ? 2 : 0);
                }
                const unsigned mA = (unsigned)__ballot(st1 & 1);
                m2 = (unsigned)__ballot(st1 & 2);
                if (mA) {  // (A) nominated for some column: G_L z of the whole item
                    zh_out = false;
                    const bool b2 = act && ((m2 >> mycol) & 1u);
                    if constexpr (ROLE == 1) {
                        if (j < 2) {
                            const int o = 24 * 64 + j * 32 + 16 * p + c;
                            if (b2) {  // test (B)'s zhat out before z replaces it
                                const float4 h4 = L.Zh[o];
                                const float zh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                                for (int r = 0; r < 4; ++r) a.z[(size_t)inst * kN + 192 + 2 * r + j] = zh[r];
                            }
                            L.Zh[o] = make_float4(z[0], z[1], z[2], z[3]);
                        }
                    } else {
#pragma unroll
                        for (int b4 = 0; b4 < 4; ++b4) {
                            const int o = (4 * tb + b4) * 64 + lane;
                            if (b2) {
                                const float4 h4 = L.Zh[o];
                                const float zh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                                for (int q = 0; q < 4; ++q) a.z[(size_t)inst * kN + row_of(tb, 4 * b4 + q, h)] = zh[q];
                            }
                            L.Zh[o] = make_float4(z[4 * b4], z[4 * b4 + 1], z[4 * b4 + 2], z[4 * b4 + 3]);
                        }
                    }
                    __syncthreads();
                    f32x16 acc;
                    f32x4 racc;
                    w32_gemm<ROLE>(L, IM2, L.Zh, lane, t, p, ++gen, acc, racc);
                    const bool nom = act && ((mA >> mycol) & 1u);
                    float vc = -INFINITY, mc = 0.0f;
                    constexpr int NB = ROLE == 1 ? 1 : 4;
#pragma unroll
                    for (int b4 = 0; b4 < NB; ++b4) {
                        if (ROLE == 1 && j >= 2) break;
                        const int o = ROLE == 1 ? 24 * 64 + j * 32 + 16 * p + c : (4 * tb + b4) * 64 + lane;
                        const float4 p4 = L.Pd[o];
                        const float pd[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int r = 4 * b4 + q;
                            const float cz = ROLE == 1 ? racc[q] : acc[r];
                            if (nom) {
                                u[r] = cz;  // the recursion restarts from the direct value
                                vc = fmaxf(vc, cz + pd[q]);
                                mc = fmaxf(mc, __builtin_fabsf(cz) + __builtin_fabsf(pd[q]));
                            }
                        }
                    }
                    const int o = ROLE == 1 ? 16 : 32;
                    vc = fmaxf(vc, __shfl_xor(vc, o, 64));
                    mc = fmaxf(mc, __shfl_xor(mc, o, 64));
                    if (ROLE == 1 ? j == 0 : h == 0)  // the stage-1 reads of every wave precede the barrier above
                        L.slots[ROLE == 1 ? 6 : tb].f[mycol] = make_float4(vc, vc, mc, INFINITY);
                    __syncthreads();
                    bool ver = false;
                    if (lane < 32 && ((mA >> lane) & 1u)) {
                        float vx = -INFINITY, mx = 0.0f;
#pragma unroll
                        for (int g = 0; g < 7; ++g) {
                            const float4 e = L.slots[g].f[lane];
                            vx = fmaxf(vx, e.x);
                            mx = fmaxf(mx, e.z);
                        }
                        ver = viol_ok((double)vx, (double)mx, a.L, a.tol, ViolMargin<float>::value);
                    }
                    m1 = (unsigned)__ballot(ver);
                    m2 &= ~m1;
                }
            }
            // ---- finished columns: results out ---------------------------------------------------
            {
                const int cdq = ((m1 >> mycol) & 1u) ? 1 : (((m2 >> mycol) & 1u) ? 2 : 0);
                if (act && (cdq != 0 || v >= N)) {
                    const size_t b = (size_t)inst;
                    constexpr int NB = ROLE == 1 ? 1 : 4;
#pragma unroll
                    for (int b4 = 0; b4 < NB; ++b4) {
                        const int o = ROLE == 1 ? 24 * 64 + j * 32 + 16 * p + c : (4 * tb + b4) * 64 + lane;
                        const float4 h4 = L.Zh[o];
                        const float zh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int r = 4 * b4 + q;
                            const int i = ROLE == 1 ? 192 + 2 * r + j : row_of(tb, r, h);
                            if (cdq != 2 || zh_out) a.z[b * kN + i] = cdq == 2 ? zh[q] : z[r];
                            a.y[b * kN + i] = y[r];
                        }
                    }
                    if (ROLE == 0 && t == 0 && h == 0) {  // one lane per column
                        a.iters[b] = v;
                        a.conv[b] = cdq;
                    }
                    act = false;
                }
            }
            live &= ~(m1 | m2);
            if (v >= N) live = 0u;
            if (v >= a.v_end || live == 0u) break;
        }
        // ---- phase end: park the survivors -------------------------------------------------------
        if (carry) {
            const bool park = act && v >= a.v_end;
            if (park) {
                const size_t b = (size_t)inst;
                constexpr int NB = ROLE == 1 ? 1 : 4;
#pragma unroll
                for (int b4 = 0; b4 < NB; ++b4) {
                    const int o = ROLE == 1 ? 24 * 64 + j * 32 + 16 * p + c : (4 * tb + b4) * 64 + lane;
                    const float4 w4 = L.Wl[o];
                    const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int r = 4 * b4 + q;
                        const int i = ROLE == 1 ? 192 + 2 * r + j : row_of(tb, r, h);
                        a.z[b * kN + i] = z[r];
                        a.y[b * kN + i] = y[r];
                        a.wc[b * kN + i] = wv[q];
                        if (use_tol) a.uc[b * kN + i] = u[r];
                    }
                }
            }
            if (ROLE == 0 && t == 0) {  // tile 0's lanes 0..31 speak for the item's 32 columns
                const unsigned long long lv = __ballot(park && h == 0);
#pragma unroll
                for (int pp = 0; pp < 2; ++pp) {
                    const unsigned pm = (unsigned)(lv >> (16 * pp)) & 0xffffu;
                    const int P = 2 * it + pp;
                    if (16 * P < count) {
                        if (lane == 0) a.seg_cnt[P] = __popc(pm);
                        if (park && h == 0 && (col >> 4) == pp)
                            a.seg_idx[16 * P + __popc(pm & ((1u << (col & 15)) - 1u))] = inst;
                    }
                }
            }
        }
        __syncthreads();
    }
    if (a.gmax_part) {
        for (int o = 32; o > 0; o >>= 1) gmx = absmax_nan(gmx, __shfl_xor(gmx, o, 64));
        if (lane == 0) L.gred[threadIdx.x >> 6] = gmx;
    }
}

}  // namespace

// Pairs only: a launch whose phase holds no more panels than workgroups returns at once (the
// one-panel layout of gpad_panel2_kernel runs those phases).
__global__ __launch_bounds__(512) void gpad_pair32_kernel(SolveArgs<float> a) {
    __shared__ W32Lds L;
    const int count = a.count_in ? __builtin_amdgcn_readfirstlane(*a.count_in) : a.batch;
    if (a.count_in && count <= a.fin_thresh) return;  // the finisher has them
    const int panels = (count + 15) / 16;
    if (panels <= a.pair32_min) return;  // gpad_panel2_kernel's one-panel layout has them
    const int items = (panels + 1) / 2;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < 2) L.hflag[threadIdx.x] = 0;
    if (threadIdx.x == 0) L.herr = 0;
    if (threadIdx.x < 8) L.gred[threadIdx.x] = 0.0f;
    __syncthreads();
    if (w >= 4) w32_run<0>(a, L, w - 4, 0, items, count);
    else if (w < 2) w32_run<1>(a, L, 0, w, items, count);
    else w32_run<2>(a, L, 0, w - 2, items, count);
    __syncthreads();
    if (threadIdx.x == 0 && L.herr) atomicOr(a.err, kDevErrHandoff);
    if (a.gmax_part && threadIdx.x == 0) {
        float g = 0.0f;
        for (int i = 0; i < 8; ++i) g = absmax_nan(g, L.gred[i]);
        a.gmax_part[blockIdx.x] = absmax_nan(a.gmax_part[blockIdx.x], (double)g);
    }
}

bool pair32_supported(int n, int m) { return n == kN && m == kN; }
size_t pair32_frag_bytes() { return 2 * kImgBytes; }

hipError_t launch_pack_pair32(const float* ML, const float* G, float mg_sign, double g_scale, void* frag,
                              hipStream_t s) {
    const int tot = kTiles * kKB * 64 + kRemB * 64;
    float4* d1 = reinterpret_cast<float4*>(frag);
    float4* d2 = reinterpret_cast<float4*>((char*)frag + kImgBytes);
    hipLaunchKernelGGL(pack_pair32_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, ML, (double)mg_sign, d1);
    hipLaunchKernelGGL(pack_pair32_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, G, g_scale, d2);
    return hipGetLastError();
}

hipError_t launch_pair32(const SolveArgs<float>& a, int grid, hipStream_t s) {
    hipLaunchKernelGGL(gpad_pair32_kernel, dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError();
}

}  // namespace gpad
