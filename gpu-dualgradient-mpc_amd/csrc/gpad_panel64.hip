// gpad_panel64.hip -- shared-matrix f64 batches on the f64 MFMA pipe (gfx950), with the
// value-function branches of Algorithm 1.
//
// The reference's own termination regime (acceldualgrad.m:12-13: e_g = e_V = 1e-6) lies below the
// f32 certification floor (include/gpad.h gpad_run), so it needs f64; with the QP Hessian bound
// (gpad_setup_hessian) the test also evaluates valuefcn / dualfcn (acceldualgrad.m:30-33, 73, 76).
// Until round 4 only the one-workgroup-per-instance stream kernel ran f64, streaming the shared
// matrices from L2 for every instance.  Here a workgroup owns a panel of 16 instances and wave t
// owns row tile t of both GEMMs, as gpad_panel_kernel does in f32:
//   Zhat[n x 16] = (-ML) W[m x 16],   C[m x 16] = G_L Zhat[n x 16]
// on v_mfma_f64_16x16x4_f64, whose result is bitwise the ascending-k fma chain
// (profiles/r04_mfma_f64.txt: 0 of 256 outputs differ over K = 200) -- so every chain here is the
// f64 stream kernel's chain4 (fma, ascending k), and the epilogues are its epilogues: z, y, w, u and
// the iteration counts equal the stream kernel's bit for bit, and the fp64 oracle's
// (orc_solve_value_f64, acceldualgrad.m's mul/add order) to rounding (tests/test_panel64.py).
//
// Layouts (f64 16x16x4: lane l supplies A[l&15][k = l>>4] and B[k = l>>4][l&15], accumulator
// register r holds D[(l>>4) + 4r][l&15]):
//   PA[b][t][lane][q] = M[16t + (lane&15)][16b + 4q + (lane>>4)]   (4 doubles = 32 B per lane)
// so accumulator register q of lane l in wave t is row 16t + 4q + (l>>4): exactly the B operand of
// k-step q of k-block t of the next GEMM.  No row permutation is needed (the f32 kernels need one,
// their accumulator layout is row 4(l>>4) + r).  Vectors cross between the GEMMs through LDS in
// that fragment order, [tile][lane][4] doubles; each lane keeps its own rows' z, y, u, g_P, p_D in
// registers.  Images: -ML, G_L and (value branches) H, each T x T tiles of 2 KiB.
//
// Value branches, per column, where the MATLAB test reaches them (test (B)'s violation part passed,
// the rest of (B) did not): V(zhat) from one H-GEMM over the panel; for columns with w not >= 0
// also D(y+) = V(z(y+)) + L y+'(G_L z(y+) + p_D), z(y+) = -ML y+ - M: three more GEMMs.  Sums over
// rows are fp64 trees (lane rows, lane groups, tiles) -- the stream kernel sums in another tree
// order, the oracle sequentially (the same values to ~1e-16 relative).
#include <hip/hip_runtime.h>

#include <atomic>

#include <cmath>

#include "gpad_internal.h"

namespace gpad {

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kP64MaxTiles = 16;  // n, m <= 256 (16 waves)

int p64_tiles(int n, int m) {
    const int t = ((n > m ? n : m) + 15) / 16;
    return t <= kP64MaxTiles ? t : 0;
}

__global__ void pack_panel64_kernel(const double* __restrict__ src, int rows, int cols, double scale, int T,
                                    double* __restrict__ dst) {
    // dst[((b*T + t)*64 + lane)*4 + q] for k-block b < T, row tile t < T
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= T * T * 64) return;
    const int lane = idx & 63, t = (idx >> 6) % T, b = (idx >> 6) / T;
    const int row = 16 * t + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int col = 16 * b + 4 * q + (lane >> 4);
        dst[(size_t)idx * 4 + q] = (row < rows && col < cols) ? scale * src[(size_t)row * cols + col] : 0.0;
    }
}

__device__ __forceinline__ f64x4 ld_a(__amdgpu_buffer_rsrc_t PA, int voff, int soff) {
    const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(PA, voff, soff, 0);
    const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(PA, voff + 16, soff, 0);
    f64x4 r;
    r[0] = __hiloint2double((int)lo.y, (int)lo.x);
    r[1] = __hiloint2double((int)lo.w, (int)lo.z);
    r[2] = __hiloint2double((int)hi.y, (int)hi.x);
    r[3] = __hiloint2double((int)hi.w, (int)hi.z);
    return r;
}

// acc = A[tile t] x B over k-blocks [0, nkb) (ascending k: the fma chain), A streamed from L2 one
// block ahead, B (fragment order) from LDS one block ahead.  Zero-padded k-steps add +0 only.
// gemm64p: block 0's A operand a0 given (loaded before the barrier that precedes the GEMM, so the
// chain does not start with an L2 round trip)
template <int T>
__device__ __forceinline__ f64x4 gemm64p(__amdgpu_buffer_rsrc_t PA, const f64x4* __restrict__ Bl, int voff, int lane,
                                         int nkb, const f64x4& a0) {
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    f64x4 a[2], b[2];
    a[0] = a0;
    b[0] = Bl[lane];
#pragma unroll
    for (int kb = 0; kb < T; ++kb) {
        const int cur = kb & 1, nxt = cur ^ 1;
        if (kb < nkb) {  // uniform (nkb < T only when n != m)
            if (kb + 1 < nkb) {
                a[nxt] = ld_a(PA, voff, (kb + 1) * T * 2048);
                b[nxt] = Bl[(kb + 1) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cur][0], b[cur][0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cur][1], b[cur][1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cur][2], b[cur][2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cur][3], b[cur][3], acc, 0, 0, 0);
            asm volatile("" ::: "memory");
        }
    }
    return acc;
}

template <int T>
__device__ __forceinline__ f64x4 gemm64(__amdgpu_buffer_rsrc_t PA, const f64x4* __restrict__ Bl, int voff, int lane,
                                        int nkb) {
    return gemm64p<T>(PA, Bl, voff, lane, nkb, ld_a(PA, voff, 0));
}

// blocks [KB0, KB1) of the chain of the tile at voff, continued from acc (a relay piece, or the
// owner's last piece): the same MFMA sequence as gemm64's, so the cut is bit-invisible
template <int T, int KB0, int KB1>
__device__ __forceinline__ void chain64(__amdgpu_buffer_rsrc_t PA, const f64x4* __restrict__ Bl, int voff, int lane,
                                        f64x4& acc, const f64x4& a0) {
    f64x4 a[2], b[2];
    a[0] = a0;  // block KB0, loaded ahead
    b[0] = Bl[KB0 * 64 + lane];
#pragma unroll
    for (int kb = KB0; kb < KB1; ++kb) {
        const int cur = (kb - KB0) & 1, nxt = cur ^ 1;
        if (kb + 1 < KB1) {
            a[nxt] = ld_a(PA, voff, (kb + 1) * T * 2048);
            b[nxt] = Bl[(kb + 1) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cur][0], b[cur][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cur][1], b[cur][1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cur][2], b[cur][2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[cur][3], b[cur][3], acc, 0, 0, 0);
        asm volatile("" ::: "memory");
    }
}

// The relay layout (round 5).  One panel per 13-wave workgroup put 4,3,3,3 chains on the SIMDs
// (the f64 pipe is saturated by ONE dependent chain per SIMD -- 74 cycles per step alone, 64 at
// full rate, profiles/r04_mfma_f64.txt -- so the busiest SIMD's chain count is the iteration time).
// With 16 waves, tile T-1's chain is cut into four pieces: k-blocks [0, C1) on relay wave 0,
// [C1, C2) on relay wave 1, [C2, C3) on relay wave 2 -- one on each SIMD that lacks tile T-1 --
// and [C3, T) plus the epilogue on the tile's owner; each piece continues from the accumulator the
// previous one parked in LDS (bit-identical: the same ascending-k MFMA sequence).  T = 13: SIMD
// loads 52,39,39,39 k-blocks -> 43,42,42,42.  Roles are dealt from the last wave down (the SIMD
// issues MFMAs oldest wave first), so the sequential relay runs on the oldest waves, at raised
// priority, as in the f32 one-panel relay (gpad_panel.hip Handoff).  Relay waves own a phantom
// tile T (no rows) everywhere else, so they follow the workgroup's control flow and barriers
// without touching the real tiles' state.
template <int T>
struct P64Relay {
    static constexpr bool on = T == 9 || T == 13;  // T % 4 == 1: SIMD 0 carries the extra tile
    static constexpr int C1 = T / 4, C2 = 2 * T / 4, C3 = 3 * T / 4;
};

struct P64Slot {  // per tile and column: the test partials / the value-function sums
    double violz[16], violh[16], wmin[16], gap[16], magh[16];
};

// max / min / sum of this lane's 4 rows over the 4 lane groups of its column (xor 16, 32)
__device__ __forceinline__ double col_max(double v) {
    v = fmax(v, __shfl_xor(v, 16, 64));
    return fmax(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ double col_min(double v) {
    v = fmin(v, __shfl_xor(v, 16, 64));
    return fmin(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ double col_sum(double v) {
    v += __shfl_xor(v, 16, 64);
    return v + __shfl_xor(v, 32, 64);
}

}  // namespace

// LDS of the kernel: w (B of GEMM 1, fragment order), zhat (B of GEMM 2), Xv (z for the (A)
// verification; the value branches' operands), g_P of the lanes' rows (registers are the limit),
// the test slots and the value sums, per tile -- plus the relay waves' phantom tile -- and:
template <int T, bool RELAY>
struct P64Lds {
    static constexpr int TL = RELAY ? T + 1 : T;
};
template <bool RELAY>
struct P64Hand {
    f64x4 hand[RELAY ? 3 : 1][64];  // relay: parked accumulators
    int hflag[3];                   // relay: hand-off generation per slot
    int herr;                       // relay: a wait expired (reported at exit, GPAD_ERR_DEVICE)
};

// bounded wait for a parked accumulator (as gpad_panel.hip handoff_wait: an expired wait is
// recorded and fails the run rather than hanging the GPU or returning stale results)
template <class Lds>
__device__ __forceinline__ f64x4 p64_wait(Lds& L, int slot, int gen, int lane) {
    for (int s = 0;; ++s) {
        if (__hip_atomic_load(&L.hflag[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == gen) break;
        if (s == (1 << 20)) {
            L.herr = 1;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    return L.hand[slot][lane];
}

template <class Lds>
__device__ __forceinline__ void p64_post(Lds& L, int slot, int gen, int lane, const f64x4& h) {
    L.hand[slot][lane] = h;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the accumulator lands before the flag
    __hip_atomic_store(&L.hflag[slot], gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// a main GEMM of tile t (gemm64), or -- relay layout -- this wave's piece of tile T-1's chain
// the first A block this wave's part of a main GEMM needs (issued before the preceding barrier)
template <int T, bool RELAY>
__device__ __forceinline__ f64x4 p64_first_a(__amdgpu_buffer_rsrc_t PA, int voff, int lane, bool on, int rrole) {
    using R = P64Relay<T>;
    if constexpr (RELAY) {
        if (rrole >= 0 && rrole <= 3) {
            const int kb = rrole == 0 ? 0 : (rrole == 1 ? R::C1 : (rrole == 2 ? R::C2 : R::C3));
            return ld_a(PA, (T - 1) * 2048 + lane * 32, kb * T * 2048);
        }
        if (rrole > 3) return f64x4{0.0, 0.0, 0.0, 0.0};
    }
    return on ? ld_a(PA, voff, 0) : f64x4{0.0, 0.0, 0.0, 0.0};
}

template <int T, bool RELAY, class Lds>
__device__ __forceinline__ f64x4 p64_gemm(Lds& L, __amdgpu_buffer_rsrc_t PA, const f64x4* __restrict__ Bl, int voff,
                                          int lane, int nkb, bool on, int rrole, int gen, const f64x4& a0) {
    using R = P64Relay<T>;
    if constexpr (RELAY) {
        const int vo = (T - 1) * 2048 + lane * 32;
        f64x4 h = {0.0, 0.0, 0.0, 0.0};
        if (rrole == 0) {
            __builtin_amdgcn_s_setprio(3);
            chain64<T, 0, R::C1>(PA, Bl, vo, lane, h, a0);
            p64_post(L, 0, gen, lane, h);
            __builtin_amdgcn_s_setprio(0);
            return f64x4{0.0, 0.0, 0.0, 0.0};
        }
        if (rrole == 1 || rrole == 2) {
            h = p64_wait(L, rrole - 1, gen, lane);
            __builtin_amdgcn_s_setprio(3);
            if (rrole == 1) chain64<T, R::C1, R::C2>(PA, Bl, vo, lane, h, a0);
            else chain64<T, R::C2, R::C3>(PA, Bl, vo, lane, h, a0);
            p64_post(L, rrole, gen, lane, h);
            __builtin_amdgcn_s_setprio(0);
            return f64x4{0.0, 0.0, 0.0, 0.0};
        }
        if (rrole == 3) {  // the owner of tile T-1: the last piece
            h = p64_wait(L, 2, gen, lane);
            __builtin_amdgcn_s_setprio(2);
            chain64<T, R::C3, T>(PA, Bl, vo, lane, h, a0);
            __builtin_amdgcn_s_setprio(0);
            return h;
        }
        if (rrole > 3) return f64x4{0.0, 0.0, 0.0, 0.0};  // idle (T = 9: waves past the relay)
    }
    return on ? gemm64p<T>(PA, Bl, voff, lane, nkb, a0) : f64x4{0.0, 0.0, 0.0, 0.0};
}

// REFILL (round 5, tol > 0 with N a multiple of the test period and more panels than workgroups):
// a finished column takes the next instance of the batch from a device counter (a.qctr) at the
// test event that finished it, instead of idling until its panel's slowest column is done.  Each
// column keeps its own iteration count vc (theta_vc, beta_vc+1 per lane); columns start only at
// test events, so every column's vc stays congruent to the workgroup's step count modulo K and the
// test events stay uniform.  Every column's arithmetic is the one-panel-at-a-time kernel's (the
// MFMA output column depends on its B column only), so z, y, counts and codes are bit-identical.
// 8192 value problems on 256 CUs (two per column on average): profiles/r05_p64_refill_ab.txt.
template <int T, bool RELAY, bool REFILL>
__global__ __launch_bounds__(RELAY ? 1024 : 64 * T) void gpad_panel64_kernel(SolveArgs<double> a) {
    constexpr int TL = P64Lds<T, RELAY>::TL;
    __shared__ f64x4 Wl[TL * 64];
    __shared__ f64x4 Zh[TL * 64];
    __shared__ f64x4 Xv[TL * 64];
    __shared__ f64x4 Gp[TL * 64];
    __shared__ P64Slot slots[TL];
    __shared__ double vsum[2][TL][16];
    __shared__ P64Hand<RELAY> L;
    __shared__ int newinst[16];  // REFILL: the instance each column takes next (-1 none, -2 keeps its own)

    const int lane = threadIdx.x & 63;
    // role: tile index (relay layout: dealt from the last wave down; roles >= T are relay waves
    // on the phantom tile T); rrole: 0..2 relay pieces, 3 the owner of tile T-1, -1 none
    const int w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int role = RELAY ? 15 - w0 : w0;
    const int t = role < T ? role : T;
    const int rrole = !RELAY ? -1 : (role == T - 1 ? 3 : (role >= T ? (role - T < 3 ? role - T : 4) : -1));
    if (RELAY) {
        if (threadIdx.x < 3) L.hflag[threadIdx.x] = 0;
        if (threadIdx.x == 0) L.herr = 0;
        __syncthreads();
    }
    int hgen = 0;
    const int j = lane >> 4, c = lane & 15;
    const int n = a.n, m = a.m, N = a.N, K = a.check_every;
    const int nkb1 = (m + 15) / 16, nkb2 = (n + 15) / 16;  // k-blocks of GEMM 1 (K = m), GEMM 2 / H (K = n)
    const bool on1 = 16 * t < n, on2 = 16 * t < m;         // this tile has output rows in GEMM 1 / 2
    const int abytes = T * T * 2048;
    const __amdgpu_buffer_rsrc_t PA1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.frag), 0, abytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t PA2 =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)a.frag + abytes), 0, abytes, 0x00020000);
    const bool value = a.hfrag64 != nullptr && a.tol > 0.0;
    const __amdgpu_buffer_rsrc_t PH =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(value ? a.hfrag64 : a.frag), 0, abytes, 0x00020000);
    const int voff = t * 2048 + lane * 32;
    const int slot = t * 64 + lane;
    const bool use_tol = a.tol > 0.0;
    const double eV = a.tol_gap;
    const int panels = (a.batch + 15) / 16;

    // (REFILL: one pass -- the panels past the first grid are dealt column by column through the queue)
    for (int p = blockIdx.x; p < panels && (!REFILL || p == (int)blockIdx.x); p += gridDim.x) {
        // REFILL with a.order: the k-th instance started is order[k] (longest predicted first, so the
        // refills pair long first instances with short later ones: list scheduling over the columns)
        const int k0 = 16 * p + c;
        bool active = k0 < a.batch;
        int inst = (REFILL && a.order && active) ? a.order[k0] : k0;
        // register r <-> row 16t + 4r + j of the column's instance
        double z[4], y[4], u[4], pd[4];
        // a column's starting state (every column at a panel's start; REFILL: the refilled ones)
        auto load_col = [&](bool mine) {
            f64x4 w, gp;
            const f64x4 w_old = Wl[slot], gp_old = Gp[slot];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * t + 4 * r + j;
                const bool okn = active && i < n, okm = active && i < m;
                const double zr = okn ? a.z[(size_t)inst * n + i] : 0.0;
                gp[r] = okn ? a.gP[(size_t)inst * a.ld_gP + i] : 0.0;
                const double yr = okm ? a.y[(size_t)inst * m + i] : 0.0;
                const double pr = okm ? a.gscale * a.g[(size_t)inst * a.ld_g + i] : 0.0;
                w[r] = __builtin_fma(a.beta[0], yr - yr, yr);  // 8a with y_0 = y_{-1}
                if (mine) {
                    z[r] = zr;
                    y[r] = yr;
                    pd[r] = pr;
                    u[r] = 0.0;
                } else {
                    w[r] = w_old[r];
                    gp[r] = gp_old[r];
                }
            }
            Wl[slot] = w;
            Gp[slot] = gp;
            Xv[slot] = f64x4{z[0], z[1], z[2], z[3]};
        };
        load_col(true);
        __syncthreads();
        if (use_tol && on2) {  // u = G_L z_{-1}, then the 8c recursion
            const f64x4 cz = gemm64<T>(PA2, Xv, voff, lane, nkb2);
#pragma unroll
            for (int r = 0; r < 4; ++r) u[r] = cz[r];
        }
        __syncthreads();

        int v = 0;   // workgroup steps (= every column's iteration count without REFILL)
        int vc = 0;  // REFILL: this column's iteration count
        f64x4 apre = p64_first_a<T, RELAY>(PA1, voff, lane, on1, rrole);  // GEMM 1's first A block
        while (true) {
            const int vi = REFILL ? vc : v;
            const double th = a.theta[vi], bn = a.beta[vi + 1];
            ++v;
            if (REFILL && active) ++vc;
            const bool chk = use_tol && (v % K) == 0;
            const double omt = 1.0 - th;
            // ---- GEMM 1 + epilogue: zhat = -ML w - g_P (8b), z = (1-th) z + th zhat (8c) ----
            {
                const f64x4 acc = p64_gemm<T, RELAY>(L, PA1, Wl, voff, lane, nkb1, on1, rrole, ++hgen, apre);
                apre = p64_first_a<T, RELAY>(PA2, voff, lane, on2, rrole);  // GEMM 2's, across the barrier
                const f64x4 gp = Gp[slot];
                f64x4 zh;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    zh[r] = acc[r] - gp[r];
                    const double zn = __builtin_fma(omt, z[r], th * zh[r]);
                    if (active) z[r] = zn;
                }
                Zh[slot] = zh;
            }
            __syncthreads();
            // ---- GEMM 2 + epilogue: y+ = [w + G_L zhat + p_D]+ (8d), next w (8a), test partials ----
            double violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0, gap = 0.0;
            {
                const f64x4 acc = p64_gemm<T, RELAY>(L, PA2, Zh, voff, lane, nkb2, on2, rrole, ++hgen, apre);
                apre = p64_first_a<T, RELAY>(PA1, voff, lane, on1, rrole);  // the next GEMM 1's
                const f64x4 wv = Wl[slot];
                f64x4 wn;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double cv = acc[r];
                    const double sv = (wv[r] + pd[r]) + cv;  // seq_functions.cpp:84
                    const double yp = (fabs(sv) + sv) * 0.5;  // seq_functions.cpp:85
                    wn[r] = __builtin_fma(bn, yp - y[r], yp);
                    if (use_tol) {
                        const double un = __builtin_fma(omt, u[r], th * cv);
                        if (active) u[r] = un;
                        if (chk && active && (16 * t + 4 * r + j) < m) {
                            const double tt = cv + pd[r];
                            violh = fmax(violh, tt);
                            magh = fmax(magh, fabs(cv) + fabs(pd[r]));
                            wmin = fmin(wmin, wv[r]);
                            gap -= wv[r] * tt;
                            violz = fmax(violz, u[r] + pd[r]);
                        }
                    }
                    if (active) y[r] = yp;
                }
                if (active) Wl[slot] = wn;  // (GEMM 2 reads Zh; the next GEMM 1 reads w after the barrier)
            }
            if (chk) {
                violz = col_max(violz);
                violh = col_max(violh);
                magh = col_max(magh);
                wmin = col_min(wmin);
                gap = col_sum(gap);
                if (j == 0) {
                    slots[t].violz[c] = violz;
                    slots[t].violh[c] = violh;
                    slots[t].magh[c] = magh;
                    slots[t].wmin[c] = wmin;
                    slots[t].gap[c] = gap;
                }
            }
            __syncthreads();
            if (REFILL ? !chk : (!chk && v < N)) continue;  // (REFILL: N % K == 0, a column reaches N at a test)
            const int vd = REFILL ? vc : v;  // this column's iteration count

            // ---- Algorithm 1, per column (lane c's column; every wave reads every tile) ----------
            int code = 0;
            if (chk) {
                int st1 = 0;
                bool vh_ok = false, w_ok = false;
                double gq = 0.0;
                if (active) {
                    double vz = -INFINITY, vh = -INFINITY, wm = INFINITY, mh = 0.0;
#pragma unroll
                    for (int s2 = 0; s2 < T; ++s2) {
                        vz = fmax(vz, slots[s2].violz[c]);
                        vh = fmax(vh, slots[s2].violh[c]);
                        mh = fmax(mh, slots[s2].magh[c]);
                        wm = fmin(wm, slots[s2].wmin[c]);
                        gq += slots[s2].gap[c];
                    }
                    vh_ok = viol_ok(vh, mh, a.L, a.tol, ViolMargin<double>::value);
                    w_ok = wm >= 0.0;
                    st1 = (vz * a.L <= a.tol ? 1 : 0) | ((vh_ok && w_ok && (gq * a.L <= a.tol_gap)) ? 2 : 0);
                }
                bool verified = false;
                if (__syncthreads_or(st1 & 1)) {  // (A) nominated somewhere: G_L z for the panel
                    Xv[slot] = f64x4{z[0], z[1], z[2], z[3]};
                    __syncthreads();
                    const f64x4 cz = on2 ? gemm64<T>(PA2, Xv, voff, lane, nkb2) : f64x4{0.0, 0.0, 0.0, 0.0};
                    double vc = -INFINITY, mc = 0.0;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if ((st1 & 1) && (16 * t + 4 * r + j) < m) {
                            u[r] = cz[r];  // the recursion restarts from the direct value
                            vc = fmax(vc, cz[r] + pd[r]);
                            mc = fmax(mc, fabs(cz[r]) + fabs(pd[r]));
                        }
                    }
                    vc = col_max(vc);
                    mc = col_max(mc);
                    if (j == 0) {  // every wave read the stage-1 slots before the barrier above
                        slots[t].violz[c] = vc;
                        slots[t].magh[c] = mc;
                    }
                    __syncthreads();
                    if (st1 & 1) {
                        double vcc = -INFINITY, mcc = 0.0;
#pragma unroll
                        for (int s2 = 0; s2 < T; ++s2) {
                            vcc = fmax(vcc, slots[s2].violz[c]);
                            mcc = fmax(mcc, slots[s2].magh[c]);
                        }
                        verified = viol_ok(vcc, mcc, a.L, a.tol, ViolMargin<double>::value);
                    }
                }
                code = ((st1 & 1) && verified) ? 1 : ((st1 & 2) ? 2 : 0);
                // value-function branches (acceldualgrad.m:73, 76) where the MATLAB test reaches them
                const bool need = value && active && code == 0 && vh_ok;
                if (value && __syncthreads_or(need)) {
                    // V(zhat) = sum_i (zhat_i / 2 + M_i) (H zhat)_i  (zhat: this iteration's, in Zh)
                    const f64x4 gp = Gp[slot], zk = Zh[slot];
                    double vp = 0.0;
                    if (on1) {
                        const f64x4 hx = gemm64<T>(PH, Zh, voff, lane, nkb2);
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (16 * t + 4 * r + j < n) vp += (0.5 * zk[r] + gp[r]) * hx[r];
                    }
                    vp = col_sum(vp);
                    if (j == 0) vsum[0][t][c] = vp;
                    __syncthreads();
                    double V = 0.0;
#pragma unroll
                    for (int s2 = 0; s2 < T; ++s2) V += vsum[0][s2][c];
                    if (need && w_ok) code = gq * a.L <= V * eV / (1.0 + eV) ? 3 : 0;  // :73
                    const bool needd = need && !w_ok;
                    if (__syncthreads_or(needd)) {
                        // z(y+) = -ML y+ - M (GEMM 1 on y+), then V(z(y+)) and y+'(G_L z(y+) + p_D)
                        // (the barrier of the vote: Xv is free, every (A) verification GEMM is done)
                        Xv[slot] = f64x4{y[0], y[1], y[2], y[3]};
                        __syncthreads();
                        f64x4 zp = {0.0, 0.0, 0.0, 0.0};
                        if (on1) {
                            const f64x4 acc = gemm64<T>(PA1, Xv, voff, lane, nkb1);
#pragma unroll
                            for (int r = 0; r < 4; ++r) zp[r] = acc[r] - gp[r];
                        }
                        __syncthreads();
                        Xv[slot] = zp;
                        __syncthreads();
                        double vq = 0.0, lin = 0.0;
                        if (on1) {
                            const f64x4 hx = gemm64<T>(PH, Xv, voff, lane, nkb2);
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (16 * t + 4 * r + j < n) vq += (0.5 * zp[r] + gp[r]) * hx[r];
                        }
                        if (on2) {
                            const f64x4 cc = gemm64<T>(PA2, Xv, voff, lane, nkb2);
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (16 * t + 4 * r + j < m) lin += y[r] * (cc[r] + pd[r]);
                        }
                        vq = col_sum(vq);
                        lin = col_sum(lin);
                        if (j == 0) {
                            vsum[0][t][c] = vq;
                            vsum[1][t][c] = lin;
                        }
                        __syncthreads();
                        double Vp = 0.0, ls = 0.0;
#pragma unroll
                        for (int s2 = 0; s2 < T; ++s2) {
                            Vp += vsum[0][s2][c];
                            ls += vsum[1][s2][c];
                        }
                        const double D = Vp + a.L * ls;
                        if (needd) code = V - D <= eV * (D > 1.0 ? D : 1.0) ? 4 : 0;  // :76
                    }
                }
            }
            // ---- finished columns: results out (tests (B), (B'), (B'') certify zhat) -----------
            if (active && (code != 0 || vd >= N)) {
                const f64x4 zk = Zh[slot];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * t + 4 * r + j;
                    if (i < n) a.z[(size_t)inst * n + i] = code >= 2 ? zk[r] : z[r];
                    if (i < m) a.y[(size_t)inst * m + i] = y[r];
                }
                if (t == 0 && j == 0) {
                    a.iters[inst] = vd;
                    a.conv[inst] = code;
                }
                active = false;
            }
            if constexpr (REFILL) {
                // finished columns take the next instances (wave 0 claims for the workgroup; the
                // instances past the first grid x 16 are dealt in claim order)
                if (w0 == 0 && lane < 16) {
                    const unsigned long long needm = __ballot(!active);
                    const int cnt = (int)__popcll(needm & 0xffffull);
                    int base = 0;
                    if (lane == 0 && cnt) base = atomicAdd(a.qctr, cnt);
                    base = __shfl(base, 0, 64);
                    const int rank = (int)__popcll(needm & ((1ull << lane) - 1ull));
                    const int k = 16 * (int)gridDim.x + base + rank;
                    newinst[lane] = active ? -2 : (k < a.batch ? (a.order ? a.order[k] : k) : -1);
                }
                __syncthreads();
                const int nk = newinst[c];
                const bool fresh_col = nk >= 0;
                if (fresh_col) {
                    inst = nk;
                    active = true;
                    vc = 0;
                }
                if (__syncthreads_or(fresh_col ? 1 : 0)) {
                    load_col(fresh_col);
                    bool znz = false;
#pragma unroll
                    for (int r = 0; r < 4; ++r) znz = znz || (fresh_col && z[r] != 0.0);
                    if (__syncthreads_or(znz ? 1 : 0)) {  // u = G_L z_{-1} for the new columns (Xv = z)
                        const f64x4 cz = on2 ? gemm64<T>(PA2, Xv, voff, lane, nkb2) : f64x4{0.0, 0.0, 0.0, 0.0};
                        if (fresh_col) {
#pragma unroll
                            for (int r = 0; r < 4; ++r) u[r] = cz[r];
                        }
                        __syncthreads();
                    }
                }
            }
            if (!__syncthreads_or(active ? 1 : 0)) break;
        }
        __syncthreads();  // the next panel reuses the LDS tiles
    }
    if (RELAY && threadIdx.x == 0 && L.herr) atomicOr(a.err, kDevErrHandoff);  // (the last barrier above)
}

bool panel64_supported(int n, int m) { return p64_tiles(n, m) > 0; }
int panel64_tiles(int n, int m) { return p64_tiles(n, m); }
size_t panel64_frag_bytes(int n, int m) {
    const int T = p64_tiles(n, m);
    return (size_t)T * T * 2048;  // one operand
}

hipError_t launch_pack_panel64(const double* src, int rows, int cols, double scale, int T, void* dst, hipStream_t s) {
    const int tot = T * T * 64;
    hipLaunchKernelGGL(pack_panel64_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, src, rows, cols, scale, T,
                       (double*)dst);
    return hipGetLastError();
}

// Workgroups per CU the kernel's registers and LDS allow (hipOccupancy...): a persistent grid of
// num_cus x that, so small tile counts fill the CU with several panels (num_cus
// workgroups of T waves left T <= 4 at 1-4 waves per CU).  Cached per instantiation and per device
// (the group API drives several devices from one process; concurrent host threads may race on a
// slot, but every writer stores the same value, atomically).
constexpr int kP64OccDevices = 64;
template <int T, bool RELAY, bool REFILL>
int p64_per_cu() {
    static std::atomic<int> occ[kP64OccDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    const bool cached = dev >= 0 && dev < kP64OccDevices;
    if (cached) {
        const int o = occ[dev].load(std::memory_order_relaxed);
        if (o) return o;
    }
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, gpad_panel64_kernel<T, RELAY, REFILL>, RELAY ? 1024 : 64 * T,
                                                     0) != hipSuccess ||
        o < 1)
        o = 1;
    if (cached) occ[dev].store(o, std::memory_order_relaxed);
    return o;
}

template <int T, bool RELAY>
hipError_t launch_p64(const SolveArgs<double>& a, hipStream_t s) {
    const int panels = (a.batch + 15) / 16;
    const int K = a.check_every > 0 ? a.check_every : 1;
    // refills need a counter, a tolerance, N on a test event, and more panels than workgroups (the
    // grid of the refill instantiation decides; its occupancy is then that of the kernel launched)
    const int cap_r = a.num_cus * p64_per_cu<T, RELAY, true>();
    const bool refill = a.qctr && a.tol > 0.0 && a.N % K == 0 && panels > cap_r && !(a.tune && a.tune->p64_no_refill);
    const int cap = refill ? cap_r : a.num_cus * p64_per_cu<T, RELAY, false>();
    const int grid = panels < cap ? panels : cap;
    if (refill) {
        hipError_t e = hipMemsetAsync(a.qctr, 0, sizeof(int), s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((gpad_panel64_kernel<T, RELAY, true>), dim3(grid), dim3(RELAY ? 1024 : 64 * T), 0, s, a);
    } else {
        hipLaunchKernelGGL((gpad_panel64_kernel<T, RELAY, false>), dim3(grid), dim3(RELAY ? 1024 : 64 * T), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_panel64(const SolveArgs<double>& a, hipStream_t s) {
    const int T = p64_tiles(a.n, a.m);
    if (!T || !a.frag || a.frag_tiles != T || a.strideA || a.strideB) return hipErrorInvalidValue;
    // fresh, whole solves only: the kernel starts every instance at v = 0 from (z_{-1}, y_0) and runs
    // no phases -- a phased caller's window, work list or carried w / u would be silently ignored
    if (a.v_begin != 0 || a.v_end != 0 || a.pwork || a.idx_in || a.count_in || a.wc || a.uc)
        return hipErrorInvalidValue;
    // the relay layout needs full-length chains in both GEMMs (tile T-1 has rows in both)
    const bool relay = (a.n + 15) / 16 == T && (a.m + 15) / 16 == T && !(a.tune && a.tune->p64_no_relay);
    switch (T) {
#define GPAD_P64(TT) \
    case TT: return launch_p64<TT, false>(a, s);
#define GPAD_P64R(TT) \
    case TT: return relay ? launch_p64<TT, true>(a, s) : launch_p64<TT, false>(a, s);
        GPAD_P64(1) GPAD_P64(2) GPAD_P64(3) GPAD_P64(4) GPAD_P64(5) GPAD_P64(6) GPAD_P64(7) GPAD_P64(8)
        GPAD_P64R(9) GPAD_P64(10) GPAD_P64(11) GPAD_P64(12) GPAD_P64R(13) GPAD_P64(14) GPAD_P64(15) GPAD_P64(16)
#undef GPAD_P64
#undef GPAD_P64R
        default: return hipErrorInvalidValue;
    }
}

}  // namespace gpad
