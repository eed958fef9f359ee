// gpad_duo.hip -- the two-instance ping-pong latency kernel (shared matrices), separate from
// gpad_kernels.hip so the two sets of template instantiations compile in parallel.
#include <hip/hip_runtime.h>

#include <cmath>

#include "gpad_chain.h"
#include "gpad_internal.h"

namespace gpad {

// =========================================================================================
// gpad_duo_kernel: shared matrices, TWO instances per workgroup in ping-pong, fed by a queue.
// =========================================================================================
// The resident kernel keeps one instance per CU, and its two half-iterations alternate: while
// the -ML waves run the 8b chains the G/L waves wait at the barrier and vice versa, so each
// SIMD issues one dependent fma chain at a time (~1/3 of its VALU issue rate).  With shared
// matrices the same register-resident rows can serve two instances X, Y at once, one half-
// iteration apart: in step s the -ML waves run 8b of slot s&1 while the G/L waves run 8d of the
// other slot, so the A and B wave of every SIMD both issue (two independent chains interleave
// on the SIMD).  Two instance-iterations per two steps instead of one, at the same per-step
// latency.  Each slot is refilled from a work list (idx_in / count_in: the survivors of a
// phased panel solve, or 0..batch-1) as its instance finishes: the first two instances of
// workgroup g are list positions g and g + G, later ones are claimed from a device counter
// (`qctr`, +2G) one refill ahead, so the matrix rows are loaded once per CU, not per instance.
//
// Slot bookkeeping (pos, vs, need8d) is computed identically by every wave from uniform values
// and LDS words, so the control flow around the DPP chains and barriers stays uniform.  Per
// instance the arithmetic is exactly the resident kernel's (same chains, same epilogues, same
// test with the same wave reductions), hence bit-identical results and iteration counts.
struct DuoSlot {  // one instance slot; bookkeeping is uniform, the floats are this lane's rows
    int pos, vs, nextp;  // list position (>= count: empty), iterations done, pre-claimed next
    int kc;              // 8d steps to the next test: the test runs at iteration vs + 1 when kc == 1
    bool need8d;         // 8b done, 8d pending
    float th, bn;        // theta_vs, beta_{vs+1}: loaded one step before their use (a deeper
                         // prefetch, or g_P / p_D in registers instead of LDS, spills: the rows
                         // take 200 of the 256 VGPRs -- profiles/r03_duo_solo.txt)
    float x0, x1, x2;    // -ML lanes: z, zhat, -;  G/L lanes: y, w, u = G_L z (g_P, p_D in LDS)
};
struct DuoCtx {
    int tid, count, G, v0, n, m, N, Kc, kc0, nA, nwaves, row, claim_base, b0;  // b0: first G/L wave
    bool fresh, use_tol, isA, live;
#ifdef GPAD_STAMP
    int step;  // steps taken (stamps)
#endif
};

// The schedule through the constant address space: the index is uniform, so theta / beta arrive by
// scalar loads into SGPRs (four fewer VGPRs next to the 200 register-resident matrix entries;
// the time per step is the same as with vector loads, profiles/r03_duo_solo.txt "duo3").
__device__ __forceinline__ float sched(const float* t, int v) {
    return ((const __attribute__((address_space(4))) float*)(t))[v];
}

// An instance's row vectors through buffer operations: the base (instance row b of a [batch][ld]
// array) is uniform and lives in SGPRs, the lane's offset is one 32-bit VGPR (4 row), so a refill
// holds no per-lane 64-bit pointers (six of them, hoisted out of the loop, were spilled to scratch).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* base, size_t b, int ld) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(static_cast<const char*>(base) + 4 * b * (size_t)ld),
                                             0, 4 * ld, 0x00020000);
}
__device__ __forceinline__ float row_ld(const void* base, size_t b, int ld, int off4) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(row_rsrc(base, b, ld), off4, 0, 0));
}
__device__ __forceinline__ void row_st(void* base, size_t b, int ld, int off4, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), row_rsrc(base, b, ld), off4, 0, 0);
}

// slot s takes list position p (empty if p >= count); uniform, contains barriers
// gp_l / pd_l: this slot's per-row constants (g_P of the -ML rows, p_D of the G/L rows)
template <int KB, int K>
__device__ __forceinline__ void duo_refill(const SolveArgs<float>& a, const DuoCtx& c, DuoSlot& s, int p,
                                           float* w_l, float* gp_l, float* pd_l, float* z_l,
                                           const float (&r)[K]) {
    s.pos = __builtin_amdgcn_readfirstlane(p);  // (uniform: scalar bookkeeping, see duo_step)
    const int v = c.v0;
    s.vs = v;
    s.kc = c.kc0;
    s.need8d = false;
    s.th = sched(a.theta, v);
    s.bn = sched(a.beta, v + 1);
    s.x0 = s.x1 = s.x2 = 0.0f;
    const bool has = p < c.count;
    if (has) {
        KernArgs& A = kargs();  // (kargs: no argument kept live across the loop)
        const size_t b = (size_t)__builtin_amdgcn_readfirstlane(A.idx_in ? A.idx_in[p] : p);
        const int o4 = 4 * c.row;
        if (c.isA) {
            if (c.live) {
                s.x0 = row_ld(A.z, b, c.n, o4);
                gp_l[c.row] = row_ld(A.gP, b, A.ld_gP, o4);
                if (c.fresh && c.use_tol) z_l[c.row] = s.x0;
            }
        } else if (c.live) {
            const float yv = row_ld(A.y, b, c.m, o4);
            s.x0 = yv;
            pd_l[c.row] = (float)(A.gscale * (double)row_ld(A.g, b, A.ld_g, o4));
            s.x1 = c.fresh ? __builtin_fmaf(A.beta[0], yv - yv, yv) : row_ld(A.wc, b, c.m, o4);
            if (c.use_tol && !c.fresh) s.x2 = row_ld(A.uc, b, c.m, o4);
            w_l[c.row] = s.x1;
        }
    }
    __syncthreads();
    if (has && c.fresh && c.use_tol) {  // u = G_L z_{-1}, then the 8c recursion
        if (!c.isA) {
            const float us = chain_regs<KB, K>(r, z_l);
            s.x2 = c.live ? us : 0.0f;
        }
        __syncthreads();  // z_l free again
    }
}

// consume the pre-claimed position of slot s, claim its next one (claim_l: this slot's cell)
template <int KB, int K>
__device__ __forceinline__ void duo_claim(const SolveArgs<float>& a, const DuoCtx& c, DuoSlot& s, int* claim_l,
                                          float* w_l, float* gp_l, float* pd_l, float* z_l,
                                          const float (&r)[K]) {
    const int p = s.nextp;
    if (c.tid == 0 && p < c.count) *claim_l = c.claim_base + atomicAdd(a.qctr, 1);
    duo_refill<KB, K>(a, c, s, p, w_l, gp_l, pd_l, z_l, r);  // (its barrier publishes *claim_l)
    s.nextp = p < c.count ? __builtin_amdgcn_readfirstlane(*claim_l) : c.count;
}

// Step anatomy stamps (diagnostic builds only, -DGPAD_STAMP): shader clock of workgroup 0, every
// wave, steps [kDStep0, kDStep0 + 8) of the workgroup (one step = one duo_step call), at five
// points: step start, chain done (a wave without a chain this step: not stamped), before the
// barrier, after it, step end (gpad_debug_duo_stamps, tools/duo_solo.py --stamps [--two]).
#ifdef GPAD_STAMP
constexpr int kDStep0 = 200;
__device__ unsigned long long g_duo_stamps[8][8][5];
#define GPAD_DSTAMP(P)                                                                              \
    do {                                                                                            \
        if (blockIdx.x == 0 && c.step >= kDStep0 && c.step < kDStep0 + 8 && (c.tid & 63) == 0)     \
            g_duo_stamps[c.tid >> 6][c.step - kDStep0][P] = __builtin_amdgcn_s_memtime();          \
    } while (0)
hipError_t read_duo_stamps(unsigned long long* out, size_t bytes) {
    if (bytes > sizeof(g_duo_stamps)) bytes = sizeof(g_duo_stamps);
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_duo_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#else
#define GPAD_DSTAMP(P) \
    do {               \
    } while (0)
#endif

// The half-steps (every wave calls the one of its role; control flow uniform per role).
// 8b + 8c of slot sa on the -ML waves: zhat to the slot's LDS vector, z updated.
template <int KA, int K>
__device__ __forceinline__ void duo_half_a(const DuoCtx& c, DuoSlot& sa, const float* wa_l, float* zha_l,
                                           const float* gpa_l, const float (&r)[K]) {
    const float th = sa.th;
    const float gpv = gpa_l[c.row];  // read before the chain: its LDS latency hides there
    const float acc = chain_regs<KA, K>(r, wa_l);
    GPAD_DSTAMP(1);
    if (c.live) {
        const float zhv = acc - gpv;
        sa.x0 = __builtin_fmaf(1.0f - th, sa.x0, th * zhv);
        zha_l[c.row] = zhv;
        sa.x1 = zhv;
    }
}

// 8d + 8a (+ the test partials when chk) of slot sb on the G/L waves: w to the slot's LDS vector.
template <int KB, int K>
__device__ __forceinline__ void duo_half_b(const DuoCtx& c, DuoSlot& sb, bool chk, const float* zhb_l, float* wb_l,
                                           const float* pdb_l, CheckSlot* slots_b, const float (&r)[K]) {
    float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
    double gap = 0.0;
    const float th = sb.th, bn = sb.bn;
    const float pdv = pdb_l[c.row];  // (before the chain, as gpv)
    const float cv = chain_regs<KB, K>(r, zhb_l);
    GPAD_DSTAMP(1);
    if (c.live) {
        const float pdi = pdv, wi = sb.x1;
        const float sv = (wi + pdi) + cv;                     // seq_functions.cpp:84
        const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;   // seq_functions.cpp:85
        if (c.use_tol) sb.x2 = __builtin_fmaf(1.0f - th, sb.x2, th * cv);
        if (chk) {
            const float t = cv + pdi;
            violh = t;
            magh = __builtin_fabsf(cv) + __builtin_fabsf(pdi);
            wmin = wi;
            gap = -((double)wi * (double)t);
            violz = sb.x2 + pdi;
        }
        sb.x1 = __builtin_fmaf(bn, yp - sb.x0, yp);
        sb.x0 = yp;
        wb_l[c.row] = sb.x1;
    }
    if (chk) check_publish<float>(slots_b, violz, violh, wmin, gap, magh);
}

// after the barrier that closes slot sb's 8d half (every wave): iteration count, schedule, the
// test's decision, and on termination the results out and the slot refilled from the queue
// PRE: the schedule of the next iteration was fetched ahead (th_n, bn_n; duo_solo), else it is
// loaded here
template <int KB, int K, bool PRE = false>
__device__ __forceinline__ void duo_post_b(const SolveArgs<float>& a, const DuoCtx& c, DuoSlot& sb, bool chk,
                                           float* wb_l, float* gpb_l, float* pdb_l, CheckSlot* slots_b,
                                           CheckSlot* vslots, int* claim_b, float* z_l, const float (&r)[K],
                                           float th_n = 0.0f, float bn_n = 0.0f) {
    sb.need8d = false;
    sb.kc = chk ? c.Kc : sb.kc - 1;
    const int v = ++sb.vs;
    if constexpr (PRE) {
        sb.th = th_n;
        sb.bn = bn_n;
    } else {
        sb.th = sched(a.theta, v);  // next iteration's schedule (tables hold N + 2 entries)
        sb.bn = sched(a.beta, v + 1);
    }
    int done = 0;
    if (chk) {
        const int st1 = check_stage1<float>(slots_b + c.b0, c.nwaves - c.nA, a.L, a.tol, a.tol_gap);
        bool verified = false;
        if (st1 & 1) {  // (A) nominated: decide on the direct chain G_L z, reset u to it
            if (c.isA && c.live) z_l[c.row] = sb.x0;
            __syncthreads();
            float vc = -INFINITY, mc = 0.0f;
            if (!c.isA) {
                const float cz = chain_regs<KB, K>(r, z_l);
                if (c.live) {
                    sb.x2 = cz;
                    vc = cz + pdb_l[c.row];
                    mc = __builtin_fabsf(cz) + __builtin_fabsf(pdb_l[c.row]);
                }
                check_publish<float>(vslots, vc, vc, vc, 0.0, mc);
            }
            __syncthreads();
            verified = check_verify<float>(vslots + c.b0, c.nwaves - c.nA, a.L, a.tol);
        }
        done = check_code(st1, verified);
    }
    if (done || v >= c.N) {
        KernArgs& A = kargs();  // (kargs: no argument kept live across the loop)
        const size_t b = (size_t)__builtin_amdgcn_readfirstlane(A.idx_in ? A.idx_in[sb.pos] : sb.pos);
        if (c.live) {
            if (c.isA) row_st(A.z, b, c.n, 4 * c.row, done == 2 ? sb.x1 : sb.x0);  // (B) certifies zhat
            else row_st(A.y, b, c.m, 4 * c.row, sb.x0);
        }
        if (c.tid == 0) {
            A.iters[b] = v;
            A.conv[b] = done;
        }
        duo_claim<KB, K>(a, c, sb, claim_b, wb_l, gpb_l, pdb_l, z_l, r);
    }
}

#ifdef GPAD_STAMP
#define GPAD_DSTEP() ++const_cast<DuoCtx&>(c).step
#else
#define GPAD_DSTEP() \
    do {             \
    } while (0)
#endif

// one step: -ML waves run 8b+8c of slot sa, G/L waves 8d+8a (+ test) of slot sb
template <int KA, int KB, int K>
__device__ __forceinline__ void duo_step(const SolveArgs<float>& a, const DuoCtx& c, DuoSlot& sa, DuoSlot& sb,
                                         float* wa_l, float* zha_l, const float* gpa_l, float* wb_l,
                                         const float* zhb_l, float* gpb_l, float* pdb_l, CheckSlot* slots_b,
                                         CheckSlot* vslots, int* claim_b, float* z_l, const float (&r)[K]) {
    // the slot bookkeeping is uniform and kept scalar (list positions via readfirstlane): the test
    // period in vector registers cost an integer division per step (profiles/r03_duo_solo.txt)
    const bool runA = sa.pos < c.count && !sa.need8d;
    const bool runB = sb.need8d;
    const bool chk = runB && c.use_tol && sb.kc == 1;  // ((vs + 1) % Kc == 0, as a countdown)
    GPAD_DSTAMP(0);
    if (c.isA) {
        if (runA) duo_half_a<KA, K>(c, sa, wa_l, zha_l, gpa_l, r);
    } else {
        if (runB) duo_half_b<KB, K>(c, sb, chk, zhb_l, wb_l, pdb_l, slots_b, r);
    }
    GPAD_DSTAMP(2);
    __syncthreads();
    GPAD_DSTAMP(3);
    if (runA) sa.need8d = true;
    if (runB) duo_post_b<KB, K>(a, c, sb, chk, wb_l, gpb_l, pdb_l, slots_b, vslots, claim_b, z_l, r);
    GPAD_DSTAMP(4);
    GPAD_DSTEP();
}

// One live slot left, the queue drained (the other slot stays empty: a slot is refilled only when
// its own instance finishes): the live slot runs the resident kernel's loop -- 8b half, barrier,
// 8d half, barrier -- without duo_step's pairing bookkeeping after every barrier (one slot in
// duo_step: 1.76 us per iteration, the resident kernel 1.37, profiles/r03_duo_solo.txt).  The
// same half-step functions, hence the same arithmetic; refills from the queue continue.
template <int KA, int KB, int K>
__device__ __forceinline__ void duo_solo(const SolveArgs<float>& a, const DuoCtx& c, DuoSlot& s, float* w_l,
                                         float* zh_l, float* gp_l, float* pd_l, CheckSlot* slots,
                                         CheckSlot* vslots, int* claim, float* z_l, const float (&r)[K]) {
    // the next iteration's theta / beta by vector loads, each role in its idle half (as the
    // resident kernel): no scalar-load latency in front of the next chain's first LDS read
    float th_n = a.theta[s.vs + 1], bn_n = a.beta[s.vs + 2];
    while (s.pos < c.count) {
        if (!s.need8d) {  // (a slot that enters after its 8b half starts at 8d)
            GPAD_DSTAMP(0);
            if (c.isA) {
                duo_half_a<KA, K>(c, s, w_l, zh_l, gp_l, r);
            } else {
                th_n = a.theta[s.vs + 1];
                bn_n = a.beta[s.vs + 2];
            }
            GPAD_DSTAMP(2);
            __syncthreads();
            GPAD_DSTAMP(3);
            GPAD_DSTAMP(4);
            GPAD_DSTEP();
        }
        const bool chk = c.use_tol && s.kc == 1;
        GPAD_DSTAMP(0);
        if (!c.isA) {
            duo_half_b<KB, K>(c, s, chk, zh_l, w_l, pd_l, slots, r);
        } else {
            th_n = a.theta[s.vs + 1];
            bn_n = a.beta[s.vs + 2];
        }
        GPAD_DSTAMP(2);
        __syncthreads();
        GPAD_DSTAMP(3);
        duo_post_b<KB, K, true>(a, c, s, chk, w_l, gp_l, pd_l, slots, vslots, claim, z_l, r, th_n, bn_n);
        GPAD_DSTAMP(4);
        GPAD_DSTEP();
    }
}

template <int KA, int KB>
__global__ __launch_bounds__(kResidentMaxThreads) void gpad_duo_kernel(SolveArgs<float> a) {
    constexpr int K = KA > KB ? KA : KB;
    constexpr int PA = (KA + 63) / 64 * 64, PB = (KB + 63) / 64 * 64;
    __shared__ __attribute__((aligned(16))) float w_l[2][PA];   // w per slot (broadcast to -ML rows)
    __shared__ __attribute__((aligned(16))) float zh_l[2][PB];  // zhat per slot (to G/L rows)
    __shared__ __attribute__((aligned(16))) float z_l[PB];      // z_{-1} of a fresh instance (u seed)
    __shared__ float gp_l[2][PB];                               // per slot: g_P of the -ML rows
    __shared__ float pd_l[2][PA];                               //           p_D of the G/L rows
    __shared__ CheckSlot slots[2][kResidentMaxThreads / 64];
    __shared__ CheckSlot vslots[kResidentMaxThreads / 64];  // verification of a nominated test (A)
    __shared__ int claim_l[2];

    DuoCtx c;
    c.tid = threadIdx.x;
#ifdef GPAD_STAMP
    c.step = 0;
#endif
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
    c.kc0 = c.Kc - c.v0 % c.Kc;
    c.nA = (c.n + 63) >> 6;
    c.nwaves = blockDim.x >> 6;
    {   // The G/L waves come first, i.e. are the older wave of each SIMD: the SIMD issues oldest
        // first, so their 8d chain finishes first and its longer epilogue (8d, 8a, test partials)
        // overlaps the tail of the -ML chain, whose short 8b/8c epilogue is what is left exposed
        // before the barrier -- two slots 2.46 -> 2.31 us per slot-iteration, C4 -0.7 %
        // (profiles/r03_duo_order_ab.txt).
        const int nB = c.nwaves - c.nA;
        c.isA = (c.tid >> 6) >= nB;
        c.row = c.isA ? c.tid - 64 * nB : c.tid;
        c.b0 = 0;
    }
    c.live = c.isA ? c.row < c.n : c.row < c.m;

    float r[K];
    {
        const int len = c.isA ? c.m : c.n;
        const float* __restrict__ Mt = c.isA ? a.MGt : a.GLt;
        const int ld = c.isA ? a.ldn : a.ldm;
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = (c.live && k < len) ? Mt[(size_t)k * ld + c.row] : 0.0f;
    }
    for (int i = c.tid; i < 2 * PA; i += blockDim.x) (&w_l[0][0])[i] = 0.0f;
    for (int i = c.tid; i < 2 * PB; i += blockDim.x) (&zh_l[0][0])[i] = 0.0f;
    for (int i = c.tid; i < PB; i += blockDim.x) z_l[i] = 0.0f;
    // Static start: slot 0 of workgroup b takes list position b, slot 1 position G + b (the list is
    // sorted longest-predicted-first); later positions are claimed from the counter.
    c.claim_base = 2 * c.G;
    if (c.tid == 0) {  // first claims of the queue (positions 2G, ...)
        claim_l[0] = c.claim_base + atomicAdd(a.qctr, 1);
        claim_l[1] = c.claim_base + atomicAdd(a.qctr, 1);
    }
    __syncthreads();
    DuoSlot s0, s1;
    s0.nextp = __builtin_amdgcn_readfirstlane(claim_l[0]);
    s1.nextp = __builtin_amdgcn_readfirstlane(claim_l[1]);
    duo_refill<KB, K>(a, c, s0, blockIdx.x, w_l[0], gp_l[0], pd_l[0], z_l, r);
    duo_refill<KB, K>(a, c, s1, blockIdx.x + c.G, w_l[1], gp_l[1], pd_l[1], z_l, r);
    while (s0.pos < c.count || s1.pos < c.count) {
        if (s0.pos >= c.count) {
            duo_solo<KA, KB, K>(a, c, s1, w_l[1], zh_l[1], gp_l[1], pd_l[1], slots[1], vslots, &claim_l[1], z_l, r);
            break;
        }
        if (s1.pos >= c.count) {
            duo_solo<KA, KB, K>(a, c, s0, w_l[0], zh_l[0], gp_l[0], pd_l[0], slots[0], vslots, &claim_l[0], z_l, r);
            break;
        }
        duo_step<KA, KB, K>(a, c, s0, s1, w_l[0], zh_l[0], gp_l[0], w_l[1], zh_l[1], gp_l[1], pd_l[1], slots[1],
                            vslots, &claim_l[1], z_l, r);
        duo_step<KA, KB, K>(a, c, s1, s0, w_l[1], zh_l[1], gp_l[1], w_l[0], zh_l[0], gp_l[0], pd_l[0], slots[0],
                            vslots, &claim_l[0], z_l, r);
    }
}

template <int KA>
static void launch_duo_b(int kb, dim3 g, dim3 bl, hipStream_t st, const SolveArgs<float>& a) {
    switch (kb) {
        case 32: hipLaunchKernelGGL((gpad_duo_kernel<KA, 32>), g, bl, 0, st, a); break;
        case 64: hipLaunchKernelGGL((gpad_duo_kernel<KA, 64>), g, bl, 0, st, a); break;
        case 96: hipLaunchKernelGGL((gpad_duo_kernel<KA, 96>), g, bl, 0, st, a); break;
        case 128: hipLaunchKernelGGL((gpad_duo_kernel<KA, 128>), g, bl, 0, st, a); break;
        case 160: hipLaunchKernelGGL((gpad_duo_kernel<KA, 160>), g, bl, 0, st, a); break;
        case 192: hipLaunchKernelGGL((gpad_duo_kernel<KA, 192>), g, bl, 0, st, a); break;
        case 200: hipLaunchKernelGGL((gpad_duo_kernel<KA, 200>), g, bl, 0, st, a); break;
        default: hipLaunchKernelGGL((gpad_duo_kernel<KA, 208>), g, bl, 0, st, a); break;
    }
}

hipError_t launch_duo(const SolveArgs<float>& a, int grid, hipStream_t st) {
    if (!resident_supported(a.n, a.m) || a.strideA || a.strideB || !a.qctr || grid < 1)
        return hipErrorInvalidValue;
    const int threads = 64 * (((a.n + 63) >> 6) + ((a.m + 63) >> 6));
    const dim3 g(grid), bl(threads);
    const int ka = res_bucket(a.m), kb = res_bucket(a.n);
    switch (ka) {
        case 32: launch_duo_b<32>(kb, g, bl, st, a); break;
        case 64: launch_duo_b<64>(kb, g, bl, st, a); break;
        case 96: launch_duo_b<96>(kb, g, bl, st, a); break;
        case 128: launch_duo_b<128>(kb, g, bl, st, a); break;
        case 160: launch_duo_b<160>(kb, g, bl, st, a); break;
        case 192: launch_duo_b<192>(kb, g, bl, st, a); break;
        case 200: launch_duo_b<200>(kb, g, bl, st, a); break;
        default: launch_duo_b<208>(kb, g, bl, st, a); break;
    }
    return hipGetLastError();
}


}  // namespace gpad
