// split_kernel.hip -- EXPERIMENT, not in the product (was csrc/gpad_split.hip in round 2; builds
// only against the round-2 csrc/ headers).  A single-instance latency kernel with split dot
// products (NOT bit-exact; tests passed at 1e-6 relative).  Measured on MI355X
// (profiles/r02_split_kernel_bench.json): C2 7.5e5 it/s vs the bit-exact resident kernel's
// 8.6e5 -- the LDS-broadcast plain chains run at ~12 cycles per step (LDS latency, as the
// lds-bcast rows of profiles/r01_dpp_chain.txt), not the 5.9 of a register-operand chain, so the
// plain half is the slower one; see DESIGN.md §5a.
//
// The bit-exact resident kernel (gpad_kernels.hip) keeps one matrix row per lane and runs each
// row's dot product as ONE sequential fmaf chain -- the reference's order (seq_functions.cpp:61,
// 82) -- so an iteration is 2 x K dependent `v_fmac_f32_dpp` steps on one wave per SIMD:
// ~5.9 cycles each, 1.18 us per iteration at C2 (n = m = 200).  The DPP broadcast is a per-SIMD
// issue resource (a second DPP wave on the SIMD doubles its step time, profiles/r01_dpp_chain.txt),
// but a DPP chain and a plain-operand chain on the same SIMD run side by side at 6.3 cycles each.
//
// Here every row's chain is split in two at k = K0 (a multiple of 8):
//   waves 0..3 ("DPP waves"):   k <  K0, the register-resident DPP chain of the resident kernel;
//   waves 4..7 ("plain waves"): k >= K0, plain v_fmac_f32 whose operand is the vector element
//                               read by every lane from the same LDS address (one ds_read_b128
//                               per 4 steps, a broadcast: no bank conflict).
// Waves w and w + 4 share a SIMD (cyclic wave placement), so each SIMD runs one chain of each kind
// concurrently: ~K/2 steps per half-iteration instead of K.  Every lane holds BOTH its primal row
// part (-ML, 8b) and its constraint row part (G/L, 8d) in VGPRs -- 8 waves, up to 256 registers
// each -- so all eight waves work in both halves of the iteration.  The plain part's partial sum
// reaches the DPP lane that owns the row through LDS, and the DPP lane finishes the row:
//   c = dpp_part + plain_part  (fixed order), then the resident kernel's epilogues verbatim.
// Summation order: ((a_0 b_0 + ... + a_{K0-1} b_{K0-1}) + (a_{K0} b_{K0} + ... + a_{K-1} b_{K-1})),
// each parenthesis an fmaf chain from +0 -- one reassociation per dot product.
// Algorithm 1 as everywhere (gpad_chain.h check_stage1/check_verify; the direct G_L z of a
// nominated test (A) is the same split chain over z).
#include <hip/hip_runtime.h>

#include <cmath>

#include "gpad_chain.h"
#include "gpad_internal.h"

namespace gpad {

constexpr int kSplitWaves = 8;  // 4 DPP + 4 plain; rows <= 256
constexpr int kSplitThreads = 64 * kSplitWaves;

// acc = sum_{k < KLEN} r[k] * v[k] in ascending k, v broadcast from LDS (same address in every
// lane), two float4 in flight.
template <int KLEN, int K>
__device__ __forceinline__ float plain_chain(const float (&r)[K], const float* v) {
    static_assert(KLEN % 4 == 0 && KLEN <= K, "bad plain chain length");
    constexpr int NQ = KLEN / 4;
    float acc = 0.0f;
    float4 c0 = *reinterpret_cast<const float4*>(v);
    float4 c1 = NQ > 1 ? *reinterpret_cast<const float4*>(v + 4) : c0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const float4 c = (q & 1) ? c1 : c0;
        float4 nx = c;
        if (q + 2 < NQ) nx = *reinterpret_cast<const float4*>(v + 4 * (q + 2));
        acc = __builtin_fmaf(r[4 * q + 0], c.x, acc);
        acc = __builtin_fmaf(r[4 * q + 1], c.y, acc);
        acc = __builtin_fmaf(r[4 * q + 2], c.z, acc);
        acc = __builtin_fmaf(r[4 * q + 3], c.w, acc);
        if (q & 1) c1 = nx;
        else c0 = nx;
        asm volatile("" : "+v"(acc) : : "memory");  // bounds the read-ahead to two float4
    }
    return acc;
}

// one role's part of a row's dot product: DPP waves k < K0, plain waves K0 <= k < K0 + K1
template <int K0, int K1, int K, bool DPP>
__device__ __forceinline__ float part_chain(const float (&r)[K], const float* v) {
    if constexpr (DPP) return chain_regs<K0, K>(r, v);
    else return plain_chain<K1, K>(r, v + K0);
}

struct SplitLds {
    float* w_l;        // w (broadcast to the 8b chains)
    float* zh_l;       // zhat (8d chains); z for the u seed and the test's direct G_L z
    float* part;       // [256] the plain waves' partial sums per row
    CheckSlot* slots;  // [2][kSplitWaves]: the test's partials, the verification of (A)
};

// One role's whole solve (DPP = waves 0..3, the row owners; else the plain waves).  Each role is
// its own instantiation (the two chain codes do not share one register allocation); both execute
// the same sequence of barriers.
template <bool DPP, int KA0, int KA1, int KB0, int KB1>
__device__ __forceinline__ void split_run(const SolveArgs<float>& a, const SplitLds& L) {
    constexpr int KA = DPP ? KA0 : KA1, KB = DPP ? KB0 : KB1;
    constexpr int PA = (KA0 + KA1 + 63) / 64 * 64 + 64, PB = (KB0 + KB1 + 63) / 64 * 64 + 64;
    const int tid = threadIdx.x;
    const int row = 64 * ((tid >> 6) & 3) + (tid & 63);
    const int b = blockIdx.x;
    const int n = a.n, m = a.m;
    const bool liveA = row < n, liveB = row < m;
    float rA[KA], rB[KB];
    {
        const float* __restrict__ Mt = a.MGt + (size_t)b * a.strideA;
        const float* __restrict__ Gt = a.GLt + (size_t)b * a.strideB;
        constexpr int ka0 = DPP ? 0 : KA0, kb0 = DPP ? 0 : KB0;
#pragma unroll
        for (int k = 0; k < KA; ++k) rA[k] = (liveA && ka0 + k < m) ? Mt[(size_t)(ka0 + k) * a.ldn + row] : 0.0f;
#pragma unroll
        for (int k = 0; k < KB; ++k) rB[k] = (liveB && kb0 + k < n) ? Gt[(size_t)(kb0 + k) * a.ldm + row] : 0.0f;
    }
    float* zg = a.z + (size_t)b * n;
    float* yg = a.y + (size_t)b * m;
    float zi = 0.0f, gpi = 0.0f, yi = 0.0f, pdi = 0.0f, wi = 0.0f, ui = 0.0f, zhi = 0.0f;  // DPP lanes
    if constexpr (DPP) {
        if (liveA) {
            zi = zg[row];
            gpi = a.gP[(size_t)b * a.ld_gP + row];
        }
        if (liveB) {
            yi = yg[row];
            pdi = (float)(a.gscale * (double)a.g[(size_t)b * a.ld_g + row]);
            wi = __builtin_fmaf(a.beta[0], yi - yi, yi);
        }
    }
    for (int i = tid; i < PA; i += kSplitThreads) L.w_l[i] = 0.0f;
    for (int i = tid; i < PB; i += kSplitThreads) L.zh_l[i] = 0.0f;
    __syncthreads();
    if (DPP && liveB) L.w_l[row] = wi;
    if (DPP && liveA) L.zh_l[row] = zi;  // z_{-1}: the u seed below
    __syncthreads();
    const bool use_tol = a.tol > 0.0;
    if (use_tol) {  // u = G_L z_{-1}, then the 8c recursion (the row's DPP lane adds both parts)
        const float pc = part_chain<KB0, KB1, KB, DPP>(rB, L.zh_l);
        if (!DPP) L.part[row] = pc;
        __syncthreads();
        if (DPP) ui = pc + L.part[row];
        __syncthreads();  // part[] and zh_l are rewritten below
    }
    // The 8d chain code appears once: a nominated test (A) re-enters the loop in "verify" mode,
    // which runs that same chain over z (in zh_l) instead of a new iteration (a second inlined
    // copy of the register-resident chain made the compiler spill the rows).
    int it = 0, done = 0, v = 0, st1 = 0;
    bool verify = false;
    float th = a.theta[0], bn = a.beta[1];
    while (v < a.N) {
        const float th_next = a.theta[v + 1], bn_next = a.beta[v + 2];
        const bool chk = !verify && use_tol && ((v + 1) % a.check_every) == 0;
        // ---- 8b + 8c --------------------------------------------------------------------
        if (!verify) {
            const float pc = part_chain<KA0, KA1, KA, DPP>(rA, L.w_l);
            if (!DPP) L.part[row] = pc;
            __syncthreads();
            if (DPP && liveA) {
                const float acc = pc + L.part[row];
                const float zhv = acc - gpi;
                zi = __builtin_fmaf(1.0f - th, zi, th * zhv);
                L.zh_l[row] = zhv;
                zhi = zhv;
            }
            __syncthreads();
        }
        // ---- 8d + next 8a (or, in verify mode, G_L z for test (A)) -------------------------
        float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
        double gap = 0.0;
        const float pc = part_chain<KB0, KB1, KB, DPP>(rB, L.zh_l);
        if (!DPP) L.part[row] = pc;
        __syncthreads();
        if (verify) {  // decide (A) on the direct split chain G_L z, reset u to it
            if (DPP && liveB) {
                const float c = pc + L.part[row];
                ui = c;
                violz = c + pdi;
                magh = __builtin_fabsf(c) + __builtin_fabsf(pdi);
            }
            check_publish<float>(L.slots + kSplitWaves, violz, violz, violz, 0.0, magh);
            __syncthreads();
            done = check_code(st1, check_verify<float>(L.slots + kSplitWaves, kSplitWaves, a.L, a.tol));
            verify = false;
            if (done) break;
            continue;
        }
        if (DPP && liveB) {
            const float c = pc + L.part[row];
            const float sv = (wi + pdi) + c;
            const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;
            if (use_tol) ui = __builtin_fmaf(1.0f - th, ui, th * c);
            if (chk) {
                const float t = c + pdi;
                violh = t;
                magh = __builtin_fabsf(c) + __builtin_fabsf(pdi);
                wmin = wi;
                gap = -((double)wi * (double)t);
                violz = ui + pdi;
            }
            wi = __builtin_fmaf(bn, yp - yi, yp);
            yi = yp;
            L.w_l[row] = wi;
        }
        if (chk) check_publish<float>(L.slots, violz, violh, wmin, gap, magh);
        __syncthreads();
        it = ++v;
        th = th_next;
        bn = bn_next;
        if (chk) {
            st1 = check_stage1<float>(L.slots, kSplitWaves, a.L, a.tol, a.tol_gap);
            if (st1 & 1) {  // (A) nominated: z into zh_l, then the verify pass
                if (DPP && liveA) L.zh_l[row] = zi;
                __syncthreads();
                verify = true;
                continue;
            }
            done = check_code(st1, false);
            if (done) break;
        }
    }
    if constexpr (DPP) {
        if (liveA) zg[row] = done == 2 ? zhi : zi;  // test (B) certifies zhat
        if (liveB) yg[row] = yi;
        if (tid == 0) {
            a.iters[b] = it;
            a.conv[b] = done;
        }
    }
}

template <int KA0, int KA1, int KB0, int KB1>
__global__ __launch_bounds__(kSplitThreads) void gpad_split_kernel(SolveArgs<float> a) {
    constexpr int PA = (KA0 + KA1 + 63) / 64 * 64 + 64, PB = (KB0 + KB1 + 63) / 64 * 64 + 64;
    __shared__ __attribute__((aligned(16))) float w_l[PA];
    __shared__ __attribute__((aligned(16))) float zh_l[PB];
    __shared__ float part[256];
    __shared__ CheckSlot slots[2 * kSplitWaves];
    const SplitLds L{w_l, zh_l, part, slots};
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < 4)
        split_run<true, KA0, KA1, KB0, KB1>(a, L);
    else
        split_run<false, KA0, KA1, KB0, KB1>(a, L);
}

// Chain-length buckets of one row (the resident kernel's) split near the middle at a multiple of
// 8: the 8b chain's DPP part rounded down, the 8d chain's rounded up, so a DPP lane (8b DPP part +
// 8d DPP part) and a plain lane (the two plain parts) hold the same number of row registers
// (C2: 96 + 104 = 104 + 96 = 200 of the 256 a lane has at two waves per SIMD).
template <int KT>
static hipError_t launch_split_b(int kbt, dim3 g, hipStream_t st, const SolveArgs<float>& a) {
    constexpr int KA0 = (KT / 2) / 8 * 8, KA1 = KT - KA0;
#define SPLIT_B(KBT)                                                                                  \
    case KBT:                                                                                         \
        hipLaunchKernelGGL((gpad_split_kernel<KA0, KA1, ((KBT / 2) + 7) / 8 * 8, KBT - ((KBT / 2) + 7) / 8 * 8>), g, \
                           dim3(kSplitThreads), 0, st, a);                                            \
        break;
    switch (kbt) {
        SPLIT_B(32) SPLIT_B(64) SPLIT_B(96) SPLIT_B(128) SPLIT_B(160) SPLIT_B(192) SPLIT_B(200)
        default: SPLIT_B(208)
    }
#undef SPLIT_B
    return hipGetLastError();
}

bool split_supported(int n, int m) { return n > 0 && m > 0 && n <= kResidentMaxRow && m <= kResidentMaxRow; }

hipError_t launch_split(const SolveArgs<float>& a, hipStream_t st) {
    if (!split_supported(a.n, a.m)) return hipErrorInvalidValue;
    const dim3 g(a.batch);
    const int kat = res_bucket(a.m), kbt = res_bucket(a.n);  // 8b chains run over m, 8d over n
    switch (kat) {
        case 32: return launch_split_b<32>(kbt, g, st, a);
        case 64: return launch_split_b<64>(kbt, g, st, a);
        case 96: return launch_split_b<96>(kbt, g, st, a);
        case 128: return launch_split_b<128>(kbt, g, st, a);
        case 160: return launch_split_b<160>(kbt, g, st, a);
        case 192: return launch_split_b<192>(kbt, g, st, a);
        case 200: return launch_split_b<200>(kbt, g, st, a);
        default: return launch_split_b<208>(kbt, g, st, a);
    }
}

}  // namespace gpad
