// gpad_chain.h -- device helpers shared by the latency kernels (gpad_kernels.hip: stream and
// resident kernels; gpad_duo.hip: the two-instance ping-pong kernel): fused-arithmetic wrappers,
// wave64 reductions and the Algorithm-1 test slots, and the register-resident DPP fmaf chains.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <utility>

#include "gpad_internal.h"

namespace gpad {

__device__ __forceinline__ float fmad(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float absd(float a) { return __builtin_fabsf(a); }
__device__ __forceinline__ double absd(double a) { return __builtin_fabs(a); }
template <typename T> __device__ __forceinline__ T neg_inf();
template <> __device__ __forceinline__ float neg_inf<float>() { return -INFINITY; }
template <> __device__ __forceinline__ double neg_inf<double>() { return -INFINITY; }

template <typename T> struct V4;
template <> struct V4<float> { using type = float4; };
template <> struct V4<double> { using type = double4; };

// ---- wave64 reductions (DPP/permute lowered by the compiler) ---------------------------
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Per-wave partials of the Algorithm-1 test -> LDS slot of the wave.
//   violz: max(u + pD) (recursive G_L z, nominates test A)   violh: max(G_L zhat + pD)
//   magh:  max(|G_L zhat| + |pD|) (test B's rounding scale)  wmin, gap: test B's other terms
// The verification of a nominated test A publishes max(G_L z + pD) in violz and
// max(|G_L z| + |pD|) in magh of a second slot array.
struct CheckSlot {
    double violz, violh, wmin, gap, magh;
};

template <typename T>
__device__ __forceinline__ void check_publish(CheckSlot* slots, T violz, T violh, T wmin,
                                              double gap, T magh) {
    const T a = wave_max(violz), b = wave_max(violh), c = wave_min(wmin), e = wave_max(magh);
    const double d = wave_sum(gap);
    if ((threadIdx.x & 63) == 0) {
        CheckSlot& s = slots[threadIdx.x >> 6];
        s.violz = (double)a;
        s.violh = (double)b;
        s.wmin = (double)c;
        s.gap = d;
        s.magh = (double)e;
    }
}

// Every thread evaluates the decision from the same LDS words -> uniform, no extra barrier.
// Returns bit 1: test (A) nominated by the recursion (L*max(u + pD) <= tol; decided later on
// the direct G_L z by check_verify), bit 2: test (B) passed
//   L*max(G_L zhat + pD) + margin L*max(|G_L zhat| + |pD|) <= tol, w >= 0, -L w't <= tol_gap.
template <typename T>
__device__ __forceinline__ int check_stage1(const CheckSlot* slots, int nwaves, double L, double tol,
                                            double tol_gap) {
    double vz = -INFINITY, vh = -INFINITY, wm = INFINITY, gap = 0.0, mh = 0.0;
    for (int i = 0; i < nwaves; ++i) {
        vz = fmax(vz, slots[i].violz);
        vh = fmax(vh, slots[i].violh);
        wm = fmin(wm, slots[i].wmin);
        gap += slots[i].gap;
        mh = fmax(mh, slots[i].magh);
    }
    const bool a = vz * L <= tol;
    const bool b = viol_ok(vh, mh, L, tol, ViolMargin<T>::value) && (wm >= 0.0) && (gap * L <= tol_gap);
    return (a ? 1 : 0) | (b ? 2 : 0);
}

// Test (A) on the direct chain c = G_L z: slots hold max(c + pD) in violz, max(|c| + |pD|) in magh.
template <typename T>
__device__ __forceinline__ bool check_verify(const CheckSlot* slots, int nwaves, double L, double tol) {
    double vc = -INFINITY, mc = 0.0;
    for (int i = 0; i < nwaves; ++i) {
        vc = fmax(vc, slots[i].violz);
        mc = fmax(mc, slots[i].magh);
    }
    return viol_ok(vc, mc, L, tol, ViolMargin<T>::value);
}

// final code from the two stages: 1 = (A) verified, 2 = (B), 0 = continue
__device__ __forceinline__ int check_code(int stage1, bool verified) {
    return ((stage1 & 1) && verified) ? 1 : ((stage1 & 2) ? 2 : 0);
}

// =========================================================================================
// register-resident DPP chains (gpad_resident_kernel, gpad_duo_kernel): one matrix row per
// lane, held in VGPRs for the whole solve.
// =========================================================================================
// Register-resident rows.  A lane owning primal row i keeps -ML[i][0..KA) (zero-padded past m);
// a lane owning constraint row i keeps G_L[i][0..KB) (zero-padded past n).  Both roles use the
// same register array r[] (they live in different waves).  KA/KB are compile-time, so the
// chains carry no per-step predicates: padded steps are fma(0, 0, acc) = acc.
//
// The broadcast vector reaches the lanes through DPP, not through LDS bandwidth: each 16-lane
// row of the wave reads the same 64 consecutive elements (lane l: a float4 at 4*(l & 15)), and
// step k of the chain is `v_fmac_f32_dpp acc, w4[k%4], r[k] row_newbcast:(k%64)/4` -- the
// element is broadcast from lane (k%64)/4 of each row inside the FMA itself.  A wave thus reads
// 64 elements per ds_read_b128 with 16 distinct addresses (a same-address float4 per 4 steps,
// all 64 lanes, made the chains LDS-bandwidth bound: ~10 cycles per step with four waves).
// v_fmac_f32 is a single-rounding fused multiply-add, so the chain is still exactly the
// reference's sequential fmaf order.  One 64-element group is prefetched ahead; an empty asm
// that reads/writes acc and clobbers memory closes each group (bounds the prefetch, pins the
// chain in place).  The first use of each ring register in a group carries `s_nop 1`: a DPP
// read 2 wait states after a VALU write of its source (only if the compiler ever copies a ring
// value with a VALU move; the inline asm hides the DPP from the hazard recognizer).
// 16 steps per asm statement (the compiler separates inline-asm statements with a wait state,
// so few, long statements keep the chain issue-bound).  Steps KI..KI+15 are elements
// 16J..16J+15 of the current 64-element group: lanes 4J..4J+3 of each row, components x..w.
#define GPAD_FMAC(SRC, R, LANE) \
    "v_fmac_f32_dpp %0, %" #SRC ", %" #R " row_newbcast:%" #LANE " row_mask:0xf bank_mask:0xf\n\t"
#define GPAD_FMAC8                                                                             \
    GPAD_FMAC(1, 5, 21) GPAD_FMAC(2, 6, 21) GPAD_FMAC(3, 7, 21) GPAD_FMAC(4, 8, 21)             \
    GPAD_FMAC(1, 9, 22) GPAD_FMAC(2, 10, 22) GPAD_FMAC(3, 11, 22) GPAD_FMAC(4, 12, 22)
#define GPAD_FMAC16                                                                            \
    GPAD_FMAC8                                                                                 \
    GPAD_FMAC(1, 13, 23) GPAD_FMAC(2, 14, 23) GPAD_FMAC(3, 15, 23) GPAD_FMAC(4, 16, 23)         \
    GPAD_FMAC(1, 17, 24) GPAD_FMAC(2, 18, 24) GPAD_FMAC(3, 19, 24) GPAD_FMAC(4, 20, 24)

// a chain length that is 8 mod 16 (the 200 bucket) ends with an 8-step statement
#define GPAD_FMAC8T                                                                            \
    GPAD_FMAC(1, 5, 13) GPAD_FMAC(2, 6, 13) GPAD_FMAC(3, 7, 13) GPAD_FMAC(4, 8, 13)             \
    GPAD_FMAC(1, 9, 14) GPAD_FMAC(2, 10, 14) GPAD_FMAC(3, 11, 14) GPAD_FMAC(4, 12, 14)
template <int KLEN, int K, int KI, int J>
__device__ __forceinline__ void chain_step16(float& acc, const float4& c, const float (&r)[K]) {
    static_assert(KLEN % 8 == 0, "chain lengths are multiples of 8");
    if constexpr (KI + 8 == KLEN) {
#define GPAD_OPS8                                                                                 \
    : "+v"(acc)                                                                                   \
    : "v"(c.x), "v"(c.y), "v"(c.z), "v"(c.w), "v"(r[KI + 0]), "v"(r[KI + 1]), "v"(r[KI + 2]),     \
      "v"(r[KI + 3]), "v"(r[KI + 4]), "v"(r[KI + 5]), "v"(r[KI + 6]), "v"(r[KI + 7]), "i"(4 * J),  \
      "i"(4 * J + 1)
        if constexpr (J == 0)
            asm("s_nop 1\n\t" GPAD_FMAC8T GPAD_OPS8);
        else
            asm(GPAD_FMAC8T GPAD_OPS8);
#undef GPAD_OPS8
    } else if constexpr (KI < KLEN) {
#define GPAD_OPS                                                                                  \
    : "+v"(acc)                                                                                   \
    : "v"(c.x), "v"(c.y), "v"(c.z), "v"(c.w), "v"(r[KI + 0]), "v"(r[KI + 1]), "v"(r[KI + 2]),     \
      "v"(r[KI + 3]), "v"(r[KI + 4]), "v"(r[KI + 5]), "v"(r[KI + 6]), "v"(r[KI + 7]),             \
      "v"(r[KI + 8]), "v"(r[KI + 9]), "v"(r[KI + 10]), "v"(r[KI + 11]), "v"(r[KI + 12]),          \
      "v"(r[KI + 13]), "v"(r[KI + 14]), "v"(r[KI + 15]), "i"(4 * J), "i"(4 * J + 1),              \
      "i"(4 * J + 2), "i"(4 * J + 3)
        if constexpr (J == 0)
            asm("s_nop 1\n\t" GPAD_FMAC16 GPAD_OPS);
        else
            asm(GPAD_FMAC16 GPAD_OPS);
#undef GPAD_OPS
    }
}
#undef GPAD_FMAC16
#undef GPAD_FMAC8
#undef GPAD_FMAC8T
#undef GPAD_FMAC

template <int KLEN, int K, int BASE, int... J>
__device__ __forceinline__ void chain_group(float& acc, const float4& c, const float (&r)[K],
                                            std::integer_sequence<int, J...>) {
    (chain_step16<KLEN, K, BASE + 16 * J, J>(acc, c, r), ...);
}

template <int KLEN, int K, int H>
__device__ __forceinline__ void chain_groups(float& acc, float4 (&ring)[2], const float (&r)[K],
                                             const float* v, int q) {
    constexpr int NH = (KLEN + 63) / 64;
    if constexpr (H < NH) {
        if constexpr (H + 1 < NH) ring[(H + 1) & 1] = *reinterpret_cast<const float4*>(v + 64 * (H + 1) + q);
        chain_group<KLEN, K, 64 * H>(acc, ring[H & 1], r, std::make_integer_sequence<int, 4>{});
        asm volatile("" : "+v"(acc) : : "memory");
        chain_groups<KLEN, K, H + 1>(acc, ring, r, v, q);
    }
}

// acc = sum_k r[k] * v[k], k = 0..KLEN-1, as one fmaf chain in ascending k.  v: LDS, padded to a
// multiple of 64 elements (the last group's float4 reads may run past KLEN).
template <int KLEN, int K>
__device__ __forceinline__ float chain_regs(const float (&r)[K], const float* v) {
    static_assert(KLEN % 4 == 0 && KLEN <= K, "bad chain length");
    const int q = 4 * (threadIdx.x & 15);
    float4 ring[2];
    ring[0] = *reinterpret_cast<const float4*>(v + q);
    float acc = 0.0f;
    chain_groups<KLEN, K, 0>(acc, ring, r, v, q);
    return acc;
}

constexpr int kResidentMaxThreads = 512;
constexpr int kResidentMaxRow = 208;

// chain-length buckets (multiples of 32 up to 192, then 200 and the 208 cap)
inline int res_bucket(int len) {
    if (len > 200) return 208;
    if (len > 192) return 200;
    return (len + 31) / 32 * 32;
}

}  // namespace gpad
