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

// ---- wave64 butterflies on the VALU ------------------------------------------------------
// __shfl_xor lowers to ds_bpermute: an LDS round trip per level, and with the latency kernels'
// register-resident rows leaving few VGPRs the levels of the test's five reductions serialize
// (~40 dependent permutes per Algorithm-1 test).  The same butterfly partners without LDS:
// xor 32 / 16 by gfx950's v_permlane32_swap / v_permlane16_swap, xor 8 by DPP row_ror:8, xor 4
// by DPP row_shl:4 into banks 0, 2 and row_shr:4 into banks 1, 3, xor 2 / 1 by DPP quad_perm.
// Each level combines the same two partials as the __shfl_xor butterfly (op(own, partner), op
// commutative), so sums are bit-identical to it and every lane ends with the same value.
template <int O>
__device__ __forceinline__ unsigned bfly_u32(unsigned x) {
    if constexpr (O == 8) return __builtin_amdgcn_update_dpp(x, x, 0x128, 0xf, 0xf, false);  // row_ror:8
    if constexpr (O == 4) {
        const unsigned t = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xf, 0x5, false);      // row_shl:4
        return __builtin_amdgcn_update_dpp(t, x, 0x114, 0xf, 0xa, false);                 // row_shr:4
    }
    if constexpr (O == 2) return __builtin_amdgcn_update_dpp(x, x, 0x4e, 0xf, 0xf, false);  // [2,3,0,1]
    if constexpr (O == 1) return __builtin_amdgcn_update_dpp(x, x, 0xb1, 0xf, 0xf, false);  // [1,0,3,2]
    static_assert(O == 1 || O == 2 || O == 4 || O == 8, "DPP levels");
    return x;
}
// one butterfly level of op: lanes l and l ^ O both get op(v_l, v_(l^O))
template <int O, typename Op>
__device__ __forceinline__ float bfly(float v, Op op) {
    const unsigned x = __float_as_uint(v);
    if constexpr (O == 32 || O == 16) {
        const auto r = O == 32 ? __builtin_amdgcn_permlane32_swap(x, x, false, false)
                               : __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return op(__uint_as_float(r[0]), __uint_as_float(r[1]));  // (own, partner) in either order
    } else {
        return op(v, __uint_as_float(bfly_u32<O>(x)));
    }
}
template <int O, typename Op>
__device__ __forceinline__ double bfly(double v, Op op) {
    const unsigned long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    if constexpr (O == 32 || O == 16) {
        const auto rl = O == 32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                                : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto rh = O == 32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                                : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        const double a = __longlong_as_double((long long)(((unsigned long long)rh[0] << 32) | rl[0]));
        const double c = __longlong_as_double((long long)(((unsigned long long)rh[1] << 32) | rl[1]));
        return op(a, c);
    } else {
        const unsigned pl = bfly_u32<O>(lo), ph = bfly_u32<O>(hi);
        return op(v, __longlong_as_double((long long)(((unsigned long long)ph << 32) | pl)));
    }
}
template <typename T, typename Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {  // levels 32, 16, ..., 1 (the shfl_xor order)
    v = bfly<32>(v, op);
    v = bfly<16>(v, op);
    v = bfly<8>(v, op);
    v = bfly<4>(v, op);
    v = bfly<2>(v, op);
    return bfly<1>(v, op);
}
struct OpMax { template <typename T> __device__ T operator()(T a, T b) const { return fmax(a, b); } };
struct OpMin { template <typename T> __device__ T operator()(T a, T b) const { return fmin(a, b); } };
struct OpAdd { template <typename T> __device__ T operator()(T a, T b) const { return a + b; } };
template <typename T>
__device__ __forceinline__ T wave_max(T v) { return wave_reduce(v, OpMax{}); }
template <typename T>
__device__ __forceinline__ T wave_min(T v) { return wave_reduce(v, OpMin{}); }
__device__ __forceinline__ double wave_sum(double v) { return wave_reduce(v, OpAdd{}); }

// max / min over lanes 0..7 (the test slots of up to 8 waves, one per lane)
template <typename Op>
__device__ __forceinline__ double lanes8_reduce(double v, Op op) {
    v = bfly<1>(v, op);
    v = bfly<2>(v, op);
    return bfly<4>(v, op);
}
__device__ __forceinline__ double lane_read(double v, int l) {  // lane l's value, wave-uniform
    const unsigned long long b = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
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
// Lane i < nwaves (<= 8) reads slot i -- one LDS round trip instead of one per slot -- the maxima
// and minima meet over lanes 0..7 by DPP (order-free), and the fp64 gap is summed in wave order
// (((0 + g_0) + g_1) + ...) from lane reads, as the sequential loop summed it.
// Returns bit 1: test (A) nominated by the recursion (L*max(u + pD) <= tol; decided later on
// the direct G_L z by check_verify), bit 2: test (B) passed
//   L*max(G_L zhat + pD) + margin L*max(|G_L zhat| + |pD|) <= tol, w >= 0, -L w't <= tol_gap.
template <typename T>
__device__ __forceinline__ int check_stage1(const CheckSlot* slots, int nwaves, double L, double tol,
                                            double tol_gap) {
    const int lane = threadIdx.x & 63;
    const bool own = lane < nwaves;
    double vz = own ? slots[lane].violz : -INFINITY, vh = own ? slots[lane].violh : -INFINITY;
    double wm = own ? slots[lane].wmin : INFINITY, mh = own ? slots[lane].magh : 0.0;
    const double g = own ? slots[lane].gap : 0.0;
    // (folded into the loop's initial values, so an all-NaN column reduces as the loop did)
    vz = fmax(-INFINITY, lane_read(lanes8_reduce(vz, OpMax{}), 0));
    vh = fmax(-INFINITY, lane_read(lanes8_reduce(vh, OpMax{}), 0));
    mh = fmax(0.0, lane_read(lanes8_reduce(mh, OpMax{}), 0));
    wm = fmin(INFINITY, lane_read(lanes8_reduce(wm, OpMin{}), 0));
    double gap = 0.0;
    for (int i = 0; i < nwaves; ++i) gap += lane_read(g, i);
    const bool a = vz * L <= tol;
    const bool b = viol_ok(vh, mh, L, tol, ViolMargin<T>::value) && (wm >= 0.0) && (gap * L <= tol_gap);
    return (a ? 1 : 0) | (b ? 2 : 0);
}

// Test (A) on the direct chain c = G_L z: slots hold max(c + pD) in violz, max(|c| + |pD|) in magh.
template <typename T>
__device__ __forceinline__ bool check_verify(const CheckSlot* slots, int nwaves, double L, double tol) {
    const int lane = threadIdx.x & 63;
    const bool own = lane < nwaves;
    const double vc = fmax(-INFINITY, lane_read(lanes8_reduce(own ? slots[lane].violz : -INFINITY, OpMax{}), 0));
    const double mc = fmax(0.0, lane_read(lanes8_reduce(own ? slots[lane].magh : 0.0, OpMax{}), 0));
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
static_assert(kResidentMaxThreads / 64 <= 8, "check_stage1 / check_verify reduce one slot per lane over lanes 0..7");
constexpr int kResidentMaxRow = 208;

// chain-length buckets (multiples of 32 up to 192, then 200 and the 208 cap)
inline int res_bucket(int len) {
    if (len > 200) return 208;
    if (len > 192) return 200;
    return (len + 31) / 32 * 32;
}

}  // namespace gpad
