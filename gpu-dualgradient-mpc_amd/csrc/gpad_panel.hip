// gpad_panel.hip -- shared-matrix batches on the f32 MFMA pipe (gfx950).
//
// When every instance of a batch shares ML and G (one plant, many states: the battery
// scenario batch), the two mat-vecs of a GPAD iteration over 16 instances are two skinny
// GEMMs:  Zhat[n x 16] = (-ML) W[m x 16]  and  Y'[m x 16] = G_L Zhat[n x 16].  One workgroup
// owns a panel of 16 instances for the whole solve (no inter-workgroup traffic at all).
// Both GEMMs are padded to T tiles of 16 rows (T = ceil(max(n, m)/16)) and the workgroup has
// T waves: wave t owns row tile t of BOTH GEMMs (one 4-register accumulator each), so every
// per-row quantity (z, y, u = G_L z, g_P, p_D) of the panel lives in registers, and W / Zhat
// are exchanged through LDS.  Many waves per SIMD hide the 40-cycle MFMA dependency and
// overlap one wave's epilogue with another wave's MFMAs.
//
// MFMA: v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate).  Lane l holds A[l&15][k=l>>4],
// B[k=l>>4][l&15] and C/D rows 4(l>>4)+r, column l&15 (r = 0..3).  Its result is bit-for-bit
// a k-ordered fmaf chain, so accumulating k-steps in ascending order reproduces the
// reference's sequential `sum += a*b` exactly (seq_functions.cpp:61,82).
//
// Row permutation pi(rho) = 4(rho&3) + (rho>>2) inside every 16-row tile of the packed A
// operands makes accumulator register r of lane (j = l>>4, c = l&15) hold original row
// 16t + 4r + j -- which is exactly the B-operand fragment of k-step 4t + r of the NEXT GEMM.
// So W and Zhat live in LDS in "fragment order" [tile][lane][4]: a ds_read_b128 per 16-k block
// yields the four B registers, with no transposes and no bank conflicts.
//
// Packed operands in HBM/L2 (built once by pack_panel_kernel at setup; T x T tiles each):
//   PA1[b][t][lane][q] = -ML[16t + pi(lane&15)][16b + 4q + (lane>>4)]   (b < TM, t < TN)
//   PA2[b][t][lane][q] = G_L[16t + pi(lane&15)][16b + 4q + (lane>>4)]   (b < TN, t < TM)
// one float4 per lane per (block, tile): 1 KiB per wave-instruction, fully coalesced.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <string>
#include <vector>

#include "gpad_chain.h"  // (the VALU butterflies of the test reductions)
#include "gpad_internal.h"

namespace gpad {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int pi16(int rho) { return 4 * (rho & 3) + (rho >> 2); }

// ---------------------------------------------------------------------------------------
// packing
// ---------------------------------------------------------------------------------------
constexpr int kPanelMaxTiles = 16;  // n, m <= 256 (1024-thread workgroups)

static int panel_tiles_for(int n, int m) {
    const int t = ((n > m ? n : m) + 15) / 16;
    return t <= kPanelMaxTiles ? t : 0;
}

__global__ void pack_panel_kernel(const float* __restrict__ src, int rows, int cols, double scale,
                                  int T, float4* __restrict__ dst) {
    // dst[(b*T + t)*64 + lane] for b < T (16-col blocks), t < T (16-row tiles)
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= T * T * 64) return;
    const int lane = idx & 63, t = (idx >> 6) % T, b = (idx >> 6) / T;
    const int row = 16 * t + pi16(lane & 15);
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int col = 16 * b + 4 * q + (lane >> 4);
        v[q] = (row < rows && col < cols) ? (float)(scale * (double)src[(size_t)row * cols + col]) : 0.0f;
    }
    dst[idx] = make_float4(v[0], v[1], v[2], v[3]);
}

// n or m beyond 256 rows: the big-panel layout (gpad_bigpanel.hip), rectangular tile grids
size_t panel_frag_bytes(int n, int m, int /*batch*/) {
    const int T = panel_tiles_for(n, m);
    if (!T) return bigpanel_frag_bytes(n, m);
    return (size_t)2 * T * T * 64 * sizeof(float4);
}

int panel_tiles(int n, int m, int /*batch*/) {
    const int T = panel_tiles_for(n, m);
    if (T) return T;
    return bigpanel_supported(n, m) ? ((n > m ? n : m) + 15) / 16 : 0;
}

hipError_t launch_pack_panel(const float* ML, const float* G, int n, int m, int /*batch*/,
                             float mg_sign, double g_scale, void* frag, hipStream_t s) {
    const int T = panel_tiles_for(n, m);
    if (!T) return bigpanel_supported(n, m) ? launch_pack_bigpanel(ML, G, n, m, mg_sign, g_scale, frag, s)
                                            : hipSuccess;
    float4* pa1 = reinterpret_cast<float4*>(frag);
    float4* pa2 = pa1 + (size_t)T * T * 64;
    const int tot = T * T * 64;
    // A1 = sign * ML (n x m);  A2 = g_scale * G (m x n)
    hipLaunchKernelGGL(pack_panel_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, ML, n, m,
                       (double)mg_sign, T, pa1);
    hipLaunchKernelGGL(pack_panel_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, G, m, n, g_scale, T,
                       pa2);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// the panel kernel: workgroup = panel of 16 instances, wave t = row tile t
// ---------------------------------------------------------------------------------------
struct PanelSlot {  // per wave (row tile), per instance partials of the Algorithm-1 test
    float violz[16], violh[16], wmin[16];
    double gap[16];
    float magh[16];  // max(|G_L zhat| + |pD|): test (B)'s rounding scale
};
// (A) nominated by the recursive u is decided on the direct G_L z (gpad_internal.h ViolMargin):
// the verification reuses violz / magh of the slots for max(G_L z + pD) / max(|G_L z| + |pD|).

// acc = A[tile t] (T k-blocks, streamed from L2 one block ahead) x B (LDS, fragment order).
// The MFMA k-order is ascending (block 0..T-1, step 0..3), i.e. the reference's sequential chain.
// A is read with buffer loads: one 32-bit lane offset (t*1 KiB + lane*16 B) in a VGPR and the
// k-block offset as a compile-time scalar, so the unrolled blocks cost no address registers.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// two rows per VALU instruction (v_pk_add / v_pk_mul / v_pk_fma_f32: IEEE f32 per element, the
// same rounding as the scalar forms, so the epilogues stay bit-identical)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 f2(float a, float b) { return f32x2{a, b}; }
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

__device__ __forceinline__ float4 as_float4(u32x4 v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                       __uint_as_float(v.w));
}

template <int T>
__device__ __forceinline__ f32x4 panel_gemm(__amdgpu_buffer_rsrc_t PA, const float* Bl, int voff,
                                            int lane) {
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    float4 a[2], b[2];
    a[0] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, 0, 0));
    b[0] = *reinterpret_cast<const float4*>(Bl + lane * 4);
#pragma unroll
    for (int kb = 0; kb < T; ++kb) {
        const int cur = kb & 1, nxt = cur ^ 1;
        if (kb + 1 < T) {
            a[nxt] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb + 1) * T * 1024, 0));
            b[nxt] = *reinterpret_cast<const float4*>(Bl + ((kb + 1) * 64 + lane) * 4);
        }
        // the next block's loads issue BEFORE this block's MFMAs (else the scheduler sinks them
        // below and waits on them at once: a full L2 round trip per k-block)
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].x, b[cur].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].y, b[cur].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].z, b[cur].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].w, b[cur].w, acc, 0, 0, 0);
        asm volatile("" ::: "memory");  // keep the prefetch one k-block deep
    }
    return acc;
}

// Phased compaction (continuous batching at phase granularity).  A solve with a tolerance is
// cut into phases of iterations [v_begin, v_end).  Within a phase every column runs the same
// global iteration index v, so theta/beta and the test events (v % K == 0) are uniform scalars
// and the per-iteration path has no per-column bookkeeping.  At a phase end the still-running
// instances park their state (z, y in the output arrays, w and u in carry buffers) and append
// their ids to a dense list; the next phase packs only those into panels.  Converged instances
// therefore stop occupying MFMA columns after at most one phase, instead of idling until the
// slowest instance of their static panel finishes.  Columns are independent in the MFMA, so an
// instance's arithmetic does not depend on its column, panel or phase (bit-exact either way).
// A workgroup walks panels grid-stride, so any batch size runs on a resident-sized grid.
template <int T>
__global__ __launch_bounds__(64 * T) void gpad_panel_kernel(SolveArgs<float> a) {
    __shared__ __attribute__((aligned(16))) float Wl[T * 256];  // [T][64][4] w    (B of GEMM 1)
    __shared__ __attribute__((aligned(16))) float Zh[T * 256];  // [T][64][4] zhat (B of GEMM 2)
    // per-lane constants of the current instance, parked in LDS rather than VGPRs:
    // g_P rows and p_D rows of tile t
    __shared__ __attribute__((aligned(16))) float Gp[T * 256];
    __shared__ __attribute__((aligned(16))) float Pd[T * 256];
    __shared__ PanelSlot slots[T];

    const int lane = threadIdx.x & 63;
    const int t = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // row tile of this wave
    const int j = lane >> 4, c = lane & 15;
    const int n = a.n, m = a.m, N = a.N, K = a.check_every;
    const int abytes = T * T * 1024;  // one packed operand
    const __amdgpu_buffer_rsrc_t PA1 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.frag), 0, abytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t PA2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)a.frag + abytes), 0, abytes, 0x00020000);
    const int voff = t * 1024 + lane * 16;
    const int slot = t * 64 + lane;  // this lane's float4 in Wl / Zh / Gp / Pd
    float4* Wl4 = reinterpret_cast<float4*>(Wl);
    float4* Zh4 = reinterpret_cast<float4*>(Zh);
    float4* Gp4 = reinterpret_cast<float4*>(Gp);
    float4* Pd4 = reinterpret_cast<float4*>(Pd);
    const bool use_tol = a.tol > 0.0;
    const bool fresh = a.v_begin == 0;      // first phase: start from the caller's z0, y0
    const bool carry = a.v_end < N;         // not the last phase: park the survivors
    const int count = a.count_in ? __builtin_amdgcn_readfirstlane(*a.count_in) : a.batch;
    if (a.count_in && count <= a.fin_thresh) return;  // the resident finisher has them
    const int panels = (count + 15) / 16;

    for (int p = blockIdx.x; p < panels; p += gridDim.x) {
        // ---- load the panel: column c <-> instance idx[16p + c] -------------------------
        const int k = 16 * p + c;
        bool active = k < count;
        const int inst = active ? (a.idx_in ? a.idx_in[k] : k) : 0;
        // register r <-> row 16t + 4r + j of the column's instance
        float z[4], y[4], u[4];
        {
            float gp[4], pd[4], w[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * t + 4 * r + j;
                const bool okn = active && i < n, okm = active && i < m;
                z[r] = okn ? a.z[(size_t)inst * n + i] : 0.0f;
                gp[r] = okn ? a.gP[(size_t)inst * a.ld_gP + i] : 0.0f;
                y[r] = okm ? a.y[(size_t)inst * m + i] : 0.0f;
                pd[r] = okm ? (float)(a.gscale * (double)a.g[(size_t)inst * a.ld_g + i]) : 0.0f;
                if (fresh) {  // w_0 = y_0 + beta_0 (y_0 - y_{-1}), y_{-1} = y_0; u set below
                    w[r] = __builtin_fmaf(a.beta[0], y[r] - y[r], y[r]);
                    u[r] = 0.0f;
                } else {
                    w[r] = okm ? a.wc[(size_t)inst * m + i] : 0.0f;
                    u[r] = okm && use_tol ? a.uc[(size_t)inst * m + i] : 0.0f;
                }
            }
            Gp4[slot] = make_float4(gp[0], gp[1], gp[2], gp[3]);
            Pd4[slot] = make_float4(pd[0], pd[1], pd[2], pd[3]);
            Wl4[slot] = make_float4(w[0], w[1], w[2], w[3]);
        }
        if (fresh && use_tol) {  // u = G_L z_{-1} (one GEMM for the panel); then the 8c recursion
            Zh4[slot] = make_float4(z[0], z[1], z[2], z[3]);
            __syncthreads();
            const f32x4 cz = panel_gemm<T>(PA2, Zh, voff, lane);
#pragma unroll
            for (int r = 0; r < 4; ++r) u[r] = cz[r];
        }
        __syncthreads();

        int v = a.v_begin;
        float th = a.theta[v], bn = a.beta[v + 1];
        while (true) {
            // schedule prefetched one iteration ahead (tables hold N + 2 entries)
            const float th_next = a.theta[v + 1], bn_next = a.beta[v + 2];
            ++v;
            const bool chk = use_tol && (v % K) == 0;  // uniform: every column is at iteration v
            const float omt = 1.0f - th;
            // ---- GEMM 1 + epilogue: zhat = -ML w - g_P (8b), z = (1-th) z + th zhat (8c) ----
            {
                const f32x4 acc = panel_gemm<T>(PA1, Wl, voff, lane);
                const float4 g4 = Gp4[slot];
                const float gp[4] = {g4.x, g4.y, g4.z, g4.w};
                float zh[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    zh[r] = acc[r] - gp[r];
                    const float zn = __builtin_fmaf(omt, z[r], th * zh[r]);
                    if (active) z[r] = zn;
                }
                Zh4[slot] = make_float4(zh[0], zh[1], zh[2], zh[3]);
            }
            __syncthreads();
            // ---- GEMM 2 + epilogue: y+ = [w + G_L zhat + p_D]+ (8d), next w (8a) ----------
            float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
            double gap = 0.0;
            {
                const f32x4 acc = panel_gemm<T>(PA2, Zh, voff, lane);
                const float4 w4 = Wl4[slot];
                const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
                const float4 p4 = Pd4[slot];
                const float pd[4] = {p4.x, p4.y, p4.z, p4.w};
                float wn[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float cv = acc[r];
                    const float sv = (wv[r] + pd[r]) + cv;
                    const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;
                    wn[r] = __builtin_fmaf(bn, yp - y[r], yp);
                    if (use_tol) {
                        const float un = __builtin_fmaf(omt, u[r], th * cv);
                        if (active) u[r] = un;
                        if (chk && active && (16 * t + 4 * r + j) < m) {
                            const float tt = cv + pd[r];
                            violh = fmaxf(violh, tt);
                            magh = fmaxf(magh, __builtin_fabsf(cv) + __builtin_fabsf(pd[r]));
                            wmin = fminf(wmin, wv[r]);
                            gap -= (double)wv[r] * (double)tt;
                            violz = fmaxf(violz, u[r] + pd[r]);
                        }
                    }
                    if (active) y[r] = yp;
                }
                if (active) Wl4[slot] = make_float4(wn[0], wn[1], wn[2], wn[3]);
            }
            th = th_next;
            bn = bn_next;
            __syncthreads();
            if (!chk && v < a.v_end) continue;

            // ---- Algorithm 1 test, per column: lane groups j, then row tiles through LDS ----
            int code = 0;
            bool zh_out = true;  // this iteration's zhat still in Zh (no verification GEMM ran)
            if (chk) {
                // lane groups j (xor 16, 32) on the VALU (gpad_chain.h: the shfl_xor butterfly's values)
                violz = bfly<32>(bfly<16>(violz, OpMax{}), OpMax{});
                violh = bfly<32>(bfly<16>(violh, OpMax{}), OpMax{});
                magh = bfly<32>(bfly<16>(magh, OpMax{}), OpMax{});
                wmin = bfly<32>(bfly<16>(wmin, OpMin{}), OpMin{});
                gap = bfly<32>(bfly<16>(gap, OpAdd{}), OpAdd{});
                if (j == 0) {
                    slots[t].violz[c] = violz;
                    slots[t].violh[c] = violh;
                    slots[t].magh[c] = magh;
                    slots[t].wmin[c] = wmin;
                    slots[t].gap[c] = gap;
                }
                __syncthreads();
                int st1 = 0;
                if (active) {
                    double vz = -INFINITY, vh = -INFINITY, wm = INFINITY, gq = 0.0, mh = 0.0;
#pragma unroll
                    for (int s2 = 0; s2 < T; ++s2) {
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
                bool verified = false;
                if (__syncthreads_or(st1 & 1)) {  // (A) nominated somewhere: G_L z for the panel
                    zh_out = false;
                    if (st1 & 2) {  // test (B)'s result (zhat) out now: Zh is about to hold z
                        const float4 h4 = Zh4[slot];
                        const float zh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int i = 16 * t + 4 * r + j;
                            if (i < n) a.z[(size_t)inst * n + i] = zh[r];
                        }
                    }
                    Zh4[slot] = make_float4(z[0], z[1], z[2], z[3]);
                    __syncthreads();
                    const f32x4 cz = panel_gemm<T>(PA2, Zh, voff, lane);
                    const float4 p4 = Pd4[slot];
                    const float pd[4] = {p4.x, p4.y, p4.z, p4.w};
                    float vc = -INFINITY, mc = 0.0f;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if ((st1 & 1) && (16 * t + 4 * r + j) < m) {
                            u[r] = cz[r];  // the recursion restarts from the direct value
                            vc = fmaxf(vc, cz[r] + pd[r]);
                            mc = fmaxf(mc, __builtin_fabsf(cz[r]) + __builtin_fabsf(pd[r]));
                        }
                    }
                    vc = bfly<32>(bfly<16>(vc, OpMax{}), OpMax{});
                    mc = bfly<32>(bfly<16>(mc, OpMax{}), OpMax{});
                    if (j == 0) {  // every wave finished reading the slots before the barrier above
                        slots[t].violz[c] = vc;
                        slots[t].magh[c] = mc;
                    }
                    __syncthreads();
                    if (st1 & 1) {
                        double vcc = -INFINITY, mcc = 0.0;
#pragma unroll
                        for (int s2 = 0; s2 < T; ++s2) {
                            vcc = fmax(vcc, (double)slots[s2].violz[c]);
                            mcc = fmax(mcc, (double)slots[s2].magh[c]);
                        }
                        verified = viol_ok(vcc, mcc, a.L, a.tol, ViolMargin<float>::value);
                    }
                }
                code = ((st1 & 1) && verified) ? 1 : ((st1 & 2) ? 2 : 0);
            }
            // ---- finished columns: results out ---------------------------------------------
            if (active && (code != 0 || v >= N)) {
                const float4 h4 = Zh4[slot];  // this iteration's zhat (own slot), unless verified over
                const float zh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * t + 4 * r + j;
                    if (i < n && (code != 2 || zh_out)) a.z[(size_t)inst * n + i] = code == 2 ? zh[r] : z[r];
                    if (i < m) a.y[(size_t)inst * m + i] = y[r];
                }
                if (t == 0 && j == 0) {
                    a.iters[inst] = v;
                    a.conv[inst] = code;
                }
                active = false;
            }
            if (v >= a.v_end || !__syncthreads_or(active ? 1 : 0)) break;
        }
        // ---- phase end: park the survivors for the next phase ------------------------------
        if (carry) {
            const bool park = active && v >= a.v_end;
            if (park) {
                const float4 w4 = Wl4[slot];  // w of iteration v (own slot)
                const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * t + 4 * r + j;
                    if (i < n) a.z[(size_t)inst * n + i] = z[r];
                    if (i < m) {
                        a.y[(size_t)inst * m + i] = y[r];
                        a.wc[(size_t)inst * m + i] = wv[r];
                        if (use_tol) a.uc[(size_t)inst * m + i] = u[r];
                    }
                }
            }
            if (t == 0) list_survivors(a, p, park, inst, lane, j);  // lanes 0..15 speak for the columns
        }
        __syncthreads();  // the next panel reuses the LDS tiles
    }
}

// Prelude priority (r05).  The SIMD issues oldest wave first, VALU and MFMA from one port: while
// an older wave has an MFMA ready (a double wave always has), a younger wave cannot issue even the
// VALU ops between the barrier and its first MFMA (uniform-branch compares, spilled-SGPR
// v_readlanes, LDS addresses), so it does not even read its first B fragment until the older
// chains are done, and each hand-over between the waves of a SIMD costs the younger wave's whole
// prelude plus the LDS latency of its B reads (~600 cycles, profiles/r05_stamp_*.txt: the loop tops
// of a SIMD's waves fall 1.3k, 5k, 7.6k cycles after the barrier).  So every wave raises its
// priority before the barriers of the solve loop and drops it right before its first MFMA of the
// next GEMM: all waves get through their preludes and issue their first B reads right after the
// barrier, and the chains then run oldest-first with their operands already in registers.
// Invariant: a wave holds priority 2 only between a loop barrier and its next chain (or the point
// where it learns it has none); every path out of that window -- a GEMM helper's prelude, the
// no-GEMM branches of the tiles past the output rows, the loop exit -- drops it to 0.
#define GPAD_PRELUDE_HI() __builtin_amdgcn_s_setprio(2)
#define GPAD_PRELUDE_LO()                  \
    do {                                   \
        __builtin_amdgcn_sched_barrier(0); \
        __builtin_amdgcn_s_setprio(0);     \
        __builtin_amdgcn_sched_barrier(0); \
    } while (0)

// ---------------------------------------------------------------------------------------
// Panel pairs (8 < T <= 16): a 16-wave workgroup owns TWO panels, balanced over the SIMDs.
// A 13-wave single-panel workgroup puts 4,3,3,3 waves (tile chains) on the CU's SIMDs, and a
// second one is not co-resident at its register budget, so the busiest SIMD carries 4 chains
// while the mean is 3.25.  Here the 2T (panel, tile) chains of two panels are dealt to 16 waves
// (4 per SIMD, waves w, w+4, w+8, w+12 share one): D = 2T-16 "double" waves own tile w of BOTH
// panels -- one A fragment feeds two MFMA chains, which also hides the 40-cycle MFMA
// dependency -- and the 32-2T "single" waves own one (panel, tile) each.  Doubles go to waves
// 0..D-1, i.e. round-robin over the SIMDs, so the SIMD loads differ by at most one chain
// (T = 13: 7,7,6,6 for 26 chains).  When a phase has no more panels than workgroups, a
// workgroup takes one panel (waves 0..T-1, one tile each): pairing would only idle CUs.
// ---------------------------------------------------------------------------------------
template <int T, bool DUAL>
__device__ __forceinline__ void panel_gemm2(__amdgpu_buffer_rsrc_t PA, const float4* B0, const float4* B1,
                                            int voff, int lane, f32x4& acc0, f32x4& acc1) {
    acc0 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    acc1 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    float4 a[2], b0[2], b1[2];
    a[0] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, 0, 0));
    b0[0] = B0[lane];
    if constexpr (DUAL) b1[0] = B1[lane];
    GPAD_PRELUDE_LO();
#pragma unroll
    for (int kb = 0; kb < T; ++kb) {
        const int cur = kb & 1, nxt = cur ^ 1;
        if (kb + 1 < T) {
            a[nxt] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb + 1) * T * 1024, 0));
            b0[nxt] = B0[(kb + 1) * 64 + lane];
            if constexpr (DUAL) b1[nxt] = B1[(kb + 1) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].x, b0[cur].x, acc0, 0, 0, 0);
        if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].x, b1[cur].x, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].y, b0[cur].y, acc0, 0, 0, 0);
        if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].y, b1[cur].y, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].z, b0[cur].z, acc0, 0, 0, 0);
        if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].z, b1[cur].z, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].w, b0[cur].w, acc0, 0, 0, 0);
        if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].w, b1[cur].w, acc1, 0, 0, 0);
        // both chains advance together, one k-block per step (else the scheduler defers the
        // second chain past the loop and keeps every B fragment live)
        if constexpr (DUAL) asm volatile("" : "+v"(acc0), "+v"(acc1)::"memory");
        else asm volatile("" : "+v"(acc0)::"memory");
    }
}

// A fragments of the first PD k-blocks, issued early (before the barrier that precedes the
// GEMM: A is the constant matrix, so its L2 latency need not start at the barrier).
template <int T, int PD>
__device__ __forceinline__ void panel_a_prefetch(__amdgpu_buffer_rsrc_t PA, int voff, float4 (&ap)[PD]) {
#pragma unroll
    for (int p = 0; p < PD; ++p)
        if (p < T) ap[p] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, p * T * 1024, 0));
}

// panel_gemm2 with an A ring PD blocks deep, seeded by panel_a_prefetch.  The last k-block
// issues only its first kq MFMA steps: k-steps past the matrix are zero in both operands, so
// skipping them is exact (an accumulator started at +0 never holds -0).  kq is wave-uniform.
template <int T, bool DUAL, int PD>
__device__ __forceinline__ void panel_gemm3(__amdgpu_buffer_rsrc_t PA, const float4* B0, const float4* B1,
                                            int voff, int lane, f32x4& acc0, f32x4& acc1,
                                            const float4 (&ap)[PD], int kq) {
    acc0 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    acc1 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    constexpr int R = PD + 1;
    float4 a[R], b0[2], b1[2];
#pragma unroll
    for (int p = 0; p < PD; ++p) a[p] = ap[p];
    b0[0] = B0[lane];
    if constexpr (DUAL) b1[0] = B1[lane];
    b0[1] = B0[64 + lane];  // (block 1 too, so the whole prelude precedes the priority drop)
    if constexpr (DUAL) b1[1] = B1[64 + lane];
    GPAD_PRELUDE_LO();
#pragma unroll
    for (int kb = 0; kb < T; ++kb) {
        const int cur = kb & 1, nxt = cur ^ 1;
        const float4 ak = a[kb % R];
        if (kb + PD < T)
            a[(kb + PD) % R] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb + PD) * T * 1024, 0));
        if (kb >= 1 && kb + 1 < T) {  // (blocks 0 and 1 were read before the loop)
            b0[nxt] = B0[(kb + 1) * 64 + lane];
            if constexpr (DUAL) b1[nxt] = B1[(kb + 1) * 64 + lane];
        }
        __builtin_amdgcn_sched_barrier(0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.x, b0[cur].x, acc0, 0, 0, 0);
        if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.x, b1[cur].x, acc1, 0, 0, 0);
        if (kb + 1 < T || kq > 1) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.y, b0[cur].y, acc0, 0, 0, 0);
            if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.y, b1[cur].y, acc1, 0, 0, 0);
        }
        if (kb + 1 < T || kq > 2) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.z, b0[cur].z, acc0, 0, 0, 0);
            if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.z, b1[cur].z, acc1, 0, 0, 0);
        }
        if (kb + 1 < T || kq > 3) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.w, b0[cur].w, acc0, 0, 0, 0);
            if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.w, b1[cur].w, acc1, 0, 0, 0);
        }
        if constexpr (DUAL) asm volatile("" : "+v"(acc0), "+v"(acc1)::"memory");
        else asm volatile("" : "+v"(acc0)::"memory");
    }
}

// Runtime-length variant for a GEMM whose K spans fewer k-blocks than the tile count
// (n != m: e.g. the battery's n = 40 against m = 180 -> 3 of 12 blocks).  Unrolled by two with
// fixed register roles (even blocks in a0, odd in a1) and every load unconditional (indices
// clamped to the last block), so each block's waitcnt counts only the loads issued after its
// operands -- a rotated ring with conditional loads made the compiler drain both counters at
// every block.  A is PD (1 or 2) blocks ahead, B one block ahead; soffset in an SGPR.
template <int T, bool DUAL, int PD>
__device__ __forceinline__ void panel_gemm_rt(__amdgpu_buffer_rsrc_t PA, const float4* B0, const float4* B1,
                                              int voff, int lane, f32x4& acc0, f32x4& acc1,
                                              const float4 (&ap)[PD], int nkb, int kq) {
    constexpr int PR = PD > 2 ? 2 : PD;  // (deeper rings seed only their first two blocks here)
    acc0 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    acc1 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int last = nkb - 1;
    auto lda = [&](int kb) -> float4 {
        return as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb < last ? kb : last) * T * 1024, 0));
    };
    auto blk = [&](const float4& ak, const float4& bk0, const float4& bk1, int steps) {
        __builtin_amdgcn_sched_barrier(0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.x, bk0.x, acc0, 0, 0, 0);
        if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.x, bk1.x, acc1, 0, 0, 0);
        if (steps > 1) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.y, bk0.y, acc0, 0, 0, 0);
            if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.y, bk1.y, acc1, 0, 0, 0);
        }
        if (steps > 2) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.z, bk0.z, acc0, 0, 0, 0);
            if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.z, bk1.z, acc1, 0, 0, 0);
        }
        if (steps > 3) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.w, bk0.w, acc0, 0, 0, 0);
            if constexpr (DUAL) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.w, bk1.w, acc1, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    float4 a0 = ap[0], a1 = PR == 2 ? ap[1] : ap[0];
    float4 e0 = B0[lane], f0 = DUAL ? B1[lane] : e0, e1, f1;
    GPAD_PRELUDE_LO();
    for (int kb = 0;; kb += 2) {
        const int k1 = kb + 1 < last ? kb + 1 : last, k2 = kb + 2 < last ? kb + 2 : last;
        if constexpr (PR == 1) a1 = lda(kb + 1);
        e1 = B0[k1 * 64 + lane];
        if constexpr (DUAL) f1 = B1[k1 * 64 + lane];
        blk(a0, e0, f0, kb < last ? 4 : kq);
        if constexpr (PR == 2) a0 = lda(kb + 2);
        if (kb + 1 > last) break;
        if constexpr (PR == 1) a0 = lda(kb + 2);
        e0 = B0[k2 * 64 + lane];
        if constexpr (DUAL) f0 = B1[k2 * 64 + lane];
        blk(a1, e1, f1, kb + 1 < last ? 4 : kq);
        if constexpr (PR == 2) a1 = lda(kb + 3);
        if (kb + 2 > last) break;
    }
    if constexpr (DUAL) asm volatile("" : "+v"(acc0), "+v"(acc1)::"memory");
    else asm volatile("" : "+v"(acc0)::"memory");
}

// k-blocks [KB0, KB1) of one chain, continuing acc (not reset): the A ring PD blocks deep is
// seeded with blocks KB0.. by panel_a_prefetch_from; the last matrix block issues kq steps.
template <int T, int PD, int KB0, int KB1, bool LO = true>
__device__ __forceinline__ void panel_chain(__amdgpu_buffer_rsrc_t PA, const float4* B0, int voff, int lane,
                                            f32x4& acc, const float4 (&ap)[PD], int kq) {
    constexpr int R = PD + 1;
    float4 a[R], b[2];
#pragma unroll
    for (int p = 0; p < PD; ++p) a[p] = ap[p];
    b[0] = B0[KB0 * 64 + lane];
    if constexpr (LO) GPAD_PRELUDE_LO();  // (LO = false: a relay piece that runs at its own priority)
#pragma unroll
    for (int kb = KB0; kb < KB1; ++kb) {
        const int i = kb - KB0, cur = i & 1, nxt = cur ^ 1;
        const float4 ak = a[i % R];
        if (kb + PD < KB1)
            a[(i + PD) % R] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb + PD) * T * 1024, 0));
        if (kb + 1 < KB1) b[nxt] = B0[(kb + 1) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.x, b[cur].x, acc, 0, 0, 0);
        if (kb + 1 < T || kq > 1) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.y, b[cur].y, acc, 0, 0, 0);
        if (kb + 1 < T || kq > 2) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.z, b[cur].z, acc, 0, 0, 0);
        if (kb + 1 < T || kq > 3) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ak.w, b[cur].w, acc, 0, 0, 0);
        asm volatile("" : "+v"(acc)::"memory");
    }
}

template <int T, int PD>
__device__ __forceinline__ void panel_a_prefetch_from(__amdgpu_buffer_rsrc_t PA, int voff, float4 (&ap)[PD],
                                                      int kb0) {
#pragma unroll
    for (int p = 0; p < PD; ++p)
        if (kb0 + p < T) ap[p] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb0 + p) * T * 1024, 0));
}

// Chain hand-off (T = 9, 11, 13, both GEMMs full-length).  A chain is an ascending-k sequence of
// f32 MFMAs whose C operand is the previous step's result; it may be cut at any k-block and
// continued on another wave -- even on another SIMD -- from an accumulator parked in LDS, and the
// result is bit-identical.  The layouts use this to even out the SIMDs' chain loads:
// * pairs: with 2T chains per GEMM the 16-wave deal leaves SIMDs 0,1 one chain above SIMDs 2,3
//   (7,7,6,6; the phase lasts 7 chains of a mean 6.5).  The single wave on SIMD 2 (3) that owns
//   tile T-1 of panel 0 (1) first runs k-blocks [0, S) of tile T-2 of the same panel -- the chain
//   of wave 12 (13) on SIMD 0 (1) -- then its own chain; wave 12 (13) continues from block S.
//   Every SIMD then carries 6.5 chains.
// * one panel per workgroup: T waves put 4,3,3,3 chains on the SIMDs while waves 13..15 idle.
//   Tile T-1's chain (wave 12, SIMD 0) instead runs as a relay: blocks [0,4) on wave 13 (SIMD 1),
//   [4,8) on 14 (SIMD 2), [8,T) and the epilogue on wave 12 -- the busiest SIMD carries 3.36
//   chains (T = 9 likewise: 3,2,2,2 chains, tile 8 over waves 9 -> 10 -> 8).  The relay is a
//   sequential path through three SIMDs (each piece issues at most every other MFMA slot of its
//   SIMD, plus ~300 cycles per hand-off), so it must stay shorter than the SIMDs' own chains:
//   raised issue priorities, whole pieces prefetched before the barrier, and a fourth hop (a
//   4-way relay) measured slower than none.
// A slot's flag carries the hand-off generation (one per GEMM, counted alike by every wave), so
// flags are never reset; a receiver waits with a bound, and a wait that expires fails the run
// (handoff_wait: GPAD_ERR_DEVICE) rather than hanging the GPU or returning stale results.
template <int T>
struct Handoff {
    // pairs: odd T with singles on waves 12..15 (T = 9, 11, 13: SIMD loads 5,5,4,4 / 6,6,5,5 /
    // 7,7,6,6); one panel: T = 9, 13 (T % 4 == 1: SIMD 0 carries the extra tile, waves T, T+1 idle)
    static constexpr bool on = T == 9 || T == 11 || T == 13;
    static constexpr bool relay = T == 9 || T == 13;
    static constexpr int S = T / 2;      // pairs: helper blocks 4S MFMAs vs 4(T-S)-4+kq on the receiver
    static constexpr int R1 = T / 3, R2 = 2 * (T / 3);  // one panel: relay cuts (equal pieces, prefetched whole)
};

// Per (panel, row tile) partials of the test, one entry per column: the four float terms packed
// (violz, violh, magh, wmin: one ds_read_b128 per tile on the reduction side) and the fp64 gap.
// The verification of a nominated (A) reuses .x / .z for max(G_L z + pD) / max(|G_L z| + |pD|).
struct PanelSlot2 {
    float4 f[16];
    double gap[16];
};

// The tile reduction of the test, every wave at once (uniform result, no vote barrier): lane
// 16 pp + cc reduces tiles [0, H) of column cc of panel pp, lane 32 + 16 pp + cc tiles [H, T);
// the halves meet through one xor-32 exchange.  The f32 maxima / minima are exact in any order
// (one conversion to fp64 after them instead of one per tile); the fp64 gap is summed per half,
// then the halves added.
template <int T>
__device__ __forceinline__ void panel2_reduce(const PanelSlot2 (&S)[2][T], int lane, float4& f, double& gap) {
    constexpr int H = (T + 1) / 2;
    const int pp = (lane >> 4) & 1, cc = lane & 15, lo = lane < 32 ? 0 : H, hi = lane < 32 ? H : T;
    f = make_float4(-INFINITY, -INFINITY, 0.0f, INFINITY);
    gap = 0.0;
#pragma unroll
    for (int s2 = 0; s2 < H; ++s2) {
        // every step but the last is in range on both halves (2H - 2 <= T - 1): no per-lane branch,
        // whose exec masks the compiler kept in spilled SGPRs; the last step selects
        const bool ok = s2 < H - 1 || lo + s2 < hi;
        const int si = ok ? lo + s2 : lo;
        const float4 e = S[pp][si].f[cc];
        const double gv = S[pp][si].gap[cc];
        f.x = ok ? fmaxf(f.x, e.x) : f.x;
        f.y = ok ? fmaxf(f.y, e.y) : f.y;
        f.z = ok ? fmaxf(f.z, e.z) : f.z;
        f.w = ok ? fminf(f.w, e.w) : f.w;
        gap = ok ? gap + gv : gap;
    }
    f.x = bfly<32>(f.x, OpMax{});  // (gfx950 v_permlane32_swap, gpad_chain.h)
    f.y = bfly<32>(f.y, OpMax{});
    f.z = bfly<32>(f.z, OpMax{});
    f.w = bfly<32>(f.w, OpMin{});
    gap = bfly<32>(gap, OpAdd{});  // (lower half + upper half on every lane, as before)
}

template <int T>
struct Panel2Lds {
    float4 Wl[2][T * 64];  // fragment order, per panel: w    (B of GEMM 1)
    float4 Zh[2][T * 64];  //                            zhat (B of GEMM 2)
    float4 Gp[2][T * 64];  //                            g_P rows
    float4 Pd[2][T * 64];  //                            p_D rows
    PanelSlot2 slots[2][T];
    float4 hand[2][64];    // hand-off accumulators (the pair helpers' / the relay's slots)
    int hflag[2];          // hand-off generation per slot
    int herr;              // a wait expired (handoff_wait): reported to the run's error word at exit
    int hdrop;             // fault injection (kDebugDropHandoff) for this workgroup
    int znz[16];           // per wave: a non-zero z_{-1} among its rows (fresh seed GEMM needed)
    float gred[16];        // per wave: max |g| over the rows it loaded (SolveArgs::gmax_part)
};

// Phase anatomy stamps (diagnostic builds only, -DGPAD_STAMP; never in the product library): the
// shader clock (s_memtime) of workgroup 0, every wave, iterations [kStampV0, kStampV0 + kStampIts),
// at six points per iteration -- loop top, GEMM-1 issued, before its barrier, after it, GEMM-2
// issued, before the closing barrier -- read back with gpad_debug_stamps (tools/stamp_panel.py).
#ifdef GPAD_STAMP
#ifndef GPAD_STAMP_V0
#define GPAD_STAMP_V0 101
#endif
#ifndef GPAD_STAMP_PHASE_V
#define GPAD_STAMP_PHASE_V 100
#endif
constexpr int kStampV0 = GPAD_STAMP_V0, kStampIts = 4, kStampPts = 8;  // 6, 7: GEMM 1 / 2 hand-off wait returned
__device__ unsigned long long g_stamps[16][kStampIts][kStampPts];
// s_memtime into SGPRs at each point (pinned by scheduling barriers), stored once per iteration after
// the closing barrier: the store's lgkmcnt wait then sits where no LDS or scalar load is in flight,
// instead of behind each stamp (where it made every stamp wait for the LDS operands and the
// schedule's scalar loads, r03_stamp_*.txt)
#define GPAD_STAMP_AT(P)                                      \
    do {                                                      \
        __builtin_amdgcn_sched_barrier(0);                    \
        stv[P] = __builtin_amdgcn_s_memtime();                \
        __builtin_amdgcn_sched_barrier(0);                    \
    } while (0)
#define GPAD_STAMP_FLUSH()                                                                  \
    do {                                                                                    \
        if (blockIdx.x == 0 && v >= kStampV0 && v < kStampV0 + kStampIts && lane == 0)      \
            for (int q_ = 0; q_ < kStampPts; ++q_) g_stamps[threadIdx.x >> 6][v - kStampV0][q_] = stv[q_]; \
    } while (0)
#define GPAD_STAMP_DECL unsigned long long stv[kStampPts] = {0, 0, 0, 0, 0, 0, 0, 0};
// phase anatomy of workgroup 0 in the phase that starts at kStampPhaseV: entry, state loaded, after
// the load barrier, loop exit, survivors parked, after the closing barrier
constexpr int kStampPhaseV = GPAD_STAMP_PHASE_V, kStampPhasePts = 10;  // 6..9: the phase's last test (below)
__device__ unsigned long long g_pstamps[16][kStampPhasePts];
#define GPAD_PSTAMP(P)                                                                              \
    do {                                                                                            \
        __builtin_amdgcn_sched_barrier(0);                                                          \
        if (blockIdx.x == 0 && a.v_begin == kStampPhaseV && (threadIdx.x & 63) == 0)               \
            g_pstamps[threadIdx.x >> 6][P] = __builtin_amdgcn_s_memtime();                          \
        __builtin_amdgcn_sched_barrier(0);                                                          \
    } while (0)
#define GPAD_STAMP_PTR(P) (&stv[P])
// the test at the phase's last iteration: entry, decisions voted, verification done, results out
#define GPAD_PSTAMP_END(P)                  \
    do {                                    \
        if (v >= a.v_end) GPAD_PSTAMP(P);   \
    } while (0)
#else
#define GPAD_PSTAMP_END(P) \
    do {                   \
    } while (0)
#define GPAD_STAMP_AT(P) \
    do {                 \
    } while (0)
#define GPAD_STAMP_FLUSH() \
    do {                   \
    } while (0)
#define GPAD_STAMP_DECL
#define GPAD_STAMP_PTR(P) nullptr
#define GPAD_PSTAMP(P) \
    do {               \
    } while (0)
#endif

struct HoSlots {
    int in, out;  // LDS hand-off slots taken / given (-1: none)
};

// The results-out and park sites launder the column's instance index and the lane through an empty
// asm before forming its row pointers and offsets (r06): otherwise the compiler hoists the six per-panel 64-bit row pointers
// (z, y, wc, uc ... of each panel) out of the solve loop, and at 128 VGPRs the double waves spilled them
// -- 240 B of scratch per lane whose dirty lines were written back to HBM, ~39 MB per phase-1 launch at
// C4 (profiles/r06_write_probe.txt: a fixed-N launch that stores only z*, y* (13 MB) wrote 52 MB).
// This lane's four rows 16t + 4r + j (r = 0..3) of one instance's vector.  vec (16-B aligned rows):
// rows4_dma, one global_load_lds_dwordx4 per lane (the 16 columns x 64 contiguous bytes of a wave's
// tile, a quarter of the requests of four 4-B loads per lane) into 1 KiB of LDS the wave owns, then
// rows4_rd.  The DMA lands lane-linearly: lane l carries column c' = l >> 2's rows 16t + 4j' .. +3,
// j' = (l & 3) ^ ((c' >> 2) & 3), so the block holds column c's 16 floats with the 16-B chunks
// XOR-swizzled by c >> 2 and the four reads are conflict-free.  colbase is column c''s instance
// row 0; the tile's rows past `rows` read the last four rows (the caller zeroes them).  r05 loaded
// into VGPRs and transposed through the block, which serialised the operands' loads behind each
// other's LDS waits; r06 stages by DMA, every operand of every panel in flight at once and no VGPRs
// held meanwhile (batching the VGPR loads instead spilled: 45-69 VGPRs in the pair kernels).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

__device__ __forceinline__ void rows4_dma(const float* colbase, int t, int rows, int lane, float4* blk) {
    const int cc = lane >> 2;
    const int jj = (lane & 3) ^ ((cc >> 2) & 3);
    const int r0 = 16 * t + 4 * jj;
    const int rr = r0 + 3 < rows ? r0 : rows - 4;
    __builtin_amdgcn_global_load_lds((gbl_void_t*)(colbase + rr), (lds_void_t*)blk, 16, 0, 0);
}

__device__ __forceinline__ void rows4_rd(const float4* blk, int lane, float (&out)[4]) {
    const float* st = reinterpret_cast<const float*>(blk);
    const int j = lane >> 4, c = lane & 15, sw = (c >> 2) & 3;
#pragma unroll
    for (int r = 0; r < 4; ++r) out[r] = st[16 * c + 4 * (r ^ sw) + j];
}

// the scalar path (rows not 16-B aligned): four 4-B loads at clamped rows
__device__ __forceinline__ void rows4(const float* base, int t, int rows, int lane, float (&out)[4]) {
    const int j = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 16 * t + 4 * r + j;
        out[r] = base[i < rows ? i : rows - 1];
    }
}

// The reverse of the loads above: this lane's rows 16t + 4r + j to an instance's vector, on lanes
// whose `on` holds (uniform over a column's four lanes); vec: transposed through the wave's LDS block
// into one 16-B store per lane of rows 16t + 4j .. +3 (every lane takes part in the transpose; rows
// past `rows` not stored).
__device__ __forceinline__ void rows4_store(float* base, int t, int rows, bool vec, float* st, int lane,
                                            const float (&v)[4], bool on) {
    const int j = lane >> 4, c = lane & 15, sw = (c >> 2) & 3;
    if (vec) {
#pragma unroll
        for (int r = 0; r < 4; ++r) st[16 * c + 4 * (r ^ sw) + j] = v[r];
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const float4 o = *reinterpret_cast<const float4*>(st + 16 * c + 4 * (j ^ sw));
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int r0 = 16 * t + 4 * j;
        if (on && r0 < rows) *reinterpret_cast<float4*>(base + r0) = o;
    } else if (on) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * t + 4 * r + j;
            if (i < rows) base[i] = v[r];
        }
    }
}

// The waves of a workgroup are co-resident, so a post always arrives unless the layout logic is
// broken; the wait is still bounded (2^20 sleeps, ~30 ms) so that such a bug cannot hang the GPU,
// and an expired wait is recorded (L.herr) and ORed into the run's error word when the workgroup
// exits (gpad_panel2_kernel): the host then fails the run with GPAD_ERR_DEVICE instead of
// returning the stale accumulator's results as GPAD_OK.  Nothing of this sits on the hand-off's
// own path: the record is made only after the bound expired.
template <int T>
__device__ __forceinline__ f32x4 handoff_wait(Panel2Lds<T>& L, int slot, int gen, int lane) {
    for (int s = 0;; ++s) {
        if (__hip_atomic_load(&L.hflag[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == gen) break;
        if (s == (1 << 20)) {
            L.herr = 1;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    const float4 hv = L.hand[slot][lane];
    return f32x4{hv.x, hv.y, hv.z, hv.w};
}

template <int T>
__device__ __forceinline__ void handoff_post(Panel2Lds<T>& L, int slot, int gen, int lane, const f32x4& h) {
    L.hand[slot][lane] = make_float4(h[0], h[1], h[2], h[3]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the accumulator lands before the flag
    __hip_atomic_store(&L.hflag[slot], gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// a piece of another wave's chain: k-blocks [KB0, KB1) (KB1 < T) of the tile at voff, continued
// from slot hs.in (or from zero), parked in slot hs.out; PRIO raises the wave's issue priority
// fault injection (DROP, the kernel's test-only instantiation; L.hdrop): the first piece of the
// first hand-off withholds its post, so its receiver's wait expires
template <int T, int PD, int KB0, int KB1, bool PRIO, bool DROP>
__device__ __forceinline__ void handoff_piece(Panel2Lds<T>& L, __amdgpu_buffer_rsrc_t PA, const float4* B0, int voff,
                                              int lane, const float4 (&aph)[PD], HoSlots hs, int gen,
                                              unsigned long long* ts = nullptr) {
    f32x4 h = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (hs.in >= 0) h = handoff_wait(L, hs.in, gen, lane);
    if (ts) *ts = __builtin_amdgcn_s_memtime();  // (stamped builds only)
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
    panel_chain<T, PD, KB0, KB1, !PRIO>(PA, B0, voff, lane, h, aph, 4);
    if (!(DROP && gen == 1 && hs.in < 0 && L.hdrop)) handoff_post(L, hs.out, gen, lane, h);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
}

// the chain's last piece on its owner: blocks [KB0, T) from slot hs.in
template <int T, int PD, int KB0, bool PRIO>
__device__ __forceinline__ void handoff_take(Panel2Lds<T>& L, __amdgpu_buffer_rsrc_t PA, const float4* B0, int voff,
                                             int lane, const float4 (&ap)[PD], HoSlots hs, int gen, int kq,
                                             f32x4& acc, unsigned long long* ts = nullptr) {
    acc = handoff_wait(L, hs.in, gen, lane);
    if (ts) *ts = __builtin_amdgcn_s_memtime();  // (stamped builds only)
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(2);
    panel_chain<T, PD, KB0, T, !PRIO>(PA, B0, voff, lane, acc, ap, kq);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
}

// Hand-off roles (Handoff): 0 none; 1 pair helper (NU = 1: blocks [KB0, KB1) of tile t-1 into
// slot hs.out, then its own chain); 2 receiver (NU = 1: its own chain from block KB0, slot hs.in);
// 3 relay (NU = 0: blocks [KB0, KB1) of tile t from slot hs.in, or zero, into slot hs.out).
// PRIO: the one-panel relay raises issue priority for its pieces.
// KQ > 0: the shape is known at compile time to have full-length chains on every tile of both
// GEMMs (16 (T-1) < n, m <= 16 T) whose last k-block issues KQ steps in both: no runtime kq tests
// (scalar branches whose conditions the compiler spilled to VGPR lanes) and no short-chain paths.
// DROP: the fault-injection instantiation (handoff_piece).
template <int T, int NU, int ROLE = 0, int KB0 = 0, int KB1 = 0, bool PRIO = false, int KQ = 0, bool DROP = false>
__device__ __forceinline__ void panel2_run(const SolveArgs<float>& a, Panel2Lds<T>& L, int t, int p0,
                                           bool pair, int items, int count, HoSlots hs = HoSlots{-1, -1}) {
    static_assert(ROLE == 0 || (Handoff<T>::on && (ROLE == 3 ? NU == 0 : NU == 1)), "hand-off roles");
    const int lane = threadIdx.x & 63;
    const int j = lane >> 4, c = lane & 15;
    const int n = a.n, m = a.m, N = a.N, K = a.check_every;
    const int abytes = T * T * 1024;
    const __amdgpu_buffer_rsrc_t PA1 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.frag), 0, abytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t PA2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)a.frag + abytes), 0, abytes, 0x00020000);
    const bool use_tol = a.tol > 0.0;
    const bool fresh = a.v_begin == 0;
    const bool carry = a.v_end < N;
    const int voff = t * 1024 + lane * 16;
    const int slot = t * 64 + lane;
    constexpr int Q = NU > 0 ? NU : 1;  // array extent
    // GEMM 1: K = m, output rows n; GEMM 2: K = n, output rows m.  The last k-block issues only
    // the steps inside K when K is the padded dimension (kq), and a wave whose tile lies past
    // the output rows skips its GEMM (zeros).
    constexpr bool FULL = KQ > 0;
    const int nkb1 = FULL ? T : (m + 15) / 16, nkb2 = FULL ? T : (n + 15) / 16;  // k-blocks of each GEMM (<= T)
    const int kq1 = FULL ? KQ : (m - 16 * (nkb1 - 1) + 3) / 4, kq2 = FULL ? KQ : (n - 16 * (nkb2 - 1) + 3) / 4;
    const bool on1 = FULL || 16 * t < n, on2 = FULL || 16 * t < m;
    const int voff_r = voff - 1024;  // helper: the receiver's tile t - 1 (Handoff)
    int hgen = 0;                    // hand-off generation, counted alike by helper and receiver
    float gmx = 0.0f;                // max |g| over the rows this lane loads (gmax_part)
    // 16-B vector state I/O (rows4 / rows4_store) when every row start is 16-B aligned (uniform)
    const bool vec_io = ((n | m | (int)a.ld_gP | (int)a.ld_g) & 3) == 0 && n >= 4 && m >= 4 &&
                        ((reinterpret_cast<size_t>(a.z) | reinterpret_cast<size_t>(a.gP) |
                          reinterpret_cast<size_t>(a.y) | reinterpret_cast<size_t>(a.g) |
                          reinterpret_cast<size_t>(a.wc) | reinterpret_cast<size_t>(a.uc)) & 15) == 0;

    for (int it = blockIdx.x; it < items; it += gridDim.x) {
        GPAD_PSTAMP(0);
        // columns still running, bit 16 pp + c for panel pp of this item: the same word in every
        // wave (derived from uniform values and LDS), so the test needs no vote barrier
        unsigned live = 0u;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            if (pp == 1 && !pair) break;
            const int left = count - 16 * (pair ? 2 * it + pp : it);
            const int cnt = left < 0 ? 0 : (left > 16 ? 16 : left);
            live |= ((1u << cnt) - 1u) << (16 * pp);
        }
        bool act[Q];
        int inst[Q];
        float z[Q][4], y[Q][4], u[Q][4];
        // The columns' state, so that the loads are in flight together (r05): the instance of each
        // column (one load), then per panel every operand load unconditionally at clamped addresses
        // (an inactive column reads instance 0, a padding row the last real row), then the selects.  Loading under per-row / per-column conditions made the compiler branch around
        // every load and drain vmcnt at the joins -- 8-18 dependent round trips to memory per wave,
        // 10-23 us per phase start (profiles/r05_phase_*.txt).
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            act[q] = false;
            inst[q] = 0;
            if constexpr (NU == 0) continue;
            const int k = 16 * (pair ? 2 * it + p0 + q : it) + c;
            act[q] = k < count;
            KernArgs& A = kargs();
            inst[q] = A.idx_in ? A.idx_in[act[q] ? k : 0] : (act[q] ? k : 0);
        }
        if constexpr (NU > 0) {
            KernArgs& A = kargs();  // (gpad_internal.h: the row pointers are not kept across the loop)
            const float beta0 = A.beta[0];
            const bool vec = vec_io;
            // vec (r06): the operands arrive by LDS-DMA (rows4_dma), every panel's in flight at once:
            // z, gP, y, g into the wave's (panel, tile) blocks of Zh, Gp, Wl, Pd, then (carried
            // phases) wc, uc into those of Zh, Wl once the first four are read.  The final Gp / Pd /
            // Wl / Zh rows are stored after the reads of the same blocks (LDS is in order per wave).
            // Before: each operand's load waited behind the previous one's LDS transpose, four to
            // six round trips to memory per panel (profiles/r05_phase_stamps_vecio_*.txt: 14-30
            // kcycles to the first barrier).
            if (vec) {
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    int ln = lane;
                    asm volatile("" : "+v"(ln));  // (offsets formed per item, not kept across the item loop)
                    const size_t bc = (size_t)__shfl(inst[q], ln >> 2);
                    const int pq = p0 + q;
                    rows4_dma(A.z + bc * n, t, n, ln, &L.Zh[pq][64 * t]);
                    rows4_dma(A.gP + bc * A.ld_gP, t, n, ln, &L.Gp[pq][64 * t]);
                    rows4_dma(A.y + bc * m, t, m, ln, &L.Wl[pq][64 * t]);
                    rows4_dma(A.g + bc * A.ld_g, t, m, ln, &L.Pd[pq][64 * t]);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                float zl[4], gpl[4], yl[4], gl[4];
                int ln = lane;
                asm volatile("" : "+v"(ln));
                const size_t b = (size_t)inst[q];
                const int pq = p0 + q;
                if (vec) {
                    rows4_rd(&L.Zh[pq][64 * t], ln, zl);
                    rows4_rd(&L.Gp[pq][64 * t], ln, gpl);
                    rows4_rd(&L.Wl[pq][64 * t], ln, yl);
                    rows4_rd(&L.Pd[pq][64 * t], ln, gl);
                } else {
                    rows4(A.z + b * n, t, n, ln, zl);
                    rows4(A.gP + b * A.ld_gP, t, n, ln, gpl);
                    rows4(A.y + b * m, t, m, ln, yl);
                    rows4(A.g + b * A.ld_g, t, m, ln, gl);
                }
                float gp[4], pd[4], wv[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * t + 4 * r + j;
                    const bool okn = act[q] && i < n, okm = act[q] && i < m;
                    z[q][r] = okn ? zl[r] : 0.0f;
                    gp[r] = okn ? gpl[r] : 0.0f;
                    y[q][r] = okm ? yl[r] : 0.0f;
                    const float gr = okm ? gl[r] : 0.0f;
                    pd[r] = (float)(A.gscale * (double)gr);
                    gmx = absmax_nan(gmx, gr);
                    // w_0 = y_0 + beta_0 (y_0 - y_{-1}), y_{-1} = y_0 (fresh; carried: wc below)
                    wv[r] = __builtin_fmaf(beta0, y[q][r] - y[q][r], y[q][r]);
                    u[q][r] = 0.0f;
                }
                L.Gp[pq][slot] = make_float4(gp[0], gp[1], gp[2], gp[3]);
                L.Pd[pq][slot] = make_float4(pd[0], pd[1], pd[2], pd[3]);
                if (fresh) {
                    L.Wl[pq][slot] = make_float4(wv[0], wv[1], wv[2], wv[3]);
                    if (use_tol) L.Zh[pq][slot] = make_float4(z[q][0], z[q][1], z[q][2], z[q][3]);
                } else if (vec) {  // round two: wc, uc into the blocks just read
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    const size_t bc = (size_t)__shfl(inst[q], ln >> 2);
                    rows4_dma(A.wc + bc * m, t, m, ln, &L.Zh[pq][64 * t]);
                    if (use_tol) rows4_dma(A.uc + bc * m, t, m, ln, &L.Wl[pq][64 * t]);
                }
            }
            if (!fresh) {
                if (vec) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __builtin_amdgcn_wave_barrier();
                }
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    float wl[4], ul[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                    int ln = lane;
                    asm volatile("" : "+v"(ln));
                    const size_t b = (size_t)inst[q];
                    const int pq = p0 + q;
                    if (vec) {
                        rows4_rd(&L.Zh[pq][64 * t], ln, wl);
                        if (use_tol) rows4_rd(&L.Wl[pq][64 * t], ln, ul);
                    } else {
                        rows4(A.wc + b * m, t, m, ln, wl);
                        if (use_tol) rows4(A.uc + b * m, t, m, ln, ul);
                    }
                    float wv[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const bool okm = act[q] && 16 * t + 4 * r + j < m;
                        wv[r] = okm ? wl[r] : 0.0f;
                        u[q][r] = okm ? ul[r] : 0.0f;
                    }
                    L.Wl[pq][slot] = make_float4(wv[0], wv[1], wv[2], wv[3]);
                }
            }
        }
#ifdef GPAD_STAMP
        if constexpr (NU > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's state is in
#endif
        GPAD_PSTAMP(1);
        if (fresh && use_tol) {  // u = G_L z_{-1} -- zero, and no GEMM, when every z_{-1} is zero
            // (a cold start: every chain step fma(G_L, 0, +0) gives +0, so u = +0 exactly)
            bool nz = false;
            if constexpr (NU > 0) {
#pragma unroll
                for (int q = 0; q < Q; ++q)
#pragma unroll
                    for (int r = 0; r < 4; ++r) nz = nz || z[q][r] != 0.0f;
            }
            const bool wnz = __ballot(nz) != 0ull;
            if (lane == 0) L.znz[threadIdx.x >> 6] = wnz ? 1 : 0;
            __syncthreads();
            int anynz = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) anynz |= L.znz[i];
            if constexpr (NU > 0) {
                if (anynz) {
                    f32x4 c0, c1;
                    panel_gemm2<T, NU == 2>(PA2, L.Zh[p0], L.Zh[NU == 2 ? 1 : p0], voff, lane, c0, c1);
#pragma unroll
                    for (int r = 0; r < 4; ++r) u[0][r] = c0[r];
                    if constexpr (NU == 2) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) u[Q - 1][r] = c1[r];
                    }
                }
            }
        }
        __syncthreads();

        // A ring depth: doubles 1 block ahead, singles 2 (deeper rings measured within noise,
        // profiles/r05_a_ring_depth_ab.txt); a relay piece prefetches its whole first piece
        constexpr int PD = NU == 2 ? 1 : (ROLE == 3 ? Handoff<T>::R1 : 2);
        float4 ap[PD];  // A blocks of the next GEMM, in flight across the barrier before it
        float4 aph[PD];  // helper / relay: the piece's first blocks
        auto prefetch = [&](__amdgpu_buffer_rsrc_t PA) {
            if constexpr (ROLE == 2) panel_a_prefetch_from<T, PD>(PA, voff, ap, KB0);
            else if constexpr (NU > 0) panel_a_prefetch<T, PD>(PA, voff, ap);
            if constexpr (ROLE == 1) panel_a_prefetch<T, PD>(PA, voff_r, aph);
            if constexpr (ROLE == 3) panel_a_prefetch_from<T, PD>(PA, voff, aph, KB0);
        };
        GPAD_PSTAMP(2);
        prefetch(PA1);
        int v = a.v_begin;
        GPAD_STAMP_DECL
        int kc = K - v % K;  // iterations to the next test: chk <=> v % K == 0 (a countdown, no division)
        float th = a.theta[v], bn = a.beta[v + 1];
        while (true) {
            GPAD_STAMP_AT(0);  // (before the schedule's scalar loads, which a later s_memtime queues behind)
            const float th_next = a.theta[v + 1], bn_next = a.beta[v + 2];
            ++v;
            const bool chk = use_tol && --kc == 0;
            if (kc == 0) kc = K;
            const float omt = 1.0f - th;
            // ---- GEMM 1 + epilogue: zhat = -ML w - g_P (8b), z = (1-th) z + th zhat (8c) ----
            if constexpr (NU > 0) {
                f32x4 acc[2];
                ++hgen;
                if constexpr (ROLE == 1)
                    handoff_piece<T, PD, KB0, KB1, PRIO, DROP>(L, PA1, L.Wl[p0], voff_r, lane, aph, hs, hgen,
                                                               GPAD_STAMP_PTR(6));
                if constexpr (ROLE == 2)
                    handoff_take<T, PD, KB0, PRIO>(L, PA1, L.Wl[p0], voff, lane, ap, hs, hgen, kq1, acc[0],
                                                   GPAD_STAMP_PTR(6));
                else if (on1 && nkb1 == T)
                    panel_gemm3<T, NU == 2, PD>(PA1, L.Wl[p0], L.Wl[NU == 2 ? 1 : p0], voff, lane, acc[0], acc[1],
                                                ap, kq1);
                else if (on1)
                    panel_gemm_rt<T, NU == 2, PD>(PA1, L.Wl[p0], L.Wl[NU == 2 ? 1 : p0], voff, lane, acc[0],
                                                   acc[1], ap, nkb1, kq1);
                else {
                    GPAD_PRELUDE_LO();
                    acc[0] = acc[1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                }
                GPAD_STAMP_AT(1);
                prefetch(PA2);
                float4 g4[Q];
#pragma unroll
                for (int q = 0; q < Q; ++q) g4[q] = L.Gp[p0 + q][slot];
                const f32x2 th2 = f2(th, th), omt2 = f2(omt, omt);
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const f32x2 h0 = f2(acc[q][0], acc[q][1]) - f2(g4[q].x, g4[q].y);
                    const f32x2 h1 = f2(acc[q][2], acc[q][3]) - f2(g4[q].z, g4[q].w);
                    L.Zh[p0 + q][slot] = make_float4(h0.x, h0.y, h1.x, h1.y);
                    // 8c on every column (see the epilogue note below)
                    const f32x2 z0 = pk_fma(omt2, f2(z[q][0], z[q][1]), th2 * h0);
                    const f32x2 z1 = pk_fma(omt2, f2(z[q][2], z[q][3]), th2 * h1);
                    z[q][0] = z0.x;
                    z[q][1] = z0.y;
                    z[q][2] = z1.x;
                    z[q][3] = z1.y;
                }
            } else if constexpr (ROLE == 3) {
                ++hgen;
                handoff_piece<T, PD, KB0, KB1, PRIO, DROP>(L, PA1, L.Wl[p0], voff, lane, aph, hs, hgen,
                                                           GPAD_STAMP_PTR(6));
                prefetch(PA2);
            } else {
                GPAD_PRELUDE_LO();  // (a wave with no chain: the window of the invariant ends here)
            }
            GPAD_STAMP_AT(2);
            GPAD_PRELUDE_HI();
            __syncthreads();
            GPAD_STAMP_AT(3);
            // ---- GEMM 2 + epilogue: y+ = [w + G_L zhat + p_D]+ (8d), next w (8a) ----------
            float violz[Q], violh[Q], wmin[Q], magh[Q];
            double gap[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                violz[q] = violh[q] = -INFINITY;
                wmin[q] = INFINITY;
                magh[q] = 0.0f;
                gap[q] = 0.0;
            }
            if constexpr (NU > 0) {
                f32x4 acc[2];
                ++hgen;
                if constexpr (ROLE == 1)
                    handoff_piece<T, PD, KB0, KB1, PRIO, DROP>(L, PA2, L.Zh[p0], voff_r, lane, aph, hs, hgen,
                                                               GPAD_STAMP_PTR(7));
                if constexpr (ROLE == 2)
                    handoff_take<T, PD, KB0, PRIO>(L, PA2, L.Zh[p0], voff, lane, ap, hs, hgen, kq2, acc[0],
                                                   GPAD_STAMP_PTR(7));
                else if (on2 && nkb2 == T)
                    panel_gemm3<T, NU == 2, PD>(PA2, L.Zh[p0], L.Zh[NU == 2 ? 1 : p0], voff, lane, acc[0], acc[1],
                                                ap, kq2);
                else if (on2)
                    panel_gemm_rt<T, NU == 2, PD>(PA2, L.Zh[p0], L.Zh[NU == 2 ? 1 : p0], voff, lane, acc[0],
                                                   acc[1], ap, nkb2, kq2);
                else {
                    GPAD_PRELUDE_LO();
                    acc[0] = acc[1] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                }
                GPAD_STAMP_AT(4);
                prefetch(PA1);
                // (reading these LDS operands before the GEMM measured no faster: profiles/r02_epilogue_ab.txt)
                float4 w4[Q], p4[Q];
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    w4[q] = L.Wl[p0 + q][slot];
                    p4[q] = L.Pd[p0 + q][slot];
                }
                // The state updates run on every column, packed two rows per instruction: a
                // finished (or padding) column's z, y, u and w are never read again -- its results
                // left at the test that finished it, and MFMA output column c depends on B column c
                // only -- so the per-element masks of the active columns are not needed.  This
                // epilogue sits between the GEMM and the barrier on every SIMD at once; packing
                // halves its VALU issue: C4 to eps +1.3-1.5 % (profiles/r02_epilogue_ab.txt).
                const f32x2 th2 = f2(th, th), omt2 = f2(omt, omt), bn2 = f2(bn, bn), half2 = f2(0.5f, 0.5f);
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const f32x2 c0 = f2(acc[q][0], acc[q][1]), c1 = f2(acc[q][2], acc[q][3]);
                    const f32x2 s0 = (f2(w4[q].x, w4[q].y) + f2(p4[q].x, p4[q].y)) + c0;
                    const f32x2 s1 = (f2(w4[q].z, w4[q].w) + f2(p4[q].z, p4[q].w)) + c1;
                    const f32x2 y0 = f2(__builtin_fabsf(s0.x) + s0.x, __builtin_fabsf(s0.y) + s0.y) * half2;
                    const f32x2 y1 = f2(__builtin_fabsf(s1.x) + s1.x, __builtin_fabsf(s1.y) + s1.y) * half2;
                    const f32x2 n0 = pk_fma(bn2, y0 - f2(y[q][0], y[q][1]), y0);
                    const f32x2 n1 = pk_fma(bn2, y1 - f2(y[q][2], y[q][3]), y1);
                    L.Wl[p0 + q][slot] = make_float4(n0.x, n0.y, n1.x, n1.y);
                    y[q][0] = y0.x;
                    y[q][1] = y0.y;
                    y[q][2] = y1.x;
                    y[q][3] = y1.y;
                    if (use_tol) {
                        const f32x2 u0 = pk_fma(omt2, f2(u[q][0], u[q][1]), th2 * c0);
                        const f32x2 u1 = pk_fma(omt2, f2(u[q][2], u[q][3]), th2 * c1);
                        u[q][0] = u0.x;
                        u[q][1] = u0.y;
                        u[q][2] = u1.x;
                        u[q][3] = u1.y;
                        if (chk && act[q]) {
                            const float wv[4] = {w4[q].x, w4[q].y, w4[q].z, w4[q].w};
                            const float pd[4] = {p4[q].x, p4[q].y, p4[q].z, p4[q].w};
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                if ((16 * t + 4 * r + j) < m) {
                                    const float cv = acc[q][r];
                                    const float tt = cv + pd[r];
                                    violh[q] = fmaxf(violh[q], tt);
                                    magh[q] = fmaxf(magh[q], __builtin_fabsf(cv) + __builtin_fabsf(pd[r]));
                                    wmin[q] = fminf(wmin[q], wv[r]);
                                    gap[q] -= (double)wv[r] * (double)tt;
                                    violz[q] = fmaxf(violz[q], u[q][r] + pd[r]);
                                }
                            }
                        }
                    }
                    if (chk) {  // this tile's per-column partials of the test -> LDS
                        // lane groups j (xor 16, 32) on the VALU (gpad_chain.h)
                        violz[q] = bfly<32>(bfly<16>(violz[q], OpMax{}), OpMax{});
                        violh[q] = bfly<32>(bfly<16>(violh[q], OpMax{}), OpMax{});
                        magh[q] = bfly<32>(bfly<16>(magh[q], OpMax{}), OpMax{});
                        wmin[q] = bfly<32>(bfly<16>(wmin[q], OpMin{}), OpMin{});
                        gap[q] = bfly<32>(bfly<16>(gap[q], OpAdd{}), OpAdd{});
                        if (j == 0) {
                            PanelSlot2& S = L.slots[p0 + q][t];
                            S.f[c] = make_float4(violz[q], violh[q], magh[q], wmin[q]);
                            S.gap[c] = gap[q];
                        }
                    }
                }
            } else if constexpr (ROLE == 3) {
                ++hgen;
                handoff_piece<T, PD, KB0, KB1, PRIO, DROP>(L, PA2, L.Zh[p0], voff, lane, aph, hs, hgen,
                                                           GPAD_STAMP_PTR(7));
                prefetch(PA1);
            } else {
                GPAD_PRELUDE_LO();
            }
            th = th_next;
            bn = bn_next;
            GPAD_STAMP_AT(5);
            GPAD_PRELUDE_HI();
            __syncthreads();
            GPAD_STAMP_FLUSH();
            if (!chk && v < a.v_end) continue;

            // ---- Algorithm 1 test per column: every wave reduces the tile partials of all the
            // item's columns (lane 16 pp + cc <-> panel pp, column cc) and votes by ballot, so the
            // outcome is uniform across the workgroup without a second barrier ---------------------
            GPAD_PSTAMP_END(6);
            unsigned m1 = 0u, m2 = 0u;
            bool zh_out = true;  // this iteration's zhat still in L.Zh (no verification GEMM ran)
            if (chk) {
                int st1 = 0;
                float4 red;
                double gq;
                panel2_reduce<T>(L.slots, lane, red, gq);
                // the pair layout re-reads the test's doubles here (kargs) rather than keeping them
                // in SGPRs across the loop: fewer spilled SGPRs reloaded in its loop (the one-panel
                // roles keep them: re-reading moved their spills to scratch)
                double tL, ttol, ttg;
                if constexpr (KQ > 0) {
                    KernArgs& A = kargs();
                    tL = A.L;
                    ttol = A.tol;
                    ttg = A.tol_gap;
                } else {
                    tL = a.L;
                    ttol = a.tol;
                    ttg = a.tol_gap;
                }
                if (lane < 32 && ((live >> lane) & 1u))
                    st1 = ((double)red.x * tL <= ttol ? 1 : 0) |
                          ((viol_ok((double)red.y, (double)red.z, tL, ttol, ViolMargin<float>::value) &&
                            (red.w >= 0.0f) && (gq * tL <= ttg)) ? 2 : 0);
                const unsigned mA = (unsigned)__ballot(st1 & 1);
                m2 = (unsigned)__ballot(st1 & 2);
                GPAD_PSTAMP_END(7);
                if (mA) {  // (A) nominated for some column of the item: G_L z of both panels
                    zh_out = false;
                    if constexpr (NU > 0) {
#pragma unroll
                        for (int q = 0; q < Q; ++q) {
                            const int bit = 16 * (p0 + q) + c;
                            if (act[q] && ((m2 >> bit) & 1u)) {  // test (B)'s zhat out before z replaces it
                                const float4 h4 = L.Zh[p0 + q][slot];
                                const float zh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    const int i = 16 * t + 4 * r + j;
                                    if (i < n) a.z[(size_t)inst[q] * n + i] = zh[r];
                                }
                            }
                            L.Zh[p0 + q][slot] = make_float4(z[q][0], z[q][1], z[q][2], z[q][3]);
                        }
                    }
                    __syncthreads();
                    if constexpr (NU > 0) {
                        f32x4 cz[2];
                        panel_gemm2<T, NU == 2>(PA2, L.Zh[p0], L.Zh[NU == 2 ? 1 : p0], voff, lane, cz[0], cz[1]);
#pragma unroll
                        for (int q = 0; q < Q; ++q) {
                            const bool nom = act[q] && ((mA >> (16 * (p0 + q) + c)) & 1u);
                            const float4 p4 = L.Pd[p0 + q][slot];
                            const float pd[4] = {p4.x, p4.y, p4.z, p4.w};
                            float vc = -INFINITY, mc = 0.0f;
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                if (nom && (16 * t + 4 * r + j) < m) {
                                    u[q][r] = cz[q][r];  // the recursion restarts from the direct value
                                    vc = fmaxf(vc, cz[q][r] + pd[r]);
                                    mc = fmaxf(mc, __builtin_fabsf(cz[q][r]) + __builtin_fabsf(pd[r]));
                                }
                            }
                            vc = bfly<32>(bfly<16>(vc, OpMax{}), OpMax{});
                            mc = bfly<32>(bfly<16>(mc, OpMax{}), OpMax{});
                            if (j == 0)  // the stage-1 reads of every wave precede the barrier above
                                L.slots[p0 + q][t].f[c] = make_float4(vc, vc, mc, INFINITY);
                        }
                    }
                    __syncthreads();
                    bool ver = false;
                    float4 vred;
                    double vgap;
                    panel2_reduce<T>(L.slots, lane, vred, vgap);
                    if (lane < 32 && ((mA >> lane) & 1u))
                        ver = viol_ok((double)vred.x, (double)vred.z, tL, ttol, ViolMargin<float>::value);
                    m1 = (unsigned)__ballot(ver);
                    m2 &= ~m1;
                }
                GPAD_PSTAMP_END(8);
            }
            // ---- finished columns: results out ---------------------------------------------
            if constexpr (NU > 0) {
                // values and row pointers first, the stores after (see the phase-end park below)
                bool out[Q];
                int cd[Q];
                float zo[Q][4];
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const int bit = 16 * (p0 + q) + c;
                    cd[q] = ((m1 >> bit) & 1u) ? 1 : (((m2 >> bit) & 1u) ? 2 : 0);
                    out[q] = act[q] && (cd[q] != 0 || v >= N);
                    const float4 h4 = L.Zh[p0 + q][slot];
                    const bool use_zh = cd[q] == 2;
                    zo[q][0] = use_zh ? h4.x : z[q][0];
                    zo[q][1] = use_zh ? h4.y : z[q][1];
                    zo[q][2] = use_zh ? h4.z : z[q][2];
                    zo[q][3] = use_zh ? h4.w : z[q][3];
                }
#pragma unroll
                for (int q = 0; q < Q; ++q) {  // (Zh's block is free again: the rows4 transpose)
                    int iq = inst[q], ln = lane;
                    asm volatile("" : "+v"(iq), "+v"(ln));  // (no hoisted row pointers / offsets: rows4 note)
                    const size_t b = (size_t)iq;
                    float* const st = reinterpret_cast<float*>(&L.Zh[p0 + q][64 * t]);
                    const bool zw = cd[q] != 2 || zh_out;  // (B)'s zhat already out before (A)'s GEMM
                    KernArgs& A = kargs();
                    rows4_store(A.z + b * n, t, n, vec_io, st, ln, zo[q], out[q] && zw);
                    rows4_store(A.y + b * m, t, m, vec_io, st, ln, y[q], out[q]);
                    if (out[q]) {
                        if (t == 0 && j == 0) {
                            A.iters[iq] = v;
                            A.conv[iq] = cd[q];
                        }
                        act[q] = false;
                    }
                }
            }
            GPAD_PSTAMP_END(9);
            live &= ~(m1 | m2);
            if (v >= N) live = 0u;
            if (v >= a.v_end || live == 0u) break;
        }
        GPAD_PRELUDE_LO();  // (the loop's last barrier left every wave at priority 2)
        // ---- phase end: park the survivors -----------------------------------------------
        GPAD_PSTAMP(3);
        if constexpr (NU > 0) {
            if (carry) {
                // the stores after every value they take (r05): vmcnt counts stores on gfx9, so a
                // spill reload between stores would wait for all the stores before it
                bool pk[Q];
                float wv[Q][4];
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    pk[q] = act[q] && v >= a.v_end;
                    const float4 w4 = L.Wl[p0 + q][slot];
                    wv[q][0] = w4.x;
                    wv[q][1] = w4.y;
                    wv[q][2] = w4.z;
                    wv[q][3] = w4.w;
                }
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    int iq = inst[q], ln = lane;
                    asm volatile("" : "+v"(iq), "+v"(ln));  // (no hoisted row pointers / offsets: rows4 note)
                    const size_t b = (size_t)iq;
                    float* const st = reinterpret_cast<float*>(&L.Zh[p0 + q][64 * t]);
                    KernArgs& A = kargs();
                    rows4_store(A.z + b * n, t, n, vec_io, st, ln, z[q], pk[q]);
                    rows4_store(A.y + b * m, t, m, vec_io, st, ln, y[q], pk[q]);
                    rows4_store(A.wc + b * m, t, m, vec_io, st, ln, wv[q], pk[q]);
                    if (use_tol) rows4_store(A.uc + b * m, t, m, vec_io, st, ln, u[q], pk[q]);
                }
                if (t == 0) {  // the tile-0 owner of each panel lists its survivors
#pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        int iq = inst[q], ln = lane;
                        asm volatile("" : "+v"(iq), "+v"(ln));
                        list_survivors(kargs(), pair ? 2 * it + p0 + q : it, pk[q], iq, ln, ln >> 4);
                    }
                }
            }
        }
        GPAD_PSTAMP(4);
        __syncthreads();
        GPAD_PSTAMP(5);
    }
    if (a.gmax_part) {  // this wave's max |g| -> L.gred (reduced by the kernel at exit)
        for (int o = 32; o > 0; o >>= 1) gmx = absmax_nan(gmx, __shfl_xor(gmx, o, 64));
        if (lane == 0) L.gred[threadIdx.x >> 6] = gmx;
    }
}

// KQ > 0 (panel2_run): the pair layout's compile-time chain shape.  The one-panel layout runs the
// runtime-shape code (KQ = 0) in every instantiation: specialised, its relay measured slower
// (6.16 vs 5.98 us per iteration at 4 panels, profiles/r03_single_mode_ab.txt).  DROP: the
// test-only fault-injection instantiation (GPAD_OPT_DEBUG_DROP_HANDOFF), launched instead of the
// product kernel only while that option is set, so the product kernel carries no trace of it.
template <int T, int KQ, bool DROP = false>
__global__ __launch_bounds__(1024) void gpad_panel2_kernel(SolveArgs<float> a) {
    static_assert(T > 8 && T <= 16, "panel pairs need 8 < T <= 16");
    constexpr int D = 2 * T - 16;  // double waves
    __shared__ Panel2Lds<T> L;
    const int count = a.count_in ? __builtin_amdgcn_readfirstlane(*a.count_in) : a.batch;
    if (a.count_in && count <= a.fin_thresh) return;  // the finisher has them
    const int panels = (count + 15) / 16;
    const bool pair = panels > (int)gridDim.x;
    // Role index.  The SIMD issues MFMAs oldest wave first, so a role's wave index sets its share
    // of the SIMD while the SIMD is contended.  One-panel layout: the roles are dealt from the
    // last wave down, so the relay pieces of tile T-1 (roles T, T+1) and its receiver run on the
    // oldest waves of their SIMDs and the sequential relay is not starved -- 5.92 -> 5.71 us per
    // iteration at one panel per CU, 6.93 -> 6.75 at 4096 (r03_wave_order_ab.txt).  Pairs: the
    // two hand-off receivers (roles 12, 13, SIMDs 0, 1) swap waves with the doubles of roles 8, 9,
    // so a receiver's chain -- which starts only when its piece arrives -- is not the youngest on
    // its SIMD: -1 to -3 % per pair iteration, C4 -0.2 to -1.0 % (r03_pair_perm_ab.txt; helpers
    // older than the singles, receivers oldest, or both, measured no better).
    const int w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = pair ? ((w0 >> 1) == 4 ? w0 + 4 : ((w0 >> 1) == 6 ? w0 - 4 : w0)) : 15 - w0;
    const int items = pair ? (panels + 1) / 2 : panels;
    // hand-off (Handoff): both GEMMs run full-length chains on tiles T-2 and T-1
    const bool ho = Handoff<T>::on && (KQ > 0 || (16 * (T - 1) < a.n && 16 * (T - 1) < a.m &&
                                                  (a.m + 15) / 16 == T && (a.n + 15) / 16 == T));
    if (threadIdx.x < 6) L.hflag[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        L.herr = 0;
        L.hdrop = DROP && blockIdx.x == 0;  // tests: workgroup 0 drops one post
    }
    if (threadIdx.x < 16) L.gred[threadIdx.x] = 0.0f;
    if (blockIdx.x == 0) {  // (r06: instead of memset dispatches before the solve)
        if (a.zero_w)
            for (int i = threadIdx.x; i < a.zero_n; i += blockDim.x) a.zero_w[i] = 0;
        if (a.gmax_part && a.v_begin == 0)  // the slots no workgroup of this launch writes
            for (int i = gridDim.x + threadIdx.x; i < kAbsmaxMaxBlocks; i += blockDim.x) a.gmax_part[i] = 0.0;
    }
    __syncthreads();
    if constexpr (Handoff<T>::on) {
        using H = Handoff<T>;
        if (pair) {  // waves 12, 13 (SIMDs 0, 1; tile T-2) receive from 14, 15 (SIMDs 2, 3; tile T-1)
            if (w < D) panel2_run<T, 2, 0, 0, 0, false, KQ, DROP>(a, L, w, 0, true, items, count);
            else if (ho && w >= 14)
                panel2_run<T, 1, 1, 0, H::S, false, KQ, DROP>(a, L, T - 1, w & 1, true, items, count, HoSlots{-1, w & 1});
            else if (ho && w >= 12)
                panel2_run<T, 1, 2, H::S, 0, false, KQ, DROP>(a, L, T - 2, w & 1, true, items, count, HoSlots{w & 1, -1});
            else panel2_run<T, 1, 0, 0, 0, false, KQ, DROP>(a, L, D + ((w - D) >> 1), (w - D) & 1, true, items, count);
        } else {  // tile T-1 as a relay: waves T -> T+1 -> T-1
            if constexpr (!H::relay) {
                if (w < T) panel2_run<T, 1, 0, 0, 0, false, 0, DROP>(a, L, w, 0, false, items, count);
                else panel2_run<T, 0, 0, 0, 0, false, 0, DROP>(a, L, 0, 0, false, items, count);
            } else if (ho && w == T - 1) panel2_run<T, 1, 2, H::R2, 0, true, 0, DROP>(a, L, w, 0, false, items, count, HoSlots{1, -1});
            else if (ho && w == T)
                panel2_run<T, 0, 3, 0, H::R1, true, 0, DROP>(a, L, T - 1, 0, false, items, count, HoSlots{-1, 0});
            else if (ho && w == T + 1)
                panel2_run<T, 0, 3, H::R1, H::R2, true, 0, DROP>(a, L, T - 1, 0, false, items, count, HoSlots{0, 1});
            else if (w < T)
                panel2_run<T, 1, 0, 0, 0, false, 0, DROP>(a, L, w, 0, false, items, count);
            else panel2_run<T, 0, 0, 0, 0, false, 0, DROP>(a, L, 0, 0, false, items, count);
        }
    } else if (pair) {
        if (w < D) panel2_run<T, 2, 0, 0, 0, false, KQ, DROP>(a, L, w, 0, true, items, count);
        else panel2_run<T, 1, 0, 0, 0, false, KQ, DROP>(a, L, D + ((w - D) >> 1), (w - D) & 1, true, items, count);
    } else {
        if (w < T) panel2_run<T, 1, 0, 0, 0, false, 0, DROP>(a, L, w, 0, false, items, count);
        else panel2_run<T, 0, 0, 0, 0, false, 0, DROP>(a, L, 0, 0, false, items, count);
    }
    if (Handoff<T>::on || a.gmax_part) {
        __syncthreads();
        // an expired hand-off or dataflow wait fails the run (GPAD_ERR_DEVICE)
        if (Handoff<T>::on && threadIdx.x == 0 && L.herr) atomicOr(a.err, kDevErrHandoff);
        if (a.gmax_part && threadIdx.x == 0) {  // the run's max |g|: this workgroup's slot
            float g = 0.0f;
            for (int i = 0; i < 16; ++i) g = absmax_nan(g, L.gred[i]);
            // the run's first launch stores (gmax_part note, gpad_internal.h), later phases max in
            a.gmax_part[blockIdx.x] = a.v_begin == 0 ? (double)g : absmax_nan(a.gmax_part[blockIdx.x], (double)g);
        }
    }
}

// schedule parameters shared by the launcher and the host's phase hint
int panel_phase_len(int check_every, const Tuning* t) {
    // a multiple of the test period (phases end right after a test); default four tests
    int len = 4 * check_every;
    if (t && t->phase_len > 0) len = t->phase_len;
    return ((len + check_every - 1) / check_every) * check_every;
}

int panel_fin_thresh(int n, int m, int num_cus, const Tuning* t) {
    // the tail of a phased solve (survivors <= 2 per CU) goes to the latency kernel: one
    // instance per workgroup at ~1/6 of a panel's iteration time (when n, m fit it); measured
    // on C4: 2/CU 5.42e8 it/s, 4/CU 5.35e8, 8/CU 5.35e8, no finisher 5.04e8
    int f = resident_supported(n, m) ? 2 * num_cus : 0;
    if (t && t->finish_thresh >= 0 && f) f = t->finish_thresh;
    return f;
}

// ---------------------------------------------------------------------------------------------
// Phase plan from the previous solve of the same handle.
//
// A phased solve's cost is set by where its phase boundaries fall against the survival curve
// s(v) = #(instances still running past iteration v): a phase [v0, v1) costs (v1 - v0) panel
// iterations whose time depends only on how many panels s(v0) fills (columns that converge
// inside the phase idle until it ends), plus the launch, the carry traffic and the seed
// product; handing the survivors to the resident finisher at v costs the longest remaining
// solve at the latency kernel's iteration time, or the remaining instance-iterations at its
// throughput, whichever is larger.  Given s(v) from the previous solve (receding-horizon and
// scenario batches repeat it closely), a dynamic programme over the test-aligned boundaries
// picks the cheapest schedule.  The plan only moves launch boundaries: every column runs the
// same global iterations with the same tests whatever the schedule, so results are bit-identical
// (tests/test_gpu_parity.py::test_panel_phase_plan_reuse_bitexact).
//
// Cost model (us; constants from profiles/r01_timeline.txt and profiles/r01_microbench.jsonl):
//   panel iteration  = (busiest SIMD's MFMA chains) x t_chain,  t_chain = 0.055 (kb1 + kb2) + 0.2
//                      single panels: ceil(T/4) chains, pairs: ceil(2T/4) (2T/4 on the hand-off
//                      shapes, r02_handoff_ab.txt: 8192 at 10.5-10.9 us), T <= 8: co-resident
//                      panels share the CU's four SIMDs
//   phase overhead   = 2 launches (finisher + panel, 5 us each) + one seed iteration
//                      + carried z, y, w, u (16 (n + m) bytes per survivor at 5 TB/s)
//   finisher         = 1.56 t_res L + 0.70 t_res W / CUs + 2 launches,  t_res = 0.0021 (n + m) + 0.38,
//                      L the longest remaining solve, W the remaining instance-iterations (r06 refit:
//                      latency and work add, see PlanModel::finisher).
namespace {
struct PlanModel {
    int T, n, m, num_cus, grid;
    bool handoff;  // gpad_panel2_kernel's hand-off shapes (Handoff)
    bool relay;    // ... and its one-panel relay (T = 9, 13)
    static constexpr double kFinLat = 1.56;     // finisher: us per remaining iteration of the longest, / t_res
    static constexpr double kFinWork = 0.70;    // finisher: us per instance-iteration per CU, / t_res
    static constexpr double kCarryBw = 5e6;     // carried state, bytes per us
    double t_chain, t_res, t_launch = 5.0;
    double iter_time(long long panels) const {
        if (panels <= 0) return 0.0;
        double chains;
        if (T > 8) {
            if (panels <= grid) {
                // the one-panel relay (Handoff): 4 -> 3.36 chains on the busiest SIMD, measured
                // 6.02 -> 5.65-5.75 us per iteration at one CU (r02_relay_ab.txt): priced as 3.5
                chains = relay ? 3.5 : (double)((T + 3) / 4);
            } else {
                const long long pairs = (panels + 1) / 2;
                // the chain hand-off evens the pair layout's SIMD loads (7,7,6,6 -> 6.5 at T = 13)
                const double per = handoff ? 2 * T / 4.0 : (double)((2 * T + 3) / 4);
                chains = (double)((pairs + grid - 1) / grid) * per;
            }
        } else {
            const int per_cu_max = 32 / T;
            const long long rounds = (panels + (long long)grid - 1) / grid;
            const long long last = panels - (rounds - 1) * (long long)grid;
            long long q = (last + num_cus - 1) / num_cus;
            if (rounds > 1 || q > per_cu_max) q = per_cu_max;
            chains = (double)((rounds - 1) * ((per_cu_max * T + 3) / 4) + (q * T + 3) / 4);
        }
        return chains * t_chain;
    }
    double phase(int v0, int v1, long long s0) const {
        const double it = iter_time((s0 + 15) / 16);
        return 2 * t_launch + (v1 - v0 + 1) * it + (double)s0 * 16.0 * (n + m) / kCarryBw;
    }
    double finisher(int longest, long long work) const {
        // r06 refit on fresh-input C4 solves (profiles/r06_plan_refit.txt): with the queue in no
        // useful order (fresh inputs: the previous solve's counts do not rank this one's instances)
        // the longest survivor waits behind part of its CU's queue, so its latency and the CU's
        // share of the work ADD -- the duo took 341-370 us from iteration 280 (L = 110, W/CU = 181)
        // and 236-262 us from 290 (L = 90-100, W/CU = 105), where max(latency, throughput) of the
        // previous constants priced 242 / 171 us and steered ~30 % of the solves to the costlier
        // earlier takeover (+47 us per solve, profiles/r06_solve_spread.txt)
        return 2 * t_launch + kFinLat * t_res * longest + kFinWork * t_res * (double)work / num_cus;
    }
};
}  // namespace

int panel_plan(const int* iters, int batch, int n, int m, int N, int check_every, int num_cus, const Tuning* t,
               PanelPlan* out) {
    out->nph = 0;
    out->N = N;
    const int T = panel_tiles_for(n, m);
    if (!T || batch <= 0 || N <= 0 || (t && !t->plan)) return 0;
    const int K = check_every > 0 ? check_every : 1;
    int maxit = 0;
    for (int b = 0; b < batch; ++b) maxit = iters[b] > maxit ? iters[b] : maxit;
    if (maxit <= 0) return 0;
    maxit = maxit < N ? maxit : N;
    // boundaries: multiples of `step` (a multiple of the test period) up to the last iteration;
    // coarse enough that the plan fits the phase-count slots with room for the run-out phases
    const int slots = kPanelMaxPhases - 4;
    int step = K;
    while ((maxit + step - 1) / step > slots) step += K;
    const int J = (maxit + step - 1) / step;  // boundary j is iteration j*step (J*step >= maxit)
    std::vector<long long> surv(J + 1, 0), work(J + 1, 0);
    std::vector<long long> hist(maxit + 2, 0);
    for (int b = 0; b < batch; ++b) hist[iters[b] < 0 ? 0 : (iters[b] > maxit ? maxit : iters[b])]++;
    // s(v) = #(iters > v), W(v) = sum_b max(0, iters_b - v)
    std::vector<long long> s(maxit + 2, 0), W(maxit + 2, 0);
    for (int v = maxit; v >= 0; --v) {
        s[v] = s[v + 1] + hist[v + 1];
        W[v] = W[v + 1] + s[v];
    }
    for (int j = 0; j <= J; ++j) {
        const int v = j * step < maxit ? j * step : maxit;
        surv[j] = s[v];
        work[j] = W[v];
    }
    PlanModel md;
    md.T = T;
    md.n = n;
    md.m = m;
    md.num_cus = num_cus;
    md.grid = T > 8 ? num_cus : num_cus * (32 / T);
    md.handoff = (T == 9 || T == 11 || T == 13) && n > 16 * (T - 1) && m > 16 * (T - 1) &&
                 (n + 15) / 16 == T && (m + 15) / 16 == T;
    md.relay = md.handoff && (T == 9 || T == 13);
    md.t_chain = 0.055 * ((m + 15) / 16 + (n + 15) / 16) + 0.2;
    md.t_res = 0.0021 * (n + m) + 0.38;
    const bool fin_ok = resident_supported(n, m);
    // best[j]: cheapest finish from boundary j (survivors surv[j] in panels); nxt[j] = next
    // boundary (or -1: finisher takes over at j)
    std::vector<double> best(J + 1, 0.0);
    std::vector<int> nxt(J + 1, J);
    for (int j = J - 1; j >= 0; --j) {
        const int v = j * step;
        double c = 1e300;
        int arg = J;
        if (surv[j] == 0) {
            best[j] = 0.0;
            nxt[j] = J;
            continue;
        }
        if (fin_ok && j > 0) {
            c = md.finisher(maxit - v, work[j]);
            arg = -1;
        }
        for (int k = j + 1; k <= J; ++k) {
            const int v1 = k * step < maxit ? k * step : maxit;
            const double ck = md.phase(v, v1, surv[j]) + best[k];
            if (ck < c) {
                c = ck;
                arg = k;
            }
        }
        best[j] = c;
        nxt[j] = arg;
    }
    // walk the plan: ends of the panel phases, then the takeover (finisher) or run-out phase
    const int fin_default = panel_fin_thresh(n, m, num_cus, t);
    int j = 0, ph = 0;
    while (j < J && ph < slots) {
        const int k = nxt[j];
        if (k < 0) break;  // finisher at boundary j
        // a panel phase: the finisher may still take its list early when the survivors fall to
        // its default threshold -- unless the plan expects several times that many, where its
        // launch would only test and return (~5 us per boundary)
        out->fins[ph] = (j > 0 && surv[j] > 4 * (long long)fin_default) ? 0 : fin_default;
        out->ends[ph++] = k * step;
        j = k;
        if (surv[j] == 0) break;
    }
    // the phase starting at the last boundary runs to N; the finisher takes it when the survivors
    // fit its threshold, sized from the previous solve's survivors there (with margin)
    long long sj = j < J ? surv[j] : 0;
    long long thr = fin_default;
    if (fin_ok && sj > 0 && 2 * sj + 64 > thr) thr = 2 * sj + 64;
    if (thr > batch) thr = batch;
    if (ph > 0 && out->ends[ph - 1] >= N) {
        out->ends[ph - 1] = N;
    } else {
        out->fins[ph] = (int)thr;
        out->ends[ph++] = N;
    }
    out->nph = ph;
    out->cost_us = best[0];
    return ph;
}

size_t panel_work_bytes(int m, int batch) {
    // idx ping-pong [2][batch] | phase counts [kPanelMaxPhases] | finisher queue counters
    // [kPanelMaxPhases] | carried w, u
    // [batch][m] each | per-panel survivor lists: seg_idx [batch + 32], seg_cnt [batch / 16 + 2]
    // (list_survivors)
    return sizeof(int) * (2 * (size_t)batch + 2 * kPanelMaxPhases) +
           2 * sizeof(float) * (size_t)batch * m +
           sizeof(int) * ((size_t)batch + 32 + (size_t)batch / 16 + 2);
}

// Phase boundary (launch_phase_compact): the survivors the previous phase listed per panel
// (list_survivors: seg_cnt[P], seg_idx[16 P + rank]) become the dense list idx[0 .. count) of the
// next phase.  One workgroup: thread t owns a contiguous run of panels, an LDS scan of the
// per-thread totals gives each run its base, and the run's entries are copied in panel order.
//
// When the list is the finisher's (count <= fin_cur) and the previous solve's counts are known
// (pred), it is then reordered longest-predicted-first so the duo kernel's queue starts the
// longest remaining solves first (list scheduling, LPT): a counting sort on the counts (4096
// bins, larger counts share the last) -- histogram, descending exclusive scan, scatter.  The order
// inside a bin is arbitrary; results never depend on the order, only the schedule does.
constexpr int kSortMax = 8192;
constexpr int kSortBins = 4096;
// exclusive scan over 1024 threads: an inclusive scan inside each wave (six shuffles), then the 16
// wave totals through LDS -- two barriers (r06; the LDS Hillis-Steele scan before it took twenty)
__device__ __forceinline__ int block_scan_1024(int* part, int tid, int v) {
    const int lane = tid & 63, w = tid >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) part[w] = x;
    __syncthreads();
    int wb = 0;
    for (int i = 0; i < w; ++i) wb += part[i];
    __syncthreads();  // (the caller's next scan rewrites part)
    return wb + x - v;
}

constexpr int kCompactMaxPanels = 8192;  // per-panel bases in LDS up to here (131072 instances)
constexpr int kCompactU = 8;             // entries per thread and round: loads issued together
__global__ __launch_bounds__(1024) void phase_compact_kernel(const int* __restrict__ seg_cnt,
                                                             const int* __restrict__ seg_idx, const int* count_prev,
                                                             int batch, int fin_prev, int* idx, int* count_out,
                                                             const int* pred, int fin_cur) {
    __shared__ int hist[kSortBins];
    __shared__ int ids[kSortMax];
    __shared__ int part[1024];
    __shared__ int pbase[kCompactMaxPanels];
    __shared__ int pcnt[kCompactMaxPanels];
    __shared__ int total_l;
    const int tid = threadIdx.x;
    // the thread -> panel runs from the batch's panel count, so the per-panel counts load together
    // with count_prev (one round trip, not two); panels past the previous phase's count as 0
    const int pmax = (batch + 15) / 16;
    const int per = (pmax + 1023) / 1024;
    const int p0 = tid * per < pmax ? tid * per : pmax, p1 = p0 + per < pmax ? p0 + per : pmax;
    constexpr int kPer = 8;  // counts held in registers per thread (pmax <= 8192 panels)
    int cl[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) cl[u] = (per <= kPer && p0 + u < p1) ? seg_cnt[p0 + u] : 0;
    const int prev = count_prev ? *count_prev : batch;
    if (count_prev && prev <= fin_prev) {  // the finisher took the previous list: nothing was listed
        if (tid == 0) *count_out = 0;
        return;
    }
    const int panels = (prev + 15) / 16;
    const bool lds_bases = panels <= kCompactMaxPanels;
    const int q1 = p1 < panels ? p1 : panels;  // this thread's panels of the previous phase: [p0, q1)
    int sum = 0;
    if (per <= kPer) {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            if (p0 + u < q1) {
                if (lds_bases) pcnt[p0 + u] = cl[u];
                sum += cl[u];
            }
        }
    } else {
        for (int p = p0; p < q1; ++p) {
            const int c = seg_cnt[p];
            if (lds_bases) pcnt[p] = c;
            sum += c;
        }
    }
    int base = block_scan_1024(part, tid, sum);
    if (tid == 1023) total_l = base + sum;
    if (lds_bases) {
        for (int p = p0; p < q1; ++p) {
            const int c = pcnt[p];
            pbase[p] = c ? base : -1;
            base += c;
        }
    }
    __syncthreads();
    const int count = total_l;
    const bool sort = pred && count > 1 && count <= fin_cur && count <= kSortMax;
    int* dst = sort ? ids : idx;
    if (lds_bases) {  // entry r of panel p by thread (16 p + r) mod 1024: coalesced loads, kCompactU of
        // them in flight per thread before any store (one L2 round trip per round, not per entry)
        for (int i0 = tid; i0 < 16 * panels; i0 += 1024 * kCompactU) {
            int v[kCompactU], at[kCompactU];
#pragma unroll
            for (int u = 0; u < kCompactU; ++u) {
                const int i = i0 + 1024 * u;
                at[u] = -1;
                v[u] = 0;
                if (i < 16 * panels) {
                    const int p = i >> 4, r = i & 15, b = pbase[p];
                    if (b >= 0 && r < pcnt[p]) {
                        at[u] = b + r;
                        v[u] = seg_idx[i];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < kCompactU; ++u)
                if (at[u] >= 0) dst[at[u]] = v[u];
        }
    } else {
        for (int p = p0; p < q1; ++p) {
            const int c = seg_cnt[p];
            for (int r = 0; r < c; ++r) dst[base + r] = seg_idx[16 * p + r];
            base += c;
        }
    }
    if (tid == 0) *count_out = count;
    if (!sort) return;
    __syncthreads();  // ids complete
    // the bins of this thread's entries (count <= kSortMax = 8 x 1024: one predicted count per entry,
    // loaded once, used by the histogram and the scatter)
    int bn[kSortMax / 1024];
#pragma unroll
    for (int u = 0; u < kSortMax / 1024; ++u) {
        const int i = tid + 1024 * u;
        bn[u] = 0;
        if (i < count) {
            const int q = pred[ids[i]];  // descending count -> ascending bin
            const int k = q < 0 ? 0 : (q >= kSortBins ? kSortBins - 1 : q);
            bn[u] = kSortBins - 1 - k;
        }
    }
    for (int i = tid; i < kSortBins; i += 1024) hist[i] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kSortMax / 1024; ++u)
        if (tid + 1024 * u < count) atomicAdd(&hist[bn[u]], 1);  // (LDS atomics)
    __syncthreads();
    int local[4], hs = 0;  // thread tid owns bins 4 tid .. 4 tid + 3
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        local[q] = hs;
        hs += hist[4 * tid + q];
    }
    const int hb = block_scan_1024(part, tid, hs);
#pragma unroll
    for (int q = 0; q < 4; ++q) hist[4 * tid + q] = hb + local[q];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kSortMax / 1024; ++u) {
        const int i = tid + 1024 * u;
        if (i < count) idx[atomicAdd(&hist[bn[u]], 1)] = ids[i];
    }
}

hipError_t launch_phase_compact(const int* seg_cnt, const int* seg_idx, const int* count_prev, int batch,
                                int fin_prev, int* idx_out, int* count_out, const int* pred, int fin_cur,
                                hipStream_t s) {
    hipLaunchKernelGGL(phase_compact_kernel, dim3(1), dim3(1024), 0, s, seg_cnt, seg_idx, count_prev, batch,
                       fin_prev, idx_out, count_out, pred, fin_cur);
    return hipGetLastError();
}

template <int T>
static void launch_panel_kernel(const SolveArgs<float>& a, int grid, hipStream_t s) {
    if constexpr (T == 0) {
        (void)launch_bigpanel(a, grid, s);
    } else if constexpr (T > 8) {
        // the C3/C4 shapes (T = 13) with full-length chains and one last-block length in both
        // GEMMs: the compile-time variant (panel2_run KQ)
        const int nkb1 = (a.m + 15) / 16, nkb2 = (a.n + 15) / 16;
        const int kq1 = (a.m - 16 * (nkb1 - 1) + 3) / 4, kq2 = (a.n - 16 * (nkb2 - 1) + 3) / 4;
        const bool full = nkb1 == T && nkb2 == T && kq1 == kq2;
        if constexpr (T == 13) {
            if (a.debug & kDebugDropHandoff) {  // tests only: the fault-injection instantiations
                if (full && kq1 == 2) hipLaunchKernelGGL((gpad_panel2_kernel<T, 2, true>), dim3(grid), dim3(1024), 0, s, a);
                else hipLaunchKernelGGL((gpad_panel2_kernel<T, 0, true>), dim3(grid), dim3(1024), 0, s, a);
                return;
            }
            if (full && kq1 == 1) { hipLaunchKernelGGL((gpad_panel2_kernel<T, 1>), dim3(grid), dim3(1024), 0, s, a); return; }
            if (full && kq1 == 2) { hipLaunchKernelGGL((gpad_panel2_kernel<T, 2>), dim3(grid), dim3(1024), 0, s, a); return; }
            if (full && kq1 == 3) { hipLaunchKernelGGL((gpad_panel2_kernel<T, 3>), dim3(grid), dim3(1024), 0, s, a); return; }
            if (full && kq1 == 4) { hipLaunchKernelGGL((gpad_panel2_kernel<T, 4>), dim3(grid), dim3(1024), 0, s, a); return; }
        }
        (void)full;
        hipLaunchKernelGGL((gpad_panel2_kernel<T, 0>), dim3(grid), dim3(1024), 0, s, a);
    } else
        hipLaunchKernelGGL((gpad_panel_kernel<T>), dim3(grid), dim3(64 * T), 0, s, a);
}

template <int T>
static hipError_t launch_panel_t(SolveArgs<float> a, hipStream_t s) {
    // Grid = resident workgroups: a panel-pair workgroup (T > 8) fills a CU; T-wave panels
    // (T <= 8) share one, 32/T of them.  Workgroups walk their panels grid-stride.
    const int panels = (a.batch + 15) / 16;
    const int resident = (T == 0 || T > 8) ? a.num_cus : a.num_cus * (32 / T);
    int grid = panels < resident ? panels : resident;
    const Tuning tn = a.tune ? *a.tune : Tuning{};
    if (tn.panel_max_grid > 0 && tn.panel_max_grid < grid) grid = tn.panel_max_grid;  // grid-stride panels
    const bool phased = a.tol > 0.0 && a.pwork != nullptr && tn.phased;
    a.fin_thresh = phased ? panel_fin_thresh(a.n, a.m, a.num_cus, &tn) : 0;
    if (!phased) {  // fixed N (or no workspace): one phase, nothing carried
        a.v_begin = 0;
        a.v_end = a.N;
        a.idx_in = nullptr;
        a.count_in = nullptr;
        launch_panel_kernel<T>(a, grid, s);
        return hipGetLastError();
    }
    int* idx0 = reinterpret_cast<int*>(a.pwork);
    int* idx1 = idx0 + a.batch;
    int* counts = idx1 + a.batch;
    int* qctrs = counts + kPanelMaxPhases;
    float* wc = reinterpret_cast<float*>(qctrs + kPanelMaxPhases);
    a.wc = wc;
    a.uc = wc + (size_t)a.batch * a.m;
    // survivors listed per panel, densified at each boundary by phase_compact_kernel (one idx
    // list suffices: phase ph reads idx0 while it lists into seg_idx)
    a.seg_idx = reinterpret_cast<int*>(a.uc + (size_t)a.batch * a.m);
    a.seg_cnt = a.seg_idx + a.batch + 32;
    a.idx_out = nullptr;
    a.count_out = nullptr;
    // the phase counters and the finisher's queue counters: zeroed by the first launch's workgroup 0
    // (panel pairs), else one memset
    hipError_t e = hipSuccess;
    if constexpr (T > 8) {
        a.zero_w = counts;
        a.zero_n = 2 * kPanelMaxPhases;
    } else if ((e = hipMemsetAsync(counts, 0, sizeof(int) * 2 * kPanelMaxPhases, s)) != hipSuccess) {
        return e;
    }
    // phase length: a multiple of the test period (phases end right after a test); default
    // four tests, doubling after 10 phases so a long tail costs O(log N) launches (a phase with
    // no survivors left costs one empty launch, ~5 us)
    const int len = panel_phase_len(a.check_every, &tn);
    const PanelPlan* plan = (a.plan && a.plan->nph > 0 && a.plan->N == a.N) ? a.plan : nullptr;
    if (a.used) {
        a.used->nph = 0;
        a.used->N = a.N;
        a.used->cost_us = plan ? plan->cost_us : 0.0;
    }
    const int fin_default = a.fin_thresh;
    int fin_prev = 0;  // the previous phase's finisher threshold
    int v0 = 0;
    for (int ph = 0; v0 < a.N; ++ph) {
        int plen = len;
        if (ph >= 10 && tn.phase_len <= 0) plen = len << (ph - 9 < 20 ? ph - 9 : 20);  // explicit: uniform
        a.fin_thresh = fin_default;
        if (plan && ph < plan->nph) {  // the previous solve's plan (panel_plan)
            plen = plan->ends[ph] - v0;
            if (ph && fin_default) a.fin_thresh = plan->fins[ph];
        }
        if (plen < 1) plen = len;
        if (ph >= kPanelMaxPhases - 1) plen = a.N;  // last slot: run to N
        const int v1 = (a.N - v0 <= plen) ? a.N : v0 + plen;
        a.v_begin = v0;
        a.v_end = v1;
        a.idx_in = ph ? idx0 : nullptr;
        a.count_in = ph ? counts + ph - 1 : nullptr;
        if (ph) {  // the boundary: phase ph-1's per-panel lists -> idx0 (LPT-ordered for the finisher)
            e = launch_phase_compact(a.seg_cnt, a.seg_idx, ph >= 2 ? counts + ph - 2 : nullptr, a.batch, fin_prev,
                                     idx0, counts + ph - 1, (a.pred && tn.lpt) ? a.pred : nullptr, a.fin_thresh, s);
            if (e != hipSuccess) return e;
        }
        fin_prev = a.fin_thresh;
        if (a.used && ph < kPanelMaxPhases) {  // (diagnostics: gpad_last_phases)
            a.used->ends[ph] = v1;
            a.used->fins[ph] = ph ? a.fin_thresh : 0;
            a.used->nph = ph + 1;
        }
        if (ph && a.fin_thresh) {  // few survivors left: the duo finisher takes them, runs to N --
            // two instances per CU in ping-pong, fed from the survivor list
            a.qctr = qctrs + ph;
            int g = a.fin_thresh < a.num_cus ? a.fin_thresh : a.num_cus;
            if (tn.duo_max_grid > 0 && tn.duo_max_grid < g) g = tn.duo_max_grid;  // more claims
            if ((e = launch_duo(a, g, s)) != hipSuccess) return e;
        }
        launch_panel_kernel<T>(a, grid, s);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        a.zero_w = nullptr;
        v0 = v1;
    }
    return hipSuccess;
}

#ifdef GPAD_STAMP
hipError_t read_stamps(unsigned long long* out, size_t bytes) {
    // g_stamps, then (when the buffer has room) g_pstamps
    size_t b0 = bytes > sizeof(g_stamps) ? sizeof(g_stamps) : bytes;
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), b0, 0, hipMemcpyDeviceToHost);
    if (e != hipSuccess || bytes <= sizeof(g_stamps)) return e;
    size_t b1 = bytes - sizeof(g_stamps);
    if (b1 > sizeof(g_pstamps)) b1 = sizeof(g_pstamps);
    return hipMemcpyFromSymbol(out + sizeof(g_stamps) / 8, HIP_SYMBOL(g_pstamps), b1, 0, hipMemcpyDeviceToHost);
}
#endif

bool panel_folds_gmax(int n, int m) {
    const int T = panel_tiles_for(n, m);
    return T > 8 && T <= kPanelMaxTiles;
}

hipError_t launch_panel(const SolveArgs<float>& a, hipStream_t s, bool* supported) {
    const int T = panel_tiles_for(a.n, a.m);
    // the fragment image must have been packed for this geometry at setup
    if (!T) {  // big panels
        *supported = a.frag != nullptr && bigpanel_supported(a.n, a.m) && a.strideA == 0 && a.strideB == 0 &&
                     a.frag_tiles == panel_tiles(a.n, a.m, a.batch);
        return *supported ? launch_panel_t<0>(a, s) : hipSuccess;
    }
    *supported = a.frag != nullptr && a.strideA == 0 && a.strideB == 0 && a.frag_tiles == T;
    if (!*supported) return hipSuccess;
    switch (T) {
        case 1: return launch_panel_t<1>(a, s);
        case 2: return launch_panel_t<2>(a, s);
        case 3: return launch_panel_t<3>(a, s);
        case 4: return launch_panel_t<4>(a, s);
        case 5: return launch_panel_t<5>(a, s);
        case 6: return launch_panel_t<6>(a, s);
        case 7: return launch_panel_t<7>(a, s);
        case 8: return launch_panel_t<8>(a, s);
        case 9: return launch_panel_t<9>(a, s);
        case 10: return launch_panel_t<10>(a, s);
        case 11: return launch_panel_t<11>(a, s);
        case 12: return launch_panel_t<12>(a, s);
        case 13: return launch_panel_t<13>(a, s);
        case 14: return launch_panel_t<14>(a, s);
        case 15: return launch_panel_t<15>(a, s);
        default: return launch_panel_t<16>(a, s);
    }
}

}  // namespace gpad
