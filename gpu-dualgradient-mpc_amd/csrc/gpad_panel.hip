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

size_t panel_frag_bytes(int n, int m, int /*batch*/) {
    const int T = panel_tiles_for(n, m);
    return T ? (size_t)2 * T * T * 64 * sizeof(float4) : 0;
}

int panel_tiles(int n, int m, int /*batch*/) { return panel_tiles_for(n, m); }

hipError_t launch_pack_panel(const float* ML, const float* G, int n, int m, int /*batch*/,
                             float mg_sign, double g_scale, void* frag, hipStream_t s) {
    const int T = panel_tiles_for(n, m);
    if (!T) return hipSuccess;
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
};

// acc = A[tile t] (T k-blocks, streamed from L2 one block ahead) x B (LDS, fragment order).
// The MFMA k-order is ascending (block 0..T-1, step 0..3), i.e. the reference's sequential chain.
// A is read with buffer loads: one 32-bit lane offset (t*1 KiB + lane*16 B) in a VGPR and the
// k-block offset as a compile-time scalar, so the unrolled blocks cost no address registers.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

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

template <int T>
__global__ __launch_bounds__(64 * T) void gpad_panel_kernel(SolveArgs<float> a) {
    __shared__ __attribute__((aligned(16))) float Wl[T * 256];  // [T][64][4] w    (B of GEMM 1)
    __shared__ __attribute__((aligned(16))) float Zh[T * 256];  // [T][64][4] zhat (B of GEMM 2)
    __shared__ PanelSlot slots[T];

    const int lane = threadIdx.x & 63;
    const int t = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // row tile of this wave
    const int j = lane >> 4, c = lane & 15;
    const int n = a.n, m = a.m;
    const int inst = blockIdx.x * 16 + c;
    const bool real = inst < a.batch;
    const int abytes = T * T * 1024;  // one packed operand
    const __amdgpu_buffer_rsrc_t PA1 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.frag), 0, abytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t PA2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)a.frag + abytes), 0, abytes, 0x00020000);
    const int voff = t * 1024 + lane * 16;
    const float4* Wl4 = reinterpret_cast<const float4*>(Wl);
    float4* Wl4w = reinterpret_cast<float4*>(Wl);
    float4* Zh4w = reinterpret_cast<float4*>(Zh);
    const int slot = t * 64 + lane;  // this lane's float4 in Wl / Zh

    // ---- prologue: this wave's rows (register r <-> row 16t + 4r + j, instance c) ------------
    float z[4], gp[4], y[4], pd[4], u[4], zh[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 16 * t + 4 * r + j;
        const bool okn = real && i < n, okm = real && i < m;
        z[r] = okn ? a.z[(size_t)inst * n + i] : 0.0f;
        gp[r] = okn ? a.gP[(size_t)inst * a.ld_gP + i] : 0.0f;
        y[r] = okm ? a.y[(size_t)inst * m + i] : 0.0f;
        pd[r] = okm ? (float)(a.gscale * (double)a.g[(size_t)inst * a.ld_g + i]) : 0.0f;
        u[r] = 0.0f;
        zh[r] = 0.0f;
    }
    const float b0 = a.beta[0];
    Wl4w[slot] = make_float4(__builtin_fmaf(b0, y[0] - y[0], y[0]), __builtin_fmaf(b0, y[1] - y[1], y[1]),
                             __builtin_fmaf(b0, y[2] - y[2], y[2]), __builtin_fmaf(b0, y[3] - y[3], y[3]));
    const bool use_tol = a.tol > 0.0;
    if (use_tol) {  // u = G_L z_{-1} (then carried by the 8c recursion)
        Zh4w[slot] = make_float4(z[0], z[1], z[2], z[3]);
        __syncthreads();
        const f32x4 cz = panel_gemm<T>(PA2, Zh, voff, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r) u[r] = cz[r];
    }
    __syncthreads();

    bool active = real;
    int my_it = 0, my_code = 0;
    float th = a.theta[0], bn = a.beta[1];
    for (int v = 0; v < a.N; ++v) {
        const float th_next = a.theta[v + 1], bn_next = a.beta[v + 2];
        const bool chk = use_tol && ((v + 1) % a.check_every) == 0;
        const float omt = 1.0f - th;
        // ---- GEMM 1 + epilogue: zhat = -ML w - g_P (8b), z = (1-th) z + th zhat (8c) -----
        {
            const f32x4 acc = panel_gemm<T>(PA1, Wl, voff, lane);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                zh[r] = acc[r] - gp[r];
                const float zn = __builtin_fmaf(omt, z[r], th * zh[r]);
                if (active) z[r] = zn;
            }
            Zh4w[slot] = make_float4(zh[0], zh[1], zh[2], zh[3]);
        }
        __syncthreads();
        // ---- GEMM 2 + epilogue: y+ = [w + G_L zhat + p_D]+ (8d), next w (8a) --------------
        float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY;
        double gap = 0.0;
        {
            const f32x4 acc = panel_gemm<T>(PA2, Zh, voff, lane);
            const float4 w4 = Wl4[slot];
            const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
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
                    if (chk && (16 * t + 4 * r + j) < m) {
                        const float tt = cv + pd[r];
                        violh = fmaxf(violh, tt);
                        wmin = fminf(wmin, wv[r]);
                        gap -= (double)wv[r] * (double)tt;
                        violz = fmaxf(violz, u[r] + pd[r]);
                    }
                }
                if (active) y[r] = yp;
            }
            if (active) Wl4w[slot] = make_float4(wn[0], wn[1], wn[2], wn[3]);
        }
        th = th_next;
        bn = bn_next;
        if (active) my_it = v + 1;
        if (!chk) {
            __syncthreads();
            continue;
        }
        // ---- Algorithm 1 test, per instance: lane groups j, then row tiles through LDS ------
#pragma unroll
        for (int o = 16; o < 64; o <<= 1) {
            violz = fmaxf(violz, __shfl_xor(violz, o, 64));
            violh = fmaxf(violh, __shfl_xor(violh, o, 64));
            wmin = fminf(wmin, __shfl_xor(wmin, o, 64));
            gap += __shfl_xor(gap, o, 64);
        }
        if (j == 0) {
            slots[t].violz[c] = violz;
            slots[t].violh[c] = violh;
            slots[t].wmin[c] = wmin;
            slots[t].gap[c] = gap;
        }
        __syncthreads();
        double vz = -INFINITY, vh = -INFINITY, wm = INFINITY, gq = 0.0;
#pragma unroll
        for (int s = 0; s < T; ++s) {
            vz = fmax(vz, (double)slots[s].violz[c]);
            vh = fmax(vh, (double)slots[s].violh[c]);
            wm = fmin(wm, (double)slots[s].wmin[c]);
            gq += slots[s].gap[c];
        }
        int code = 0;
        if (vz * a.L <= a.tol) code = 1;
        else if ((vh * a.L <= a.tol) && (wm >= 0.0) && (gq * a.L <= a.tol)) code = 2;
        if (active && code) {
            my_code = code;
            if (code == 2) {  // zhat certified: it becomes z*
#pragma unroll
                for (int r = 0; r < 4; ++r) z[r] = zh[r];
            }
            active = false;
        }
        // leave when no instance of the panel is still iterating (uniform: same LDS reads);
        // the barrier also orders the slot reads above before the next check's writes
        if (!__syncthreads_or(active ? 1 : 0)) break;
    }
    // ---- write back ---------------------------------------------------------------------
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = 16 * t + 4 * r + j;
        if (real && i < n) a.z[(size_t)inst * n + i] = z[r];
        if (real && i < m) a.y[(size_t)inst * m + i] = y[r];
    }
    if (t == 0 && j == 0 && real) {
        a.iters[inst] = my_it;
        a.conv[inst] = my_code;
    }
}

template <int T>
static hipError_t launch_panel_t(const SolveArgs<float>& a, hipStream_t s) {
    const int groups = (a.batch + 15) / 16;
    hipLaunchKernelGGL(gpad_panel_kernel<T>, dim3(groups), dim3(64 * T), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_panel(const SolveArgs<float>& a, hipStream_t s, bool* supported) {
    const int T = panel_tiles_for(a.n, a.m);
    // the fragment image must have been packed for this geometry at setup
    *supported = a.frag != nullptr && T && a.strideA == 0 && a.strideB == 0 && a.frag_tiles == T;
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
