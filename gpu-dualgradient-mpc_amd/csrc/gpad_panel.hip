// gpad_panel.hip -- shared-matrix batches on the f32 MFMA pipe (gfx950).
//
// When every instance of a batch shares ML and G (one plant, many states: the battery
// scenario batch), the two mat-vecs of a GPAD iteration over 16 instances are two skinny
// GEMMs:  Zhat[n x 16] = (-ML) W[m x 16]  and  Y'[m x 16] = G_L Zhat[n x 16].  One workgroup
// owns a panel of 16 instances for the whole solve (no inter-workgroup traffic at all);
// its SPLIT waves split the 16-row tiles of each GEMM and exchange W / Zhat through LDS.
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
// Packed operands in HBM/L2 (built once by pack_panel_kernel at setup):
//   PA1[b][t][lane][q] = -ML[16t + pi(lane&15)][16b + 4q + (lane>>4)]   (b < TM, t < TN)
//   PA2[b][t][lane][q] = G_L[16t + pi(lane&15)][16b + 4q + (lane>>4)]   (b < TN, t < TM)
// one float4 per lane per (block, tile): 1 KiB per wave-instruction, fully coalesced.
#include <hip/hip_runtime.h>

#include <cmath>

#include "gpad_internal.h"

namespace gpad {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int pi16(int rho) { return 4 * (rho & 3) + (rho >> 2); }

// Geometry.  A panel of 16 instances is owned by a workgroup of SPLIT waves; every GEMM's
// rows are padded to T = NL*SPLIT tiles (the same T for n and m), so each wave owns exactly NL
// tiles (t = u*SPLIT + w) and no MFMA sits behind a guard.  Padding rows/columns are zero in
// the packed operands, so padded k-steps are fma(0, x, acc) = acc.
struct PanelGeom {
    int split, nl, tiles;
};

static constexpr int kNlSplit2[] = {1, 2, 4, 7};
static constexpr int kNlSplit4[] = {1, 2, 4};

static PanelGeom panel_geom(int n, int m, int batch) {
    const int groups = (batch + 15) / 16;
    const int need = ((n > m ? n : m) + 15) / 16;
    PanelGeom g{groups >= 512 ? 2 : 4, 0, 0};  // aim for >= 4 waves per CU
    if (g.split == 2) {
        for (int nl : kNlSplit2)
            if (nl * 2 >= need) { g.nl = nl; break; }
    } else {
        for (int nl : kNlSplit4)
            if (nl * 4 >= need) { g.nl = nl; break; }
        if (!g.nl) {  // too tall for 4-wave panels: try 2-wave panels
            g.split = 2;
            for (int nl : kNlSplit2)
                if (nl * 2 >= need) { g.nl = nl; break; }
        }
    }
    g.tiles = g.nl * g.split;
    return g;
}

// ---------------------------------------------------------------------------------------
// packing
// ---------------------------------------------------------------------------------------
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

size_t panel_frag_bytes(int n, int m, int batch) {
    const PanelGeom g = panel_geom(n, m, batch);
    if (!g.nl) return 0;
    return (size_t)2 * g.tiles * g.tiles * 64 * sizeof(float4);
}

hipError_t launch_pack_panel(const float* ML, const float* G, int n, int m, int batch, float mg_sign,
                             double g_scale, void* frag, hipStream_t s) {
    const PanelGeom g = panel_geom(n, m, batch);
    if (!g.nl) return hipSuccess;
    const int T = g.tiles;
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
// the panel kernel
// ---------------------------------------------------------------------------------------
struct PanelSlot {  // per wave, per instance partials of the Algorithm-1 test
    float violz[16], violh[16], wmin[16];
    double gap[16];
};

// One 16-deep k-block: acc[u] += A[b][u*SPLIT + w] * B[b] (four MFMA k-steps per tile).
template <int NL>
__device__ __forceinline__ void panel_kblock(const float4 (&a)[NL], const float4 bf, f32x4 (&acc)[NL]) {
#pragma unroll
    for (int u = 0; u < NL; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].x, bf.x, acc[u], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < NL; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].y, bf.y, acc[u], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < NL; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].z, bf.z, acc[u], 0, 0, 0);
#pragma unroll
    for (int u = 0; u < NL; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u].w, bf.w, acc[u], 0, 0, 0);
}

template <int SPLIT, int NL>
__device__ __forceinline__ void panel_load(const float4* __restrict__ PA, int b, int w, int lane,
                                           float4 (&a)[NL]) {
    constexpr int T = NL * SPLIT;
#pragma unroll
    for (int u = 0; u < NL; ++u) a[u] = PA[((size_t)b * T + u * SPLIT + w) * 64 + lane];
}

// acc (+)= A * B over T k-blocks (T even); A streamed from L2 one k-block ahead, B fragments
// from LDS in fragment order.  The empty asm bounds the prefetch to one k-block.
template <int SPLIT, int NL>
__device__ __forceinline__ void panel_gemm(const float4* __restrict__ PA, const float* Bl, int w, int lane,
                                           f32x4 (&acc)[NL]) {
    constexpr int T = NL * SPLIT;
    float4 a0[NL], a1[NL];
    panel_load<SPLIT, NL>(PA, 0, w, lane, a0);
#pragma unroll 1
    for (int b = 0; b < T; b += 2) {
        panel_load<SPLIT, NL>(PA, b + 1, w, lane, a1);
        float4 bf = *reinterpret_cast<const float4*>(Bl + (b * 64 + lane) * 4);
        panel_kblock<NL>(a0, bf, acc);
        asm volatile("" ::: "memory");
        panel_load<SPLIT, NL>(PA, b + 2 < T ? b + 2 : b + 1, w, lane, a0);
        bf = *reinterpret_cast<const float4*>(Bl + ((b + 1) * 64 + lane) * 4);
        panel_kblock<NL>(a1, bf, acc);
        asm volatile("" ::: "memory");
    }
}

template <int SPLIT, int NL>
__global__ __launch_bounds__(64 * SPLIT) void gpad_panel_kernel(SolveArgs<float> a) {
    constexpr int T = NL * SPLIT;  // 16-row tiles of both GEMMs (n and m padded to 16T)
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* Wl = lds;                  // [T][64][4]  w    (B of GEMM 1)
    float* Zh = Wl + T * 256;         // [T][64][4]  zhat (B of GEMM 2)
    float* Zs = Zh + T * 256;         // [T][64][4]  z
    float* Gp = Zs + T * 256;         // [T][64][4]  g_P
    float* Pd = Gp + T * 256;         // [T][64][4]  p_D
    PanelSlot* slots = reinterpret_cast<PanelSlot*>(Pd + T * 256);

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave index, provably uniform
    const int j = lane >> 4, c = lane & 15;
    const int n = a.n, m = a.m;
    const int inst = blockIdx.x * 16 + c;
    const bool real = inst < a.batch;
    const float4* PA1 = reinterpret_cast<const float4*>(a.frag);
    const float4* PA2 = PA1 + (size_t)T * T * 64;

    // ---- prologue: per-instance vectors into fragment order ------------------------------
    for (int e = tid; e < T * 256; e += 64 * SPLIT) {
        const int t = e >> 8, l = (e >> 2) & 63, r = e & 3;
        const int i = 16 * t + 4 * r + (l >> 4), ci = blockIdx.x * 16 + (l & 15);
        const bool okn = i < n && ci < a.batch;
        const bool okm = i < m && ci < a.batch;
        Zs[e] = okn ? a.z[(size_t)ci * n + i] : 0.0f;
        Gp[e] = okn ? a.gP[(size_t)ci * a.ld_gP + i] : 0.0f;
        Zh[e] = 0.0f;
        const float yv = okm ? a.y[(size_t)ci * m + i] : 0.0f;
        Pd[e] = okm ? (float)(a.gscale * (double)a.g[(size_t)ci * a.ld_g + i]) : 0.0f;
        Wl[e] = __builtin_fmaf(a.beta[0], yv - yv, yv);  // 8a with y_0 = y_{-1}
    }
    // y of this wave's constraint tiles stays in registers
    float Y[NL][4];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const int t = u * SPLIT + w;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * t + 4 * r + j;
            Y[u][r] = (i < m && real) ? a.y[(size_t)inst * m + i] : 0.0f;
        }
    }
    __syncthreads();

    bool active = real;  // this lane's instance still iterating
    int my_it = 0, my_code = 0;
    float th = a.theta[0], bn = a.beta[1];
    const bool use_tol = a.tol > 0.0;
    for (int v = 0; v < a.N; ++v) {
        const float th_next = a.theta[v + 1], bn_next = a.beta[v + 2];
        const bool chk = use_tol && ((v + 1) % a.check_every) == 0;
        // ---- GEMM 1: zhat = -ML w ------------------------------------------------------
        f32x4 acc1[NL];
#pragma unroll
        for (int u = 0; u < NL; ++u) acc1[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        panel_gemm<SPLIT, NL>(PA1, Wl, w, lane, acc1);
        // ---- epilogue 1: 8b tail + 8c ----------------------------------------------------
        const float omt = 1.0f - th;
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int t = u * SPLIT + w;
            float* zs = Zs + (t * 64 + lane) * 4;
            const float4 gp = *reinterpret_cast<const float4*>(Gp + (t * 64 + lane) * 4);
            const float4 z4 = *reinterpret_cast<const float4*>(zs);
            float4 zh, zn;
            zh.x = acc1[u][0] - gp.x;
            zh.y = acc1[u][1] - gp.y;
            zh.z = acc1[u][2] - gp.z;
            zh.w = acc1[u][3] - gp.w;
            zn.x = __builtin_fmaf(omt, z4.x, th * zh.x);
            zn.y = __builtin_fmaf(omt, z4.y, th * zh.y);
            zn.z = __builtin_fmaf(omt, z4.z, th * zh.z);
            zn.w = __builtin_fmaf(omt, z4.w, th * zh.w);
            *reinterpret_cast<float4*>(Zh + (t * 64 + lane) * 4) = zh;
            if (active) *reinterpret_cast<float4*>(zs) = zn;
        }
        __syncthreads();
        // ---- GEMM 2: G_L zhat -----------------------------------------------------------
        f32x4 acc2[NL];
#pragma unroll
        for (int u = 0; u < NL; ++u) acc2[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        panel_gemm<SPLIT, NL>(PA2, Zh, w, lane, acc2);
        // ---- epilogue 2: 8d + next 8a ----------------------------------------------------
        float violh = -INFINITY, wmin = INFINITY;
        double gap = 0.0;
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int t = u * SPLIT + w;
            float* wl = Wl + (t * 64 + lane) * 4;
            const float4 w4 = *reinterpret_cast<const float4*>(wl);
            const float4 p4 = *reinterpret_cast<const float4*>(Pd + (t * 64 + lane) * 4);
            const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
            const float pv[4] = {p4.x, p4.y, p4.z, p4.w};
            float wn[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float cval = acc2[u][r];
                const float sv = (wv[r] + pv[r]) + cval;
                const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;
                if (chk && (16 * t + 4 * r + j) < m) {
                    const float tt = cval + pv[r];
                    violh = fmaxf(violh, tt);
                    wmin = fminf(wmin, wv[r]);
                    gap -= (double)wv[r] * (double)tt;
                }
                wn[r] = __builtin_fmaf(bn, yp - Y[u][r], yp);
                if (active) Y[u][r] = yp;
            }
            if (active) *reinterpret_cast<float4*>(wl) = make_float4(wn[0], wn[1], wn[2], wn[3]);
        }
        __syncthreads();
        th = th_next;
        bn = bn_next;
        if (!chk) {
            if (active) my_it = v + 1;
            continue;
        }
        // ---- Algorithm 1 test: (A) needs G_L z --------------------------------------------
        f32x4 accz[NL];
#pragma unroll
        for (int u = 0; u < NL; ++u) accz[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        panel_gemm<SPLIT, NL>(PA2, Zs, w, lane, accz);
        float violz = -INFINITY;
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int t = u * SPLIT + w;
            const float4 p4 = *reinterpret_cast<const float4*>(Pd + (t * 64 + lane) * 4);
            const float pv[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if ((16 * t + 4 * r + j) < m) violz = fmaxf(violz, accz[u][r] + pv[r]);
        }
        // per instance: reduce over the four lane groups j, then over waves through LDS
#pragma unroll
        for (int o = 16; o < 64; o <<= 1) {
            violz = fmaxf(violz, __shfl_xor(violz, o, 64));
            violh = fmaxf(violh, __shfl_xor(violh, o, 64));
            wmin = fminf(wmin, __shfl_xor(wmin, o, 64));
            gap += __shfl_xor(gap, o, 64);
        }
        if (j == 0) {
            slots[w].violz[c] = violz;
            slots[w].violh[c] = violh;
            slots[w].wmin[c] = wmin;
            slots[w].gap[c] = gap;
        }
        __syncthreads();
        double vz = -INFINITY, vh = -INFINITY, wm = INFINITY, gp = 0.0;
#pragma unroll
        for (int s = 0; s < SPLIT; ++s) {
            vz = fmax(vz, (double)slots[s].violz[c]);
            vh = fmax(vh, (double)slots[s].violh[c]);
            wm = fmin(wm, (double)slots[s].wmin[c]);
            gp += slots[s].gap[c];
        }
        int code = 0;
        if (vz * a.L <= a.tol) code = 1;
        else if ((vh * a.L <= a.tol) && (wm >= 0.0) && (gp * a.L <= a.tol)) code = 2;
        if (active) {
            my_it = v + 1;
            if (code) {
                my_code = code;
                if (code == 2) {  // zhat certified: it becomes z* (own primal tiles)
#pragma unroll
                    for (int u = 0; u < NL; ++u) {
                        const int t = u * SPLIT + w;
                        const float4 zh = *reinterpret_cast<const float4*>(Zh + (t * 64 + lane) * 4);
                        *reinterpret_cast<float4*>(Zs + (t * 64 + lane) * 4) = zh;
                    }
                }
                active = false;
            }
        }
        // leave when no instance of the panel is still iterating (same answer in every wave)
        if (!__any(active)) break;
        __syncthreads();  // Zs / slots reads above complete before the next epilogue writes
    }
    // ---- write back -------------------------------------------------------------------
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const int t = u * SPLIT + w;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * t + 4 * r + j;
            if (i < m && real) a.y[(size_t)inst * m + i] = Y[u][r];
        }
    }
    for (int e = tid; e < T * 256; e += 64 * SPLIT) {
        const int t = e >> 8, l = (e >> 2) & 63, r = e & 3;
        const int i = 16 * t + 4 * r + (l >> 4), ci = blockIdx.x * 16 + (l & 15);
        if (i < n && ci < a.batch) a.z[(size_t)ci * n + i] = Zs[e];
    }
    if (w == 0 && j == 0 && real) {
        a.iters[inst] = my_it;
        a.conv[inst] = my_code;
    }
}

template <int SPLIT, int NL>
static hipError_t launch_panel_t(const SolveArgs<float>& a, hipStream_t s) {
    constexpr int T = NL * SPLIT;
    const size_t lds = sizeof(float) * 256 * (size_t)(5 * T) + sizeof(PanelSlot) * SPLIT;
    hipError_t e = hipFuncSetAttribute((const void*)gpad_panel_kernel<SPLIT, NL>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    const int groups = (a.batch + 15) / 16;
    hipLaunchKernelGGL((gpad_panel_kernel<SPLIT, NL>), dim3(groups), dim3(64 * SPLIT), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_panel(const SolveArgs<float>& a, hipStream_t s, bool* supported) {
    const PanelGeom g = panel_geom(a.n, a.m, a.batch);
    // the fragment image must have been packed for this geometry (setup saw the same batch)
    *supported = a.frag != nullptr && g.nl && a.strideA == 0 && a.strideB == 0 &&
                 a.frag_tiles == g.tiles;
    if (!*supported) return hipSuccess;
    if (g.split == 2) {
        switch (g.nl) {
            case 1: return launch_panel_t<2, 1>(a, s);
            case 2: return launch_panel_t<2, 2>(a, s);
            case 4: return launch_panel_t<2, 4>(a, s);
            default: return launch_panel_t<2, 7>(a, s);
        }
    }
    switch (g.nl) {
        case 1: return launch_panel_t<4, 1>(a, s);
        case 2: return launch_panel_t<4, 2>(a, s);
        default: return launch_panel_t<4, 4>(a, s);
    }
}

int panel_tiles(int n, int m, int batch) { return panel_geom(n, m, batch).tiles; }

}  // namespace gpad
