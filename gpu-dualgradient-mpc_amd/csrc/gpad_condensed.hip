// gpad_condensed.hip -- GPAD_KERNEL_CONDENSED: the latency kernel on the condensed operator
// (opt-in through gpad_dims_t.kernel; NOT the reference's arithmetic, see include/gpad.h).
//
// Why: the bit-exact latency kernel (gpad_resident_kernel) is bound by its critical path, one
// m-long (8b) and one n-long (8d) dependent fmaf chain per iteration (seq_functions.cpp:61,82):
// (m + n) x ~5.3-5.9 cycles, 1.17 us per iteration at n = m = 200 -- no schedule of the
// reference's own summation order can go below (m + n) dependent steps.  Eliminating zhat,
//     G_L zhat_v = G_L (MGneg w_v - gP) = H w_v + c,   H = G_L MGneg (m x m),  c = -G_L gP,
// leaves ONE m-long chain per iteration; and because theta_0 = 1 the averaged primal iterate is
// z_v = MGneg wbar_v - gP with wbar_v = (1 - theta_v) wbar_{v-1} + theta_v w_v (8c carried on the
// dual side), so z is formed only when Algorithm 1 decides and at the end.  Same iteration in
// exact arithmetic; in fp32 a reassociation (H rounded once from an fp64 product), which the
// oracle restates bit for bit (oracle/gpad_oracle.c orc_solve_condensed_f32).
//
// Layout: one workgroup per instance, ceil(max(n, m) / 64) waves; lane i holds row i of H in
// VGPRs (k-major image from condense_kernel) and its constraint state (y, w, wbar, p_D, c, u);
// the H chain is the resident kernel's DPP chain (gpad_chain.h chain_regs) over w in LDS, double
// buffered so an iteration has ONE barrier.  The rare direct chains (c at the start, the decided
// tests, the returned z) read -ML / G_L from their k-major images in global memory (L2).
// Algorithm 1 stays certified on the returned point: test (A) is nominated by the recursion u
// and test (B) by s = H w + c; both are decided on direct chains G_L x of the very z / zhat that
// is returned (the margins of gpad_chain.h).
#include <hip/hip_runtime.h>

#include <cmath>

#include "gpad_chain.h"
#include "gpad_internal.h"

namespace gpad {

constexpr int kCondMaxThreads = 256;

// H[i][k] = fl32(sum_j GL[i][j] MGneg[j][k]) as an fp64 fma chain in ascending j, written k-major
// (Ht[k][ldm], the layout the row loader reads).  GL[i][j] = GLt[j][i], MGneg[j][k] = MGt[k][j].
__global__ void condense_kernel(const float* __restrict__ GLt, const float* __restrict__ MGt, int n, int m,
                                int ldn, int ldm, long long strideA, long long strideB, long long strideH,
                                float* __restrict__ Ht) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int k = blockIdx.y;
    const long long mat = blockIdx.z;
    if (i >= m) return;
    const float* G = GLt + mat * strideB;
    const float* Mk = MGt + mat * strideA + (size_t)k * ldn;
    double acc = 0.0;
    for (int j = 0; j < n; ++j) acc = __builtin_fma((double)G[(size_t)j * ldm + i], (double)Mk[j], acc);
    Ht[mat * strideH + (size_t)k * ldm + i] = (float)acc;
}

// sum_{k < len} Mt[k][row] v[k] as one fmaf chain in ascending k (Mt k-major in global memory,
// v in LDS): the rare direct evaluations.
__device__ __forceinline__ float chain_gmem(const float* __restrict__ Mt, int ld, int row, const float* v,
                                            int len) {
    float acc = 0.0f;
    int k = 0;
    for (; k + 8 <= len; k += 8) {
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = Mt[(size_t)(k + j) * ld + row];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc = __builtin_fmaf(e[j], v[k + j], acc);
    }
    for (; k < len; ++k) acc = __builtin_fmaf(Mt[(size_t)k * ld + row], v[k], acc);
    return acc;
}

template <int KH>
__global__ __launch_bounds__(kCondMaxThreads) void gpad_condensed_kernel(SolveArgs<float> a) {
    constexpr int PH = (KH + 63) / 64 * 64;  // whole 64-element groups for the DPP chain
    __shared__ __attribute__((aligned(16))) float w_l[2][PH];  // w, double buffered
    __shared__ float v_l[kCondMaxThreads];                     // vector of a direct chain (len m)
    __shared__ float x_l[kCondMaxThreads];                     // its z / zhat (len n)
    __shared__ CheckSlot slots[2][kCondMaxThreads / 64];       // test, decision

    // finisher mode (after a condensed panel phase): a persistent grid walks the survivor list,
    // each instance resumed at iteration v_begin from the carried y, w, wbar, u, c; shared H rows
    // are loaded once per workgroup
    const bool fin = a.count_in != nullptr;
    const int count = fin ? __builtin_amdgcn_readfirstlane(*a.count_in) : a.batch;
    const int tid = threadIdx.x;
    const int v0 = fin ? a.v_begin : 0;
    const int n = a.n, m = a.m, nwaves = blockDim.x >> 6;
    const bool live = tid < m;  // constraint row / row of H
    const bool prow = tid < n;  // primal row
    float r[KH];  // row tid of H, zero-padded (padded steps are fma(0, 0, acc) = acc)
    bool have_r = false;
    for (int kk = blockIdx.x; kk < count; kk += gridDim.x) {
    const int b = fin ? a.idx_in[kk] : kk;
    const float* __restrict__ MGt = a.MGt + b * a.strideA;
    const float* __restrict__ GLt = a.GLt + b * a.strideB;
    if (!have_r || a.strideH != 0) {
        const float* __restrict__ Ht = a.Hc + b * a.strideH;
#pragma unroll
        for (int k = 0; k < KH; ++k) r[k] = (live && k < m) ? Ht[(size_t)k * a.ldm + tid] : 0.0f;
        have_r = true;
    }

    float* zg = a.z + (size_t)b * n;
    float* yg = a.y + (size_t)b * m;
    const float gpi = prow ? a.gP[(size_t)b * a.ld_gP + tid] : 0.0f;
    float yi = 0.0f, pdi = 0.0f, wi = 0.0f, wbar = 0.0f, ui = 0.0f, ci = 0.0f, wcur = 0.0f;
    for (int i = tid; i < 2 * PH; i += blockDim.x) (&w_l[0][0])[i] = 0.0f;
    if (prow) v_l[tid] = gpi;
    __syncthreads();
    if (live) {
        ci = fin ? a.cc[(size_t)b * m + tid] : -chain_gmem(GLt, a.ldm, tid, v_l, n);  // c = -G_L gP
        yi = yg[tid];
        pdi = (float)(a.gscale * (double)a.g[(size_t)b * a.ld_g + tid]);
        if (fin) {
            const size_t o = (size_t)b * m + tid;
            wi = a.wc[o];
            wbar = a.wbc[o];
            ui = a.uc[o];
        } else {
            wi = __builtin_fmaf(a.beta[0], yi - yi, yi);  // 8a at v = 0 (y_{-1} = y_0)
        }
        w_l[v0 & 1][tid] = wi;
    }
    __syncthreads();

    // x = MGneg v - gP on the primal lanes (returned when `keep`), then G_L x on the constraint
    // lanes; every thread calls it (barriers inside)
    auto direct = [&](float vsrc, float& xo, bool gl) -> float {
        if (live) v_l[tid] = vsrc;
        __syncthreads();
        if (prow) {
            xo = chain_gmem(MGt, a.ldn, tid, v_l, m) - gpi;  // seq_functions.cpp:61-62 order
            x_l[tid] = xo;
        }
        __syncthreads();
        return (gl && live) ? chain_gmem(GLt, a.ldm, tid, x_l, n) : 0.0f;
    };

    const bool use_tol = a.tol > 0.0;
    int it = 0, done = 0;
    float zout = 0.0f;
    float th = a.theta[v0], bn = a.beta[v0 + 1];
    for (int v = v0; v < a.N; ++v) {
        const float th_next = a.theta[v + 1], bn_next = a.beta[v + 2];
        const bool chk = use_tol && ((v + 1) % a.check_every) == 0;
        const float acc = chain_regs<KH, KH>(r, w_l[v & 1]);  // (uniform: DPP reads every lane)
        float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
        double gap = 0.0;
        if (live) {
            const float s = acc + ci;  // G_L zhat_v by the condensed operator
            const float omt = 1.0f - th;
            wbar = __builtin_fmaf(omt, wbar, th * wi);  // 8c on the dual side
            const float sv = (wi + pdi) + s;            // 8d, seq_functions.cpp:84
            const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;
            if (use_tol) ui = __builtin_fmaf(omt, ui, th * s);  // u_0 = s (theta_0 = 1, seed 0)
            if (chk) {
                const float t = s + pdi;
                violz = ui + pdi;
                violh = t;
                magh = __builtin_fabsf(s) + __builtin_fabsf(pdi);
                wmin = wi;
                gap = -((double)wi * (double)t);
            }
            wcur = wi;
            wi = __builtin_fmaf(bn, yp - yi, yp);  // next 8a
            yi = yp;
            w_l[(v + 1) & 1][tid] = wi;
        }
        if (chk) check_publish<float>(slots[0], violz, violh, wmin, gap, magh);
        __syncthreads();
        it = v + 1;
        th = th_next;
        bn = bn_next;
        if (chk) {
            const int st1 = check_stage1<float>(slots[0], nwaves, a.L, a.tol, a.tol_gap);
            if (st1 & 1) {  // (A) nominated: decide on G_L z of z = MGneg wbar - gP, u reset to it
                float xz = 0.0f;
                const float cz = direct(wbar, xz, true);
                float vc = -INFINITY, mc = 0.0f;
                if (live) {
                    ui = cz;
                    vc = cz + pdi;
                    mc = __builtin_fabsf(cz) + __builtin_fabsf(pdi);
                }
                check_publish<float>(slots[1], vc, vc, vc, 0.0, mc);
                __syncthreads();
                if (check_verify<float>(slots[1], nwaves, a.L, a.tol)) {
                    done = 1;
                    zout = xz;
                }
            }
            if (!done && (st1 & 2)) {  // (B) nominated on s: decide on G_L zhat of zhat = MGneg w - gP
                float xh = 0.0f;
                const float ch = direct(wcur, xh, true);
                float vh = -INFINITY, mh = 0.0f, wm = INFINITY;
                double gp = 0.0;
                if (live) {
                    const float t = ch + pdi;
                    vh = t;
                    mh = __builtin_fabsf(ch) + __builtin_fabsf(pdi);
                    wm = wcur;
                    gp = -((double)wcur * (double)t);
                }
                check_publish<float>(slots[1], -INFINITY, vh, wm, gp, mh);
                __syncthreads();
                if (check_stage1<float>(slots[1], nwaves, a.L, a.tol, a.tol_gap) & 2) {
                    done = 2;
                    zout = xh;
                }
            }
        }
        if (done) break;
    }
    if (it > 0 && !done) {
        float xz = 0.0f;
        (void)direct(wbar, xz, false);  // z = MGneg wbar - gP
        zout = xz;
    }
    if (prow && it > 0) zg[tid] = zout;
    if (live) yg[tid] = yi;
    if (tid == 0) {
        a.iters[b] = it;
        a.conv[b] = done;
    }
    __syncthreads();  // the next instance reuses the LDS vectors
    }
}

bool condensed_supported(int n, int m) { return m <= kResidentMaxRow && n <= kCondMaxThreads && n > 0 && m > 0; }

hipError_t launch_condense(const float* GLt, const float* MGt, int n, int m, int ldn, int ldm, int nmats,
                           long long strideA, long long strideB, float* Ht, hipStream_t s) {
    const dim3 grid((m + 255) / 256, m, nmats);
    hipLaunchKernelGGL(condense_kernel, grid, dim3(256), 0, s, GLt, MGt, n, m, ldn, ldm, strideA, strideB,
                       (long long)m * ldm, Ht);
    return hipGetLastError();
}

hipError_t launch_condensed(const SolveArgs<float>& a, hipStream_t s, bool* supported) {
    *supported = condensed_supported(a.n, a.m) && a.Hc != nullptr;
    if (!*supported) return hipSuccess;
    const int rows = a.n > a.m ? a.n : a.m;
    // one instance per workgroup; as the finisher a persistent grid over the survivor list (a grid
    // of `batch` mostly empty workgroups cost ~0.1 ms of dispatch alone)
    const int g = a.count_in ? (a.batch < 2 * a.num_cus ? a.batch : 2 * a.num_cus) : a.batch;
    const dim3 grid(g), block(64 * ((rows + 63) / 64));
    switch (res_bucket(a.m)) {
        case 32: hipLaunchKernelGGL((gpad_condensed_kernel<32>), grid, block, 0, s, a); break;
        case 64: hipLaunchKernelGGL((gpad_condensed_kernel<64>), grid, block, 0, s, a); break;
        case 96: hipLaunchKernelGGL((gpad_condensed_kernel<96>), grid, block, 0, s, a); break;
        case 128: hipLaunchKernelGGL((gpad_condensed_kernel<128>), grid, block, 0, s, a); break;
        case 160: hipLaunchKernelGGL((gpad_condensed_kernel<160>), grid, block, 0, s, a); break;
        case 192: hipLaunchKernelGGL((gpad_condensed_kernel<192>), grid, block, 0, s, a); break;
        case 200: hipLaunchKernelGGL((gpad_condensed_kernel<200>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((gpad_condensed_kernel<208>), grid, block, 0, s, a); break;
    }
    return hipGetLastError();
}

}  // namespace gpad
