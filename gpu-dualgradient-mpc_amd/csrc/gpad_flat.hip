// gpad_flat.hip -- the "flat" battery GPAD path.
//
// For the battery-balancing MPC with EQUAL cell capacities the condensed matrices have a
// Kronecker structure (H = kron(Hs, I_{n_u})): column k of the first 4 n_u N constraints touches
// only cell k % n_u, and the 2N coupling rows (the K blocks) touch every cell with the same
// coefficient.  The reference stores only the distinct entries (ENABLE_FLATTEN_MATRICES:
// M_G is N x m, G_L is m x N, main.cu:39-56) and evaluates the two mat-vecs over the structural
// nonzeros only (StepTwoGPADFlatSequential seq_functions.cpp:5-20, StepFourGPADFlatSequential
// :23-43, StepFourGPADFlatParRows kernel_functions.cu:74-109): 6N products per primal row
// instead of m, N (or N n_u) per constraint row instead of n -- ~3x fewer flops and n_u x fewer
// matrix bytes at the C1 shape.
//
// Arithmetic = the reference's flat CPU steps, bit for bit (oracle orc_*_flat_f32):
//   zhat[i n_u + j] = chain(k = j, j+n_u, .. < 4 n_u N; k = 4 n_u N .. m-1) MGf[i][k] w[k] - g_P
//   row r < 4 n_u N : s = chain_t GLf[r][t] zhat[t n_u + r % n_u]
//   row r >= 4 n_u N: s = chain_(t, k) GLf[r][t] zhat[t n_u + k]
//   y+ = (s + w) + p_D, then y+ < 0 -> 0       (NOT the non-flat ((w + p_D) + s, (|s|+s)/2))
// (the reference's GPU flat kernel thresholds at COMP_EPSILON = 1e-8 instead of 0; we pin the
// CPU path, which is also what the MATLAB max(., 0) does).
//
// Kernel: one workgroup per instance (256 threads), every vector in LDS, rows looped over the
// threads; the flat matrices (shared by the batch) are staged once into LDS when they fit
// (C1: 14 KB), else read through L2.  G_L is kept t-major (GLfT[t][r]) so consecutive constraint
// rows read consecutive words.
#include <hip/hip_runtime.h>

#include <cmath>

#include "gpad_chain.h"
#include "gpad_internal.h"

namespace gpad {

constexpr int kFlatBlock = 256;
static_assert(kFlatBlock / 64 <= 8, "test slots: one per lane over lanes 0..7 (gpad_chain.h check_stage1)");
constexpr size_t kFlatStageMax = 64 * 1024;  // bytes of flat matrices staged in LDS


// primal row r = (i, j): the structural nonzeros of row r of -ML, ascending k
__device__ __forceinline__ float flat_row2(const float* MG, const float* w, int i, int j, int n_u, int mc,
                                           int m) {
    const float* row = MG + (size_t)i * m;
    float acc = 0.0f;
    for (int k = j; k < mc; k += n_u) acc = __builtin_fmaf(row[k], w[k], acc);
    for (int k = mc; k < m; ++k) acc = __builtin_fmaf(row[k], w[k], acc);
    return acc;
}

// constraint row r: the structural nonzeros of row r of G_L (GLT is t-major: GLT[t*m + r])
__device__ __forceinline__ float flat_row4(const float* GLT, const float* x, int r, int Nh, int n_u, int mc,
                                           int m) {
    float acc = 0.0f;
    if (r < mc) {
        const int c = r % n_u;
        for (int t = 0; t < Nh; ++t) acc = __builtin_fmaf(GLT[(size_t)t * m + r], x[t * n_u + c], acc);
    } else {
        for (int t = 0; t < Nh; ++t) {
            const float g = GLT[(size_t)t * m + r];
            for (int k = 0; k < n_u; ++k) acc = __builtin_fmaf(g, x[t * n_u + k], acc);
        }
    }
    return acc;
}

__global__ __launch_bounds__(kFlatBlock) void gpad_flat_kernel(SolveArgs<float> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int b = blockIdx.x;
    const int n = a.n, m = a.m, n_u = a.n_u, Nh = n / n_u, mc = 4 * n_u * Nh;
    float* w = reinterpret_cast<float*>(smem);  // [m]
    float* ys = w + m;                          // [m]
    float* pd = ys + m;                         // [m]
    float* us = pd + m;                         // [m]  u = G_L z (test, by recursion)
    float* zh = us + m;                         // [n]
    float* zs = zh + n;                         // [n]
    float* gp = zs + n;                         // [n]
    // [2][waves]: the test's partials, the verification of a nominated test (A)
    CheckSlot* slots = reinterpret_cast<CheckSlot*>(gp + n + ((n & 1) ? 1 : 0));
    float* stage = reinterpret_cast<float*>(slots + 2 * (kFlatBlock / 64));
    const bool staged = a.flat_staged != 0;
    const float* MG = a.MGt;  // flat -ML, Nh x m
    const float* GLT = a.GLt;  // flat G_L, t-major Nh x m
    if (staged) {  // stage both flat matrices (shared by the batch) once
        float* sMG = stage;
        float* sGL = stage + (size_t)Nh * m;
        for (int e = tid; e < Nh * m; e += kFlatBlock) {
            sMG[e] = MG[e];
            sGL[e] = GLT[e];
        }
        MG = sMG;
        GLT = sGL;
    }
    float* zg = a.z + (size_t)b * n;
    float* yg = a.y + (size_t)b * m;
    for (int i = tid; i < n; i += kFlatBlock) {
        zs[i] = zg[i];
        gp[i] = a.gP[(size_t)b * a.ld_gP + i];
        zh[i] = 0.0f;
    }
    for (int i = tid; i < m; i += kFlatBlock) {
        const float yv = yg[i];
        ys[i] = yv;
        pd[i] = (float)(a.gscale * (double)a.g[(size_t)b * a.ld_g + i]);
        w[i] = __builtin_fmaf(a.beta[0], yv - yv, yv);  // 8a with y_0 = y_{-1}
    }
    __syncthreads();
    const bool use_tol = a.tol > 0.0;
    if (use_tol)
        for (int r = tid; r < m; r += kFlatBlock) us[r] = flat_row4(GLT, zs, r, Nh, n_u, mc, m);

    int it = 0, done = 0;
    for (int v = 0; v < a.N; ++v) {
        const float th = a.theta[v], omt = 1.0f - th, bnext = a.beta[v + 1];
        // ---- 8b + 8c (StepTwoGPADFlatSequential, StepThreeGPADSequential) --------------
        for (int r = tid; r < n; r += kFlatBlock) {
            const float zhv = flat_row2(MG, w, r / n_u, r % n_u, n_u, mc, m) - gp[r];
            zh[r] = zhv;
            zs[r] = __builtin_fmaf(omt, zs[r], th * zhv);
        }
        __syncthreads();
        // ---- 8d + next 8a (StepFourGPADFlatSequential) ----------------------------------
        const bool chk = use_tol && ((v + 1) % a.check_every) == 0;
        float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
        double gap = 0.0;
        for (int r = tid; r < m; r += kFlatBlock) {
            const float s = flat_row4(GLT, zh, r, Nh, n_u, mc, m);
            const float wi = w[r], pdi = pd[r], yi = ys[r];
            const float sv = (s + wi) + pdi;        // seq_functions.cpp:37
            const float yp = sv < 0.0f ? 0.0f : sv;  // seq_functions.cpp:40-42
            if (use_tol) {
                const float ui = __builtin_fmaf(omt, us[r], th * s);
                us[r] = ui;
                if (chk) {
                    const float t = s + pdi;
                    violh = fmaxf(violh, t);
                    magh = fmaxf(magh, __builtin_fabsf(s) + __builtin_fabsf(pdi));
                    wmin = fminf(wmin, wi);
                    gap -= (double)wi * (double)t;
                    violz = fmaxf(violz, ui + pdi);
                }
            }
            w[r] = __builtin_fmaf(bnext, yp - yi, yp);
            ys[r] = yp;
        }
        constexpr int nw = kFlatBlock / 64;
        if (chk) check_publish<float>(slots, violz, violh, wmin, gap, magh);
        __syncthreads();
        it = v + 1;
        if (chk) {
            const int st1 = check_stage1<float>(slots, nw, a.L, a.tol, a.tol_gap);
            bool verified = false;
            if (st1 & 1) {  // (A) nominated: decide on the direct flat chain G_L z, reset u to it
                float vc = -INFINITY, mcz = 0.0f;
                for (int r = tid; r < m; r += kFlatBlock) {
                    const float cz = flat_row4(GLT, zs, r, Nh, n_u, mc, m);
                    us[r] = cz;
                    vc = fmaxf(vc, cz + pd[r]);
                    mcz = fmaxf(mcz, __builtin_fabsf(cz) + __builtin_fabsf(pd[r]));
                }
                check_publish<float>(slots + nw, vc, vc, vc, 0.0, mcz);
                __syncthreads();
                verified = check_verify<float>(slots + nw, nw, a.L, a.tol);
            }
            done = check_code(st1, verified);
        }
        if (done) break;
    }
    const float* zout = done == 2 ? zh : zs;  // test (B) certifies zhat
    for (int i = tid; i < n; i += kFlatBlock) zg[i] = zout[i];
    for (int i = tid; i < m; i += kFlatBlock) yg[i] = ys[i];
    if (tid == 0) {
        a.iters[b] = it;
        a.conv[b] = done;
    }
}

static size_t flat_vec_bytes(int n, int m) {
    return sizeof(float) * (size_t)(4 * m + 3 * n + 1) + sizeof(CheckSlot) * 2 * (kFlatBlock / 64) + 16;
}

hipError_t launch_flat(const SolveArgs<float>& a, hipStream_t s) {
    const int Nh = a.n / a.n_u;
    const size_t mat = 2 * sizeof(float) * (size_t)Nh * a.m;
    SolveArgs<float> b = a;
    b.flat_staged = mat <= kFlatStageMax;
    const size_t lds = flat_vec_bytes(a.n, a.m) + (b.flat_staged ? mat : 0);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)gpad_flat_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(gpad_flat_kernel, dim3(a.batch), dim3(kFlatBlock), lds, s, b);
    return hipGetLastError();
}

// ---- per-step entry points (StepTwoGPADFlatSequential / StepFourGPADFlatParRows with the CPU
//      step's arithmetic; flat matrices row-major as the reference stores them) -------------
__global__ void step2_flat_kernel(const float* __restrict__ MGf, const float* __restrict__ w,
                                  const float* __restrict__ gP, float* __restrict__ zhat, int Nh,
                                  int n_u, int m) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= Nh * n_u) return;
    zhat[r] = flat_row2(MGf, w, r / n_u, r % n_u, n_u, 4 * n_u * Nh, m) - gP[r];
}

__global__ void step4_flat_kernel(const float* __restrict__ GLf, float* __restrict__ yp1,
                                  const float* __restrict__ w, const float* __restrict__ pD,
                                  const float* __restrict__ zhat, int Nh, int n_u, int m) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const int mc = 4 * n_u * Nh;
    float acc = 0.0f;
    for (int t = 0; t < Nh; ++t) {  // G_L row-major here (m x Nh), as kernel_functions.cu:98-104
        const float g = GLf[(size_t)r * Nh + t];
        if (r < mc) {
            acc = __builtin_fmaf(g, zhat[t * n_u + (r % n_u)], acc);
        } else {
            for (int k = 0; k < n_u; ++k) acc = __builtin_fmaf(g, zhat[t * n_u + k], acc);
        }
    }
    const float s = (acc + w[r]) + pD[r];
    yp1[r] = s < 0.0f ? 0.0f : s;
}

hipError_t launch_step2_flat(const float* MGf, const float* w, const float* gP, float* zhat, int Nh, int n_u,
                             int m, hipStream_t s) {
    const int n = Nh * n_u;
    hipLaunchKernelGGL(step2_flat_kernel, dim3((n + 255) / 256), dim3(256), 0, s, MGf, w, gP, zhat, Nh, n_u, m);
    return hipGetLastError();
}

hipError_t launch_step4_flat(const float* GLf, float* yp1, const float* w, const float* pD, const float* zhat,
                             int Nh, int n_u, int m, hipStream_t s) {
    hipLaunchKernelGGL(step4_flat_kernel, dim3((m + 255) / 256), dim3(256), 0, s, GLf, yp1, w, pD, zhat, Nh,
                       n_u, m);
    return hipGetLastError();
}

// flat G_L (m x Nh, row-major) -> t-major image (Nh x m) for the solve kernel
__global__ void transpose_flat_kernel(const float* __restrict__ in, float* __restrict__ out, int rows,
                                      int cols) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rows * cols) return;
    const int r = e / cols, c = e % cols;
    out[(size_t)c * rows + r] = in[e];
}

hipError_t launch_transpose_flat(const float* in, float* out, int rows, int cols, hipStream_t s) {
    const int tot = rows * cols;
    hipLaunchKernelGGL(transpose_flat_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, in, out, rows, cols);
    return hipGetLastError();
}

// flat G_L (m x Nh row-major) -> the full constraint rows as a k-major image out[k*ld + r]
// (k < n = n_u Nh): row r < 4 n_u Nh touches column t n_u + r % n_u, coupling rows every column
__global__ void expand_flat_gl_kernel(const float* __restrict__ GLf, float* __restrict__ out, int Nh,
                                      int n_u, int m, int ld) {
    const int n = Nh * n_u, mc = 4 * n_u * Nh;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * ld) return;
    const int k = e / ld, r = e % ld;
    const int t = k / n_u, c = k % n_u;
    float v = 0.0f;
    if (r < m && (r >= mc || c == r % n_u)) v = GLf[(size_t)r * Nh + t];
    out[e] = v;
}

hipError_t launch_expand_flat_gl(const float* GLf, float* out, int Nh, int n_u, int m, int ld, hipStream_t s) {
    const int tot = Nh * n_u * ld;
    hipLaunchKernelGGL(expand_flat_gl_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, GLf, out, Nh, n_u, m, ld);
    return hipGetLastError();
}

}  // namespace gpad
