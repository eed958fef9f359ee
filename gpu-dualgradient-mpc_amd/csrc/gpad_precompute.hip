// gpad_precompute.hip -- the one-time QP precompute of acceldualgrad.m:11,20-21 on the device
// ("one-time batched Cholesky/inverse of H"), fp64:
//   L  = ||H||_F^2            (acceldualgrad.m:11)
//   ML = inv(H) A_i'  (n x m) (acceldualgrad.m:20, M_G)
//   gP = inv(H) f'    (n)     (acceldualgrad.m:21, g_P; optional)
// The reference forms inv(H) explicitly and multiplies; here one workgroup per instance runs
// Gauss-Jordan elimination on the augmented rows [H | A_i' | f'] (no pivoting: H is symmetric
// positive definite), which yields inv(H) [A_i' | f'] directly -- the same quantity, different
// rounding (~1e-15 relative; parity is a tolerance, tests/test_precompute.py).  The augmented
// rows live in a global workspace (L2-resident for the sizes here); the pivot row and the
// pivot column of each step are staged in LDS.
#include <hip/hip_runtime.h>

#include <cmath>

#include "gpad_internal.h"

namespace gpad {

constexpr int kPreBlock = 1024;

// block b (instance b0 + b): H + sH b, A + sA b, nf right-hand sides f + sF b + c n (c < nf)
__global__ __launch_bounds__(kPreBlock) void precompute_gj_kernel(int n, int m, int nf, const double* __restrict__ H,
                                                                  long long sH, const double* __restrict__ A,
                                                                  long long sA, const double* __restrict__ f,
                                                                  long long sF, double* __restrict__ work,
                                                                  double* __restrict__ ML, double* __restrict__ gP,
                                                                  double* __restrict__ Lout, int b0) {
    extern __shared__ double pre_lds[];
    const int W = n + m + nf;  // augmented row length
    double* rowk = pre_lds;        // [W]
    double* colk = pre_lds + W;    // [n]
    __shared__ double red[kPreBlock / 64];
    const int b = b0 + blockIdx.x;
    const int tid = threadIdx.x;
    const double* Hb = H + sH * b;
    const double* Ab = A + sA * b;
    double* Wb = work + (size_t)blockIdx.x * n * W;
    // ---- L = ||H||_F^2 (acceldualgrad.m:11) and the augmented rows ----------------------------
    double ss = 0.0;
    for (int e = tid; e < n * n; e += kPreBlock) ss = fma(Hb[e], Hb[e], ss);
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    for (long long e = tid; e < (long long)n * W; e += kPreBlock) {
        const int i = (int)(e / W), j = (int)(e - (long long)i * W);
        double v;
        if (j < n) v = Hb[(size_t)i * n + j];
        else if (j < n + m) v = Ab[(size_t)(j - n) * n + i];  // A_i' (A_i is m x n row-major)
        else v = f ? f[sF * b + (size_t)(j - n - m) * n + i] : (j - n - m == i ? 1.0 : 0.0);  // f null: I
        Wb[e] = v;
    }
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
        for (int w = 0; w < kPreBlock / 64; ++w) s += red[w];
        const double nf = sqrt(s);
        Lout[b] = nf * nf;  // norm(H, 'fro')^2
    }
    // ---- Gauss-Jordan: step k normalises row k and eliminates column k from every other row ---
    for (int k = 0; k < n; ++k) {
        const double piv = Wb[(size_t)k * W + k];
        for (int j = k + 1 + tid; j < W; j += kPreBlock) {
            const double v = Wb[(size_t)k * W + j] / piv;
            rowk[j] = v;
            Wb[(size_t)k * W + j] = v;
        }
        for (int i = tid; i < n; i += kPreBlock) colk[i] = i == k ? 0.0 : Wb[(size_t)i * W + k];
        __syncthreads();
        // rows over the 16 waves, columns over the lanes (coalesced row segments)
        for (int i = tid >> 6; i < n; i += kPreBlock / 64) {
            const double c = colk[i];
            if (c == 0.0) continue;
            double* Wi = Wb + (size_t)i * W;
            for (int j = k + 1 + (tid & 63); j < W; j += 64) Wi[j] = fma(-c, rowk[j], Wi[j]);
        }
        __syncthreads();
    }
    // ---- outputs: ML = inv(H) A_i' (n x m row-major), gP = inv(H) f' ---------------------------
    double* MLb = ML + (size_t)b * n * m;
    for (long long e = tid; e < (long long)n * m; e += kPreBlock) {
        const int i = (int)(e / m), j = (int)(e - (long long)i * m);
        MLb[e] = Wb[(size_t)i * W + n + j];
    }
    for (long long e = tid; e < (long long)nf * n; e += kPreBlock) {
        const int c = (int)(e / n), i = (int)(e - (long long)c * n);
        gP[sF * b + (size_t)c * n + i] = Wb[(size_t)i * W + n + m + c];
    }
}

// gP[b][i] = sum_c inv(H)[i][c] f[b][c], c ascending; Hinv column-major as the elimination
// writes it (Hinv[c * n + i]), one thread per (b, i)
__global__ void apply_inv_kernel(int n, int batch, const double* __restrict__ Hinv, const double* __restrict__ f,
                                 double* __restrict__ gP) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long long)batch * n) return;
    const int b = (int)(e / n), i = (int)(e - (long long)b * n);
    const double* fb = f + (size_t)b * n;
    double acc = 0.0;
    for (int c = 0; c < n; ++c) acc = fma(Hinv[(size_t)c * n + i], fb[c], acc);
    gP[e] = acc;
}

hipError_t launch_apply_inv(int n, int batch, const double* Hinv, const double* f, double* gP, hipStream_t s) {
    const long long tot = (long long)batch * n;
    hipLaunchKernelGGL(apply_inv_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, n, batch, Hinv, f, gP);
    return hipGetLastError();
}

size_t precompute_work_bytes(int n, int m, int nf, int count) {
    return sizeof(double) * (size_t)count * n * (n + m + nf);
}

bool precompute_supported(int n, int m, int nf) {
    return n > 0 && m >= 0 && nf >= 0 && 2 * n + m + nf <= 8000;  // pivot row + column in 64 KiB of LDS
}

hipError_t launch_precompute(int n, int m, int nf, const double* H, long long sH, const double* A, long long sA,
                             const double* f, long long sF, double* work, double* ML, double* gP, double* L, int b0,
                             int count, hipStream_t s) {
    const size_t lds = sizeof(double) * (size_t)(2 * n + m + nf);
    hipLaunchKernelGGL(precompute_gj_kernel, dim3(count), dim3(kPreBlock), lds, s, n, m, nf, H, sH, A, sA, f, sF,
                       work, ML, gP, L, b0);
    return hipGetLastError();
}

}  // namespace gpad
