// gpad_kernels.hip -- GPAD inner-loop kernels for MI355X (gfx950, CDNA4, wave64).
//
// Two fused, persistent solve kernels (the whole iteration loop of main.cu:160-175 lives
// inside ONE launch: no per-iteration launches, host syncs or y-copy kernels):
//
//   gpad_stream_kernel<T>   generic family (f32 / f64, any n, m up to the LDS budget).
//                           One workgroup per instance; -ML and G/L are read every
//                           iteration from HBM/L2 in k-major layout, 4 rows per lane
//                           (one 16-B/32-B load per lane per k -> 1 KiB per wave-instruction,
//                           fully coalesced), 8 k-steps in flight per lane.
//   gpad_resident_kernel<K> latency family (f32, n, m <= 208).  One workgroup per
//                           instance; each lane holds ONE matrix row in VGPRs for the
//                           whole solve (loaded once), so an iteration touches no memory but
//                           LDS.  Waves [0,nA) own the rows of -ML, waves [nA,nA+nB) the rows
//                           of G/L; w and zhat are broadcast through LDS (ds_read_b128).
//
// Numerics (bit-exact with the reference CPU path, see oracle/gpad_oracle.h): every dot
// product is ONE sequential fmaf chain per output row, k = 0..K-1 from +0 -- exactly what
// seq_functions.cpp:61,82 compute under FMA contraction and what the reference's
// one-thread-per-row CUDA kernels compute (kernel_functions.cu:46-61,176-191).  The file is
// compiled with -ffp-contract=off; every fused multiply-add is an explicit __builtin_fma.
//
// Per-step kernels mirroring kernel_functions.h one-for-one are at the end of this file.

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include <utility>

#include "gpad_chain.h"
#include "gpad_internal.h"

namespace gpad {

// =========================================================================================
// gpad_stream_kernel
// =========================================================================================
constexpr int kStreamBlock = 256;
static_assert(kStreamBlock / 64 <= 8, "test slots: one per lane over lanes 0..7 (gpad_chain.h check_stage1)");
constexpr int kUnrollK = 8;

template <typename T>
struct StreamLds {
    T *w, *zh, *zs, *ys, *gp, *pd, *us;
    CheckSlot* slots;
    double* red;  // [waves] block-sum partials of the value functions
    double* zp;   // [ldn] z(y+) of the dual function (value-function branches only)
};

template <typename T>
__device__ __forceinline__ StreamLds<T> stream_lds(unsigned char* smem, int ldn, int ldm) {
    StreamLds<T> s;
    s.w = reinterpret_cast<T*>(smem);   // [ldm] current w (read by every lane in phase 1)
    s.zh = s.w + ldm;                   // [ldn] zhat (read by every lane in phase 2)
    s.zs = s.zh + ldn;                  // [ldn] z (averaged primal)
    s.ys = s.zs + ldn;                  // [ldm] y
    s.gp = s.ys + ldm;                  // [ldn] g_P
    s.pd = s.gp + ldn;                  // [ldm] p_D
    s.us = s.pd + ldm;                  // [ldm] u = G_L z (termination test, by recursion)
    s.slots = reinterpret_cast<CheckSlot*>(s.us + ldm);  // [2][waves]: test, verification of (A)
    s.red = reinterpret_cast<double*>(s.slots + 2 * (kStreamBlock / 64));
    s.zp = s.red + kStreamBlock / 64;
    return s;
}

// LDS bytes of the stream kernel: the vectors, the test slots and (value branches) the block-sum
// partials and z(y+)
template <typename T>
size_t stream_lds_bytes(int ldn, int ldm, bool value) {
    return sizeof(T) * (size_t)(3 * ldn + 4 * ldm) + sizeof(CheckSlot) * 2 * (kStreamBlock / 64) +
           (value ? sizeof(double) * (size_t)(kStreamBlock / 64 + ldn) : 0);
}

// acc[r] = sum_k Mt[k*ld + r0 + r] * v[k], sequential in k, 4 rows per lane.
template <typename T>
__device__ __forceinline__ void chain4(const T* __restrict__ Mt, int ld, int r0, const T* v, int K,
                                       T (&acc)[4]) {
    using V = typename V4<T>::type;
    const T* col = Mt + r0;
    int k = 0;
    for (; k + kUnrollK <= K; k += kUnrollK) {
        V a[kUnrollK];
#pragma unroll
        for (int u = 0; u < kUnrollK; ++u) a[u] = *reinterpret_cast<const V*>(col + (size_t)(k + u) * ld);
#pragma unroll
        for (int u = 0; u < kUnrollK; ++u) {
            const T vk = v[k + u];
            acc[0] = fmad(a[u].x, vk, acc[0]);
            acc[1] = fmad(a[u].y, vk, acc[1]);
            acc[2] = fmad(a[u].z, vk, acc[2]);
            acc[3] = fmad(a[u].w, vk, acc[3]);
        }
    }
    for (; k < K; ++k) {
        const V a = *reinterpret_cast<const V*>(col + (size_t)k * ld);
        const T vk = v[k];
        acc[0] = fmad(a.x, vk, acc[0]);
        acc[1] = fmad(a.y, vk, acc[1]);
        acc[2] = fmad(a.z, vk, acc[2]);
        acc[3] = fmad(a.w, vk, acc[3]);
    }
}

// acc[r] = sum_k Mt[k*ld + r0 + r] * v[k] as fp64 fma chains (ascending k) over the run's own
// matrix and vector values: the products of the value-function branches
template <typename T, typename V>
__device__ __forceinline__ void chain4d(const T* __restrict__ Mt, int ld, int r0, const V* v, int K,
                                        double (&acc)[4]) {
    using W = typename V4<T>::type;
    const T* col = Mt + r0;
    for (int k = 0; k < K; ++k) {
        const W x = *reinterpret_cast<const W*>(col + (size_t)k * ld);
        const double vk = (double)v[k];
        acc[0] = __builtin_fma((double)x.x, vk, acc[0]);
        acc[1] = __builtin_fma((double)x.y, vk, acc[1]);
        acc[2] = __builtin_fma((double)x.z, vk, acc[2]);
        acc[3] = __builtin_fma((double)x.w, vk, acc[3]);
    }
}

// sum over the workgroup (every thread gets it): wave sums, then the waves' partials in order
__device__ __forceinline__ double block_sum(double v, double* red) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < kStreamBlock / 64; ++i) t += red[i];
    __syncthreads();  // red is reused by the next sum
    return t;
}

// valuefcn V(x) = sum_i (x_i / 2 + M_i) (H x)_i (acceldualgrad.m:30 with f = H M)
template <typename T, typename V>
__device__ __forceinline__ double stream_valuefcn(const T* __restrict__ Hq, int ldn, int n, const V* x, const T* gp,
                                                  double* red) {
    double part = 0.0;
    for (int r0 = 4 * threadIdx.x; r0 < n; r0 += 4 * kStreamBlock) {
        double hx[4] = {0.0, 0.0, 0.0, 0.0};
        chain4d<T, V>(Hq, ldn, r0, x, n, hx);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (r0 + r < n) part += (0.5 * (double)x[r0 + r] + (double)gp[r0 + r]) * hx[r];
    }
    return block_sum(part, red);
}

// The value-function branches of Algorithm 1 (acceldualgrad.m:73,76), reached after test (B)'s
// violation part passed (w_ok: w >= 0 with the gap term above e_V, else w not >= 0); the same
// fp64 quantities as orc_value_branch_f32 / _f64 (oracle/gpad_oracle.c).  Returns 3, 4 or 0.
template <typename T>
__device__ int stream_value_branch(const SolveArgs<T>& a, const StreamLds<T>& s, const T* __restrict__ MGt,
                                   const T* __restrict__ GLt, const T* __restrict__ Hq, bool w_ok, double gapL) {
    const int n = a.n, m = a.m, ldn = a.ldn, ldm = a.ldm;
    const double eV = a.tol_gap;
    const double V = stream_valuefcn<T, T>(Hq, ldn, n, s.zh, s.gp, s.red);
    if (w_ok) return gapL <= V * eV / (1.0 + eV) ? 3 : 0;  // :73
    // dualfcn(y+) = V(z(y+)) + y+'(G z(y+) - g), z(y+) = -ML y+ - M       (:31-33, :76)
    for (int r0 = 4 * threadIdx.x; r0 < n; r0 += 4 * kStreamBlock) {
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
        chain4d<T, T>(MGt, ldn, r0, s.ys, m, acc);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (r0 + r < n) s.zp[r0 + r] = acc[r] - (double)s.gp[r0 + r];
    }
    __syncthreads();
    const double Vp = stream_valuefcn<T, double>(Hq, ldn, n, s.zp, s.gp, s.red);
    double lin = 0.0;
    for (int r0 = 4 * threadIdx.x; r0 < m; r0 += 4 * kStreamBlock) {
        double c[4] = {0.0, 0.0, 0.0, 0.0};
        chain4d<T, double>(GLt, ldm, r0, s.zp, n, c);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (r0 + r < m) lin += (double)s.ys[r0 + r] * (c[r] + (double)s.pd[r0 + r]);
    }
    const double D = Vp + a.L * block_sum(lin, s.red);
    return V - D <= eV * (D > 1.0 ? D : 1.0) ? 4 : 0;  // :76
}

template <typename T>
__global__ __launch_bounds__(kStreamBlock) void gpad_stream_kernel(SolveArgs<T> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int b = blockIdx.x;
    const int n = a.n, m = a.m, ldn = a.ldn, ldm = a.ldm;
    const StreamLds<T> s = stream_lds<T>(smem, ldn, ldm);
    const T* __restrict__ MGt = a.MGt + (size_t)b * a.strideA;
    const T* __restrict__ GLt = a.GLt + (size_t)b * a.strideB;
    T* zg = a.z + (size_t)b * n;
    T* yg = a.y + (size_t)b * m;
    const T* gPg = a.gP + (size_t)b * a.ld_gP;
    const T* gg = a.g + (size_t)b * a.ld_g;
    const T beta0 = a.beta[0];

    for (int i = tid; i < ldn; i += kStreamBlock) {
        s.zs[i] = i < n ? zg[i] : T(0);
        s.gp[i] = i < n ? gPg[i] : T(0);
        s.zh[i] = T(0);
    }
    for (int i = tid; i < ldm; i += kStreamBlock) {
        const T yv = i < m ? yg[i] : T(0);
        s.ys[i] = yv;
        s.pd[i] = i < m ? (T)(a.gscale * (double)gg[i]) : T(0);
        s.w[i] = fmad(beta0, yv - yv, yv);  // 8a with y_0 = y_{-1} (acceldualgrad.m:16,43)
    }
    __syncthreads();
    const bool use_tol = a.tol > 0.0;
    if (use_tol) {  // u = G_L z_{-1}; afterwards u follows the 8c recursion (u = G_L z exactly)
        for (int r0 = 4 * tid; r0 < m; r0 += 4 * kStreamBlock) {
            T c[4] = {T(0), T(0), T(0), T(0)};
            chain4<T>(GLt, ldm, r0, s.zs, n, c);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (r0 + r < m) s.us[r0 + r] = c[r];
        }
    }

    const int nwaves = kStreamBlock / 64;
    int it = 0;
    int done = 0;
    for (int v = 0; v < a.N; ++v) {
        const T th = a.theta[v];
        const T omt = T(1) - th;
        const T bnext = a.beta[v + 1];
        // ---- phase 1: 8b + 8c, rows of -ML ----------------------------------------------
        for (int r0 = 4 * tid; r0 < n; r0 += 4 * kStreamBlock) {
            T acc[4] = {T(0), T(0), T(0), T(0)};
            chain4<T>(MGt, ldn, r0, s.w, m, acc);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = r0 + r;
                if (i < n) {
                    const T zhv = acc[r] - s.gp[i];                 // seq_functions.cpp:63
                    s.zh[i] = zhv;
                    s.zs[i] = fmad(omt, s.zs[i], th * zhv);         // seq_functions.cpp:70
                }
            }
        }
        __syncthreads();
        // ---- phase 2: 8d + next 8a, rows of G/L ------------------------------------------
        const bool chk = use_tol && ((v + 1) % a.check_every) == 0;
        T violz = neg_inf<T>(), violh = neg_inf<T>(), wmin = -neg_inf<T>(), magh = T(0);
        double gap = 0.0;
        for (int r0 = 4 * tid; r0 < m; r0 += 4 * kStreamBlock) {
            T c[4] = {T(0), T(0), T(0), T(0)};
            chain4<T>(GLt, ldm, r0, s.zh, n, c);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = r0 + r;
                if (i < m) {
                    const T wi = s.w[i], pdi = s.pd[i], yi = s.ys[i];
                    const T sv = (wi + pdi) + c[r];                 // seq_functions.cpp:84
                    const T yp = (absd(sv) + sv) * T(0.5);          // seq_functions.cpp:85
                    if (use_tol) {
                        const T ui = fmad(omt, s.us[i], th * c[r]);  // u = G_L z (8c form)
                        s.us[i] = ui;
                        if (chk) {
                            const T t = c[r] + pdi;
                            violh = fmax(violh, t);
                            magh = fmax(magh, absd(c[r]) + absd(pdi));
                            wmin = fmin(wmin, wi);
                            gap -= (double)wi * (double)t;
                            violz = fmax(violz, ui + pdi);
                        }
                    }
                    s.w[i] = fmad(bnext, yp - yi, yp);               // next 8a
                    s.ys[i] = yp;
                }
            }
        }
        if (chk) check_publish<T>(s.slots, violz, violh, wmin, gap, magh);
        __syncthreads();
        it = v + 1;
        if (chk) {
            const int st1 = check_stage1<T>(s.slots, nwaves, a.L, a.tol, a.tol_gap);
            bool verified = false;
            if (st1 & 1) {  // (A) nominated: decide on the direct chain G_L z, reset u to it
                T vc = neg_inf<T>(), mc = T(0);
                for (int r0 = 4 * tid; r0 < m; r0 += 4 * kStreamBlock) {
                    T c[4] = {T(0), T(0), T(0), T(0)};
                    chain4<T>(GLt, ldm, r0, s.zs, n, c);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int i = r0 + r;
                        if (i < m) {
                            s.us[i] = c[r];
                            vc = fmax(vc, c[r] + s.pd[i]);
                            mc = fmax(mc, absd(c[r]) + absd(s.pd[i]));
                        }
                    }
                }
                check_publish<T>(s.slots + nwaves, vc, vc, vc, 0.0, mc);
                __syncthreads();
                verified = check_verify<T>(s.slots + nwaves, nwaves, a.L, a.tol);
            }
            done = check_code(st1, verified);
            if (!done && a.Hq) {  // value-function branches where the MATLAB test reaches them
                double vh = -INFINITY, mh = 0.0, wm = INFINITY, gq = 0.0;
                for (int i = 0; i < nwaves; ++i) {
                    vh = fmax(vh, s.slots[i].violh);
                    mh = fmax(mh, s.slots[i].magh);
                    wm = fmin(wm, s.slots[i].wmin);
                    gq += s.slots[i].gap;
                }
                if (viol_ok(vh, mh, a.L, a.tol, ViolMargin<T>::value))  // uniform
                    done = stream_value_branch<T>(a, s, MGt, GLt, a.Hq + (size_t)b * a.strideHq, wm >= 0.0,
                                                  gq * a.L);
            }
        }
        if (done) break;
    }
    const T* zout = done >= 2 ? s.zh : s.zs;  // tests (B), (B'), (B'') certify zhat
    for (int i = tid; i < n; i += kStreamBlock) zg[i] = zout[i];
    for (int i = tid; i < m; i += kStreamBlock) yg[i] = s.ys[i];
    if (tid == 0) {
        a.iters[b] = it;
        a.conv[b] = done;
    }
}

template <typename T>
hipError_t launch_stream(const SolveArgs<T>& a, hipStream_t st) {
    const size_t lds = stream_lds_bytes<T>(a.ldn, a.ldm, a.Hq != nullptr);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)gpad_stream_kernel<T>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(gpad_stream_kernel<T>, dim3(a.batch), dim3(kStreamBlock), lds, st, a);
    return hipGetLastError();
}
template hipError_t launch_stream<float>(const SolveArgs<float>&, hipStream_t);
template hipError_t launch_stream<double>(const SolveArgs<double>&, hipStream_t);


// FLAT = the structure-exploiting battery variant (gpad_flat.hip header; seq_functions.cpp:5-43):
// a primal row (i, j) carries only its 6N structural coefficients (KA = bucket(6N)) and chains
// over a per-cell permuted copy of w (wP[j][s] = w[j + n_u s], s < 4N; w[4 n_u N + s - 4N] after),
// so the 8b half-iteration is 6N steps long instead of m.  A-lanes are laid out so every 16-lane
// DPP row serves one cell j (lane = 16 times of that cell), hence one broadcast segment per row.
// Constraint rows chain over the natural zhat with the flat G_L expanded to full rows (exact: the
// added terms are exact zeros), with the flat step's epilogue (s + w) + p_D, y < 0 -> 0.
constexpr int kFlatMaxCells = 16;

// Iteration anatomy stamps of the resident kernel (diagnostic builds only, -DGPAD_STAMP): shader
// clock of workgroup 0, every wave, iterations [101, 105), at six points -- loop top, 8b chain done,
// after the first barrier, 8d chain done, its epilogue done, after the second barrier
// (gpad_debug_res_stamps, tools/stamp_resident.py).
#ifdef GPAD_STAMP
__device__ unsigned long long g_res_stamps[8][4][6];
#define GPAD_RSTAMP(P)                                                                         \
    do {                                                                                       \
        if (blockIdx.x == 0 && v >= 101 && v < 105 && (tid & 63) == 0)                        \
            g_res_stamps[tid >> 6][v - 101][P] = __builtin_amdgcn_s_memtime();                 \
    } while (0)
hipError_t read_res_stamps(unsigned long long* out, size_t bytes) {
    if (bytes > sizeof(g_res_stamps)) bytes = sizeof(g_res_stamps);
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_res_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#else
#define GPAD_RSTAMP(P) \
    do {               \
    } while (0)
#endif

template <int KA, int KB, bool FLAT>
__global__ __launch_bounds__(kResidentMaxThreads) void gpad_resident_kernel(SolveArgs<float> a) {
    constexpr int K = KA > KB ? KA : KB;
    constexpr int PA = (KA + 63) / 64 * 64, PB = (KB + 63) / 64 * 64;  // whole 64-element groups
    __shared__ __attribute__((aligned(16))) float w_l[FLAT ? kFlatMaxCells * PA : PA];  // w (flat: wP)
    __shared__ __attribute__((aligned(16))) float zh_l[PB];  // zhat, broadcast to G/L rows
    __shared__ __attribute__((aligned(16))) float z_l[PB];   // z_{-1}, to seed u = G_L z
    __shared__ CheckSlot slots[2][kResidentMaxThreads / 64];  // test, verification of (A)

    const int tid = threadIdx.x;
    const int b = blockIdx.x;
    const int n = a.n, m = a.m;
    const int n_u = FLAT ? a.n_u : 1, Nh = FLAT ? n / n_u : 0, mc = 4 * n_u * Nh;
    const int nq = (Nh + 15) >> 4;  // flat: 16-lane DPP rows per cell
    const int nA = FLAT ? (n_u * nq * 16 + 63) >> 6 : (n + 63) >> 6;
    const int nwaves = blockDim.x >> 6;
    const bool isA = (tid >> 6) < nA;               // wave-uniform role
    int row = isA ? tid : tid - 64 * nA;
    int cell = 0;                                   // flat A-lanes: cell j of this lane
    bool live = isA ? row < n : row < m;
    if (FLAT && isA) {  // lane -> (cell j, time i): row r = i n_u + j
        const int q = tid >> 4, i = 16 * (q % nq) + (tid & 15);
        cell = q / nq;
        live = cell < n_u && i < Nh;
        row = live ? i * n_u + cell : 0;
    }

    // preload the row once
    float r[K];
    if (FLAT && isA) {  // flat -ML row i (Nh x m, row-major): the 6N structural entries
        const float* Mi = a.MGt + (size_t)(row / n_u) * m;
#pragma unroll
        for (int k = 0; k < K; ++k)
            r[k] = (!live || k >= 6 * Nh) ? 0.0f : Mi[k < 4 * Nh ? cell + n_u * k : mc + (k - 4 * Nh)];
    } else {  // k-major images: consecutive lanes read consecutive words
        const int len = isA ? m : n;
        const float* __restrict__ Mt = isA ? a.MGt + (size_t)b * a.strideA : a.GLt + (size_t)b * a.strideB;
        const int ld = isA ? a.ldn : a.ldm;
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = (live && k < len) ? Mt[(size_t)k * ld + row] : 0.0f;
    }
    // where constraint row `row` lands in the A-side vector
    auto put_w = [&](float wv) {
        if constexpr (FLAT) {
            if (row < mc) {
                w_l[(row % n_u) * PA + row / n_u] = wv;
            } else {
                for (int j = 0; j < n_u; ++j) w_l[j * PA + 4 * Nh + (row - mc)] = wv;
            }
        } else {
            w_l[row] = wv;
        }
    };
    const float* wvec = FLAT ? w_l + cell * PA : w_l;  // this lane's broadcast segment

    float* zg = a.z + (size_t)b * n;
    float* yg = a.y + (size_t)b * m;
    float zi = 0.0f, gpi = 0.0f, yi = 0.0f, pdi = 0.0f, wi = 0.0f;
    if (isA) {
        if (live) {
            zi = zg[row];
            gpi = a.gP[(size_t)b * a.ld_gP + row];
        }
    } else if (live) {
        yi = yg[row];
        pdi = (float)(a.gscale * (double)a.g[(size_t)b * a.ld_g + row]);
        wi = __builtin_fmaf(a.beta[0], yi - yi, yi);
    }
    for (int i = tid; i < (FLAT ? kFlatMaxCells * PA : PA); i += blockDim.x) w_l[i] = 0.0f;
    for (int i = tid; i < PB; i += blockDim.x) {
        zh_l[i] = 0.0f;
        z_l[i] = 0.0f;
    }
    __syncthreads();
    if (!isA && live) put_w(wi);
    if (isA && live) z_l[row] = zi;
    __syncthreads();
    const bool use_tol = a.tol > 0.0;
    float ui = 0.0f;  // u = G_L z: seeded once, then the 8c recursion (no extra chain per test)
    if (use_tol && !isA) {
        const float us = chain_regs<KB, K>(r, z_l);  // (uniform control flow around the DPP chain)
        ui = us;
    }

    int it = 0;
    int done = 0;
    float zhi = 0.0f;
    // theta/beta are fetched one iteration ahead, by each role in its idle half (the A waves while
    // the 8d chains run, the B waves while the 8b chains run), and the test period is a countdown:
    // between barrier 2 and the next 8b chain only the loop branch remains (tables hold N + 2
    // entries).
    float th = a.theta[0], bn = a.beta[1];
    float th_next = 0.0f, bn_next = 0.0f;
    const int Kc = a.check_every;
    int kc = Kc;  // iterations to the next test: chk <=> (v + 1) % Kc == 0
    for (int v = 0; v < a.N; ++v) {
        const bool chk = use_tol && --kc == 0;
        if (chk) kc = Kc;
        GPAD_RSTAMP(0);
        if (isA) {  // ---- 8b + 8c --------------------------------------------------------
            const float acc = chain_regs<KA, K>(r, wvec);
            GPAD_RSTAMP(1);
            if (live) {
                const float zhv = acc - gpi;
                zh_l[row] = zhv;  // (the exchange first: 8c is off the critical path)
                zi = __builtin_fmaf(1.0f - th, zi, th * zhv);
                zhi = zhv;
            }
        } else {
            th_next = a.theta[v + 1];
            bn_next = a.beta[v + 2];
        }
        __syncthreads();
        GPAD_RSTAMP(2);
        float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY, magh = 0.0f;
        double gap = 0.0;
        if (!isA) {  // ---- 8d + next 8a ------------------------------------------------
            const float c = chain_regs<KB, K>(r, zh_l);
            GPAD_RSTAMP(3);
            if (live) {
                float sv, yp;
                if constexpr (FLAT) {
                    sv = (c + wi) + pdi;             // seq_functions.cpp:37
                    yp = sv < 0.0f ? 0.0f : sv;      // seq_functions.cpp:40-42
                } else {
                    sv = (wi + pdi) + c;             // seq_functions.cpp:84
                    yp = (__builtin_fabsf(sv) + sv) * 0.5f;
                }
                const float wn = __builtin_fmaf(bn, yp - yi, yp);
                put_w(wn);  // (the exchange first: u and the test partials are off the critical path)
                if (use_tol) ui = __builtin_fmaf(1.0f - th, ui, th * c);
                if (chk) {
                    const float t = c + pdi;
                    violh = t;
                    magh = __builtin_fabsf(c) + __builtin_fabsf(pdi);
                    wmin = wi;
                    gap = -((double)wi * (double)t);
                    violz = ui + pdi;
                }
                wi = wn;
                yi = yp;
            }
        } else {
            th_next = a.theta[v + 1];
            bn_next = a.beta[v + 2];
        }
        if (chk) check_publish<float>(slots[0], violz, violh, wmin, gap, magh);
        GPAD_RSTAMP(4);
        __syncthreads();
        GPAD_RSTAMP(5);
        it = v + 1;
        th = th_next;
        bn = bn_next;
        if (chk) {
            const int st1 = check_stage1<float>(slots[0], nwaves, a.L, a.tol, a.tol_gap);
            bool verified = false;
            if (st1 & 1) {  // (A) nominated: decide on the direct chain G_L z, reset u to it
                if (isA && live) z_l[row] = zi;
                __syncthreads();
                float vc = -INFINITY, mc = 0.0f;
                if (!isA) {
                    const float cz = chain_regs<KB, K>(r, z_l);
                    if (live) {
                        ui = cz;
                        vc = cz + pdi;
                        mc = __builtin_fabsf(cz) + __builtin_fabsf(pdi);
                    }
                }
                check_publish<float>(slots[1], vc, vc, vc, 0.0, mc);
                __syncthreads();
                verified = check_verify<float>(slots[1], nwaves, a.L, a.tol);
            }
            done = check_code(st1, verified);
        }
        if (done) break;
    }
    if (live) {
        if (isA)
            zg[row] = done == 2 ? zhi : zi;  // test (B) certifies zhat
        else
            yg[row] = yi;
    }
    if (tid == 0) {
        a.iters[b] = it;
        a.conv[b] = done;
    }
}


template <int KA, bool FLAT = false>
static void launch_res_b(int kb, dim3 g, dim3 bl, hipStream_t st, const SolveArgs<float>& a) {
    switch (kb) {
        case 32: hipLaunchKernelGGL((gpad_resident_kernel<KA, 32, FLAT>), g, bl, 0, st, a); break;
        case 64: hipLaunchKernelGGL((gpad_resident_kernel<KA, 64, FLAT>), g, bl, 0, st, a); break;
        case 96: hipLaunchKernelGGL((gpad_resident_kernel<KA, 96, FLAT>), g, bl, 0, st, a); break;
        case 128: hipLaunchKernelGGL((gpad_resident_kernel<KA, 128, FLAT>), g, bl, 0, st, a); break;
        case 160: hipLaunchKernelGGL((gpad_resident_kernel<KA, 160, FLAT>), g, bl, 0, st, a); break;
        case 192: hipLaunchKernelGGL((gpad_resident_kernel<KA, 192, FLAT>), g, bl, 0, st, a); break;
        case 200: hipLaunchKernelGGL((gpad_resident_kernel<KA, 200, FLAT>), g, bl, 0, st, a); break;
        default: hipLaunchKernelGGL((gpad_resident_kernel<KA, 208, FLAT>), g, bl, 0, st, a); break;
    }
}

bool resident_supported(int n, int m) {
    const int mx = n > m ? n : m;
    const int threads = 64 * (((n + 63) >> 6) + ((m + 63) >> 6));
    return mx <= kResidentMaxRow && threads <= kResidentMaxThreads && n > 0 && m > 0;
}

static hipError_t launch_resident_grid(const SolveArgs<float>& a, int nblocks, hipStream_t st) {
    const int threads = 64 * (((a.n + 63) >> 6) + ((a.m + 63) >> 6));
    const dim3 grid(nblocks), block(threads);
    const int ka = res_bucket(a.m), kb = res_bucket(a.n);  // A rows run over m, B rows over n
    switch (ka) {
        case 32: launch_res_b<32>(kb, grid, block, st, a); break;
        case 64: launch_res_b<64>(kb, grid, block, st, a); break;
        case 96: launch_res_b<96>(kb, grid, block, st, a); break;
        case 128: launch_res_b<128>(kb, grid, block, st, a); break;
        case 160: launch_res_b<160>(kb, grid, block, st, a); break;
        case 192: launch_res_b<192>(kb, grid, block, st, a); break;
        case 200: launch_res_b<200>(kb, grid, block, st, a); break;
        default: launch_res_b<208>(kb, grid, block, st, a); break;
    }
    return hipGetLastError();
}

hipError_t launch_resident(const SolveArgs<float>& a, hipStream_t st, bool* supported) {
    *supported = resident_supported(a.n, a.m);
    if (!*supported) return hipSuccess;
    return launch_resident_grid(a, a.batch, st);  // whole batch, from iteration 0
}

// flat battery variant: primal chains of 6N, constraint chains of n (flat G_L expanded to the
// k-major image a.GLt by the host at gpad_setup_flat); a.MGt = flat -ML (Nh x m row-major)
bool flat_resident_supported(int n, int m, int n_u) {
    if (n_u <= 0 || n_u > kFlatMaxCells || n % n_u) return false;
    const int Nh = n / n_u;
    const int laneA = n_u * ((Nh + 15) / 16) * 16;
    const int threads = 64 * ((laneA + 63) / 64) + 64 * ((m + 63) / 64);
    return 6 * Nh <= kResidentMaxRow && n <= kResidentMaxRow && threads <= kResidentMaxThreads &&
           m >= 4 * n;
}

hipError_t launch_flat_resident(const SolveArgs<float>& a, hipStream_t st) {
    const int Nh = a.n / a.n_u;
    const int laneA = a.n_u * ((Nh + 15) / 16) * 16;
    const int threads = 64 * ((laneA + 63) / 64) + 64 * ((a.m + 63) / 64);
    const SolveArgs<float>& b = a;
    const dim3 grid(a.batch), block(threads);
    const int ka = res_bucket(6 * Nh), kb = res_bucket(a.n);
    switch (ka) {
        case 32: launch_res_b<32, true>(kb, grid, block, st, b); break;
        case 64: launch_res_b<64, true>(kb, grid, block, st, b); break;
        case 96: launch_res_b<96, true>(kb, grid, block, st, b); break;
        case 128: launch_res_b<128, true>(kb, grid, block, st, b); break;
        case 160: launch_res_b<160, true>(kb, grid, block, st, b); break;
        case 192: launch_res_b<192, true>(kb, grid, block, st, b); break;
        case 200: launch_res_b<200, true>(kb, grid, block, st, b); break;
        default: launch_res_b<208, true>(kb, grid, block, st, b); break;
    }
    return hipGetLastError();
}

// =========================================================================================
// layout kernels
// =========================================================================================
// out[k*ld + i] = (T)(scale * in[i*cols + k]); 32x32 tiles through LDS so both the read of
// the row-major input and the write of the k-major output are coalesced.
template <typename T>
__global__ __launch_bounds__(256) void pack_kmajor_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                          int rows, int cols, int ld, double scale,
                                                          long long in_stride, long long out_stride) {
    __shared__ T tile[32][33];
    const T* src = in + (size_t)blockIdx.z * in_stride;
    T* dst = out + (size_t)blockIdx.z * out_stride;
    const int i0 = blockIdx.y * 32, k0 = blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int r = ty; r < 32; r += 8) {
        const int i = i0 + r, k = k0 + tx;
        tile[r][tx] = (i < rows && k < cols) ? (T)(scale * (double)src[(size_t)i * cols + k]) : T(0);
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int k = k0 + r, i = i0 + tx;
        if (k < cols && i < ld) dst[(size_t)k * ld + i] = tile[tx][r];
    }
}

template <typename T>
hipError_t launch_pack_kmajor(const T* in, T* out, int rows, int cols, int ld, double scale,
                              int batch, long long in_stride, long long out_stride, hipStream_t s) {
    const dim3 grid((cols + 31) / 32, (ld + 31) / 32, batch);
    hipLaunchKernelGGL(pack_kmajor_kernel<T>, grid, dim3(256), 0, s, in, out, rows, cols, ld, scale,
                       in_stride, out_stride);
    return hipGetLastError();
}
template hipError_t launch_pack_kmajor<float>(const float*, float*, int, int, int, double, int,
                                              long long, long long, hipStream_t);
template hipError_t launch_pack_kmajor<double>(const double*, double*, int, int, int, double, int,
                                               long long, long long, hipStream_t);

// =========================================================================================
// per-step kernels (kernel_functions.h:9-41 one for one; seq_functions.cpp semantics)
// =========================================================================================
__global__ void step1_kernel(const float* __restrict__ y, const float* __restrict__ ym1,
                             float* __restrict__ w, float beta, int m) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
        w[i] = __builtin_fmaf(beta, y[i] - ym1[i], y[i]);
}

// One lane per output row, sequential chain over the row (bit-exact with the CPU step);
// the vector is staged in LDS (as StepTwoGPADKernel's w_vs, kernel_functions.cu:37-42).
__global__ __launch_bounds__(256) void step_gemv_kernel(const float* __restrict__ A,
                                                        const float* __restrict__ x, int rows, int cols,
                                                        const float* __restrict__ bias, float bsign,
                                                        const float* __restrict__ addv,
                                                        float* __restrict__ out, int relu) {
    extern __shared__ __attribute__((aligned(16))) float xs[];
    for (int k = threadIdx.x; k < cols; k += blockDim.x) xs[k] = x[k];
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows) return;
    const float* row = A + (size_t)i * cols;
    float acc = 0.0f;
    for (int k = 0; k < cols; ++k) acc = __builtin_fmaf(row[k], xs[k], acc);
    if (!relu) {
        out[i] = acc - bias[i];  // 8b: zhat = MGneg w - gP
    } else {
        const float s = (addv[i] + bias[i]) + acc;  // 8d: (w + pD) + sum
        out[i] = (__builtin_fabsf(s) + s) * 0.5f;
    }
    (void)bsign;
}

__global__ void step3_kernel(float theta, const float* zm1, const float* __restrict__ zhat, float* z,
                             int n) {
    const float omt = 1.0f - theta;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        z[i] = __builtin_fmaf(omt, zm1[i], theta * zhat[i]);
}

static dim3 grid1d(int n) {
    int g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > 2048) g = 2048;
    return dim3(g);
}

hipError_t launch_step1(const float* y, const float* ym1, float* w, float beta, int m, hipStream_t s) {
    hipLaunchKernelGGL(step1_kernel, grid1d(m), dim3(256), 0, s, y, ym1, w, beta, m);
    return hipGetLastError();
}
hipError_t launch_step2(const float* MGneg, const float* w, const float* gP, float* zhat, int n,
                        int m, hipStream_t s) {
    hipLaunchKernelGGL(step_gemv_kernel, dim3((n + 255) / 256), dim3(256), sizeof(float) * (size_t)m, s,
                       MGneg, w, n, m, gP, -1.0f, (const float*)nullptr, zhat, 0);
    return hipGetLastError();
}
hipError_t launch_step3(float theta, const float* zm1, const float* zhat, float* z, int n,
                        hipStream_t s) {
    hipLaunchKernelGGL(step3_kernel, grid1d(n), dim3(256), 0, s, theta, zm1, zhat, z, n);
    return hipGetLastError();
}
hipError_t launch_step4(const float* GL, float* yp1, const float* w, const float* pD,
                        const float* zhat, int n, int m, hipStream_t s) {
    hipLaunchKernelGGL(step_gemv_kernel, dim3((m + 255) / 256), dim3(256), sizeof(float) * (size_t)n, s,
                       GL, zhat, m, n, pD, 1.0f, w, yp1, 1);
    return hipGetLastError();
}

}  // namespace gpad
