// gpad_plant.hip -- per-state QP data and plant update on the device.
//
// The reference rebuilds the state-dependent QP data on the host for every MPC step
// (gpad.m:80-85: f = x0'F, b_i(x0)) and then runs GPAD (acceldualgrad.m:20-23 precompute,
// :38-64 loop).  For an LTI plant both vectors are affine in the state x:
//     M(x) = M0 + PM x        (n;  PM = H^-1 F', so M = H^-1 f'   -- acceldualgrad.m:21)
//     g(x) = g0 + Pg x        (m;  b_i(x), gpad.m:85)
// and the receding-horizon update is x+ = A x + B u with u = z*[0:nu] (gpad.m:91-93).
// These kernels evaluate both on the device so a batch of states (or a whole closed-loop
// simulation) never leaves HBM.
//
// Arithmetic (restated by oracle/gpad_oracle.c orc_affine / orc_plant_step, bit-exact):
//   affine:  acc = c0[i] (0 if absent); for k < nx: acc = fma(P[i][k], x[k], acc)
//   plant :  acc = 0;  for k < nx: acc = fma(A[i][k], x[k], acc);
//                      for j < nu: acc = fma(B[i][j], u[j], acc)
// The work is O(batch (n + m) nx) per step -- a few hundred flops per instance against the
// O(iterations n m) of the solve -- so one thread per output row with the short chain in
// registers is the right shape; P rows are re-read from L2 by every instance.
#include "gpad_internal.h"

namespace gpad {

// out1[b][i] = affine row i (i < rows1) ; out2[b][j] = affine row j (j < rows2).
// grid.x covers the rows of one instance, grid.y the instances (grid-stride beyond 65535):
// no integer division on the path, the state x[b] is a broadcast read per block.
template <typename T>
__global__ __launch_bounds__(256) void affine2_kernel(const T* __restrict__ P1, const T* __restrict__ c1,
                                                      int rows1, T* __restrict__ out1,
                                                      const T* __restrict__ P2, const T* __restrict__ c2,
                                                      int rows2, T* __restrict__ out2,
                                                      const T* __restrict__ x, int nx, int batch) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows1 + rows2) return;
    const T* P = P1;
    const T* c = c1;
    T* out = out1;
    int ld = rows1;
    if (i >= rows1) {
        i -= rows1;
        P = P2;
        c = c2;
        out = out2;
        ld = rows2;
    }
    const T* Pi = P + (size_t)i * nx;
    const T c0 = c ? c[i] : T(0);
    for (int b = blockIdx.y; b < batch; b += gridDim.y) {
        const T* xb = x + (size_t)b * nx;
        T acc = c0;
        for (int k = 0; k < nx; ++k) acc = __builtin_fma(Pi[k], xb[k], acc);
        out[(size_t)b * ld + i] = acc;
    }
}

// xn[b] = A x[b] + B z[b][0:nu];  optional trajectories xs[b] = x[b], us[b] = z[b][0:nu]
template <typename T>
__global__ __launch_bounds__(256) void plant_step_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                         const T* __restrict__ x, const T* __restrict__ z,
                                                         long long ldz, T* __restrict__ xn, int nx, int nu,
                                                         int batch, T* __restrict__ xs, T* __restrict__ us) {
    const int per = nx > nu ? nx : nu;
    const long long total = (long long)batch * per;
    for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int b = (int)(t / per);
        const int i = (int)(t - (long long)b * per);
        const T* xb = x + (long long)b * nx;
        const T* ub = z + (long long)b * ldz;
        if (i < nx) {
            T acc = T(0);
            const T* Ai = A + (long long)i * nx;
            for (int k = 0; k < nx; ++k) acc = __builtin_fma(Ai[k], xb[k], acc);
            const T* Bi = B + (long long)i * nu;
            for (int j = 0; j < nu; ++j) acc = __builtin_fma(Bi[j], ub[j], acc);
            xn[(long long)b * nx + i] = acc;
            if (xs) xs[(long long)b * nx + i] = xb[i];
        }
        if (i < nu && us) us[(long long)b * nu + i] = ub[i];
    }
}

static dim3 grid_for(long long total) {
    long long blocks = (total + 255) / 256;
    if (blocks > 65535) blocks = 65535;
    if (blocks < 1) blocks = 1;
    return dim3((unsigned)blocks);
}

template <typename T>
hipError_t launch_affine2(const T* P1, const T* c1, int rows1, T* out1, const T* P2, const T* c2,
                          int rows2, T* out2, const T* x, int nx, int batch, hipStream_t s) {
    const dim3 grid((rows1 + rows2 + 255) / 256, batch < 65535 ? batch : 65535);
    hipLaunchKernelGGL(affine2_kernel<T>, grid, dim3(256), 0, s, P1, c1, rows1, out1, P2, c2, rows2, out2, x,
                       nx, batch);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_plant_step(const T* A, const T* B, const T* x, const T* z, long long ldz, T* xn, int nx,
                             int nu, int batch, T* xs, T* us, hipStream_t s) {
    const int per = nx > nu ? nx : nu;
    hipLaunchKernelGGL(plant_step_kernel<T>, grid_for((long long)batch * per), dim3(256), 0, s, A, B, x, z,
                       ldz, xn, nx, nu, batch, xs, us);
    return hipGetLastError();
}

template hipError_t launch_affine2<float>(const float*, const float*, int, float*, const float*,
                                          const float*, int, float*, const float*, int, int, hipStream_t);
template hipError_t launch_affine2<double>(const double*, const double*, int, double*, const double*,
                                           const double*, int, double*, const double*, int, int,
                                           hipStream_t);
template hipError_t launch_plant_step<float>(const float*, const float*, const float*, const float*,
                                             long long, float*, int, int, int, float*, float*, hipStream_t);
template hipError_t launch_plant_step<double>(const double*, const double*, const double*, const double*,
                                              long long, double*, int, int, int, double*, double*,
                                              hipStream_t);

// acc += sum of per-instance iteration counts (one workgroup; wave sums then one atomic per wave)
__global__ void accumulate_iters_kernel(const int* __restrict__ iters, long long count, long long* acc) {
    long long sum = 0;
    for (long long i = threadIdx.x; i < count; i += blockDim.x) sum += iters[i];
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(acc), (unsigned long long)sum);
}

hipError_t launch_accumulate_iters(const int* iters, long long count, long long* acc, hipStream_t s) {
    hipLaunchKernelGGL(accumulate_iters_kernel, dim3(1), dim3(1024), 0, s, iters, count, acc);
    return hipGetLastError();
}

// part[b] = max |g_i| of workgroup b, the other slots zeroed (the certification floor, include/gpad.h
// gpad_run): up to 1024 workgroups of 256 threads, 16 elements per thread and pass with the loads of
// a pass issued together (one pass at the C4 shard), each workgroup reducing through LDS into its
// own slot.  No atomics: hundreds of same-address atomics serialise at L2 (~30 us per solve
// measured); the host reduces the slots when it reads the stats.
template <typename T>
__global__ __launch_bounds__(256) void absmax_kernel(const T* __restrict__ g, long long count, double* part) {
    __shared__ double red[4];
    double mx = 0.0;
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long base = (long long)blockIdx.x * blockDim.x + threadIdx.x; base < count; base += 16 * stride) {
        T v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const long long i = base + u * stride;
            v[u] = i < count ? g[i] : T(0);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) mx = absmax_nan(mx, (double)v[u]);
    }
    for (int o = 32; o > 0; o >>= 1) mx = absmax_nan(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {  // (the run's only writer of part: SolveArgs::gmax_part)
        mx = absmax_nan(absmax_nan(red[0], red[1]), absmax_nan(red[2], red[3]));
        part[blockIdx.x] = mx;
    }
    if (blockIdx.x == 0)
        for (int i = gridDim.x + threadIdx.x; i < kAbsmaxMaxBlocks; i += blockDim.x) part[i] = 0.0;
}

template <typename T>
hipError_t launch_absmax(const T* g, long long count, double* part, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(absmax_kernel<T>, dim3(absmax_blocks(count)), dim3(256), 0, s, g, count, part);
    return hipGetLastError();
}
template hipError_t launch_absmax<float>(const float*, long long, double*, hipStream_t);
template hipError_t launch_absmax<double>(const double*, long long, double*, hipStream_t);

}  // namespace gpad
