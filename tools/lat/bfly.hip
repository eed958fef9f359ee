// VALU butterflies (gpad_chain.h: permlane swaps + DPP) against the __shfl_xor butterfly they
// replace: bit-identical sums / maxima / minima on every lane, random data incl. NaN / inf / -0.
//   hipcc --offload-arch=gfx950 -O3 -I../../gpu-dualgradient-mpc_amd/csrc -I../../include bfly.hip -o bfly
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "gpad_chain.h"

using namespace gpad;

template <typename T>
__device__ T shfl_sum(T v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <typename T>
__device__ T shfl_max(T v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
template <typename T>
__device__ T shfl_min(T v) {
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}

__global__ void kern(const double* xd, const float* xf, double* od, float* of) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    const double d = xd[i];
    const float f = xf[i];
    od[6 * i + 0] = wave_sum(d);
    od[6 * i + 1] = shfl_sum(d);
    od[6 * i + 2] = wave_max(d);
    od[6 * i + 3] = shfl_max(d);
    od[6 * i + 4] = wave_min(d);
    od[6 * i + 5] = shfl_min(d);
    of[4 * i + 0] = wave_max(f);
    of[4 * i + 1] = shfl_max(f);
    of[4 * i + 2] = wave_min(f);
    of[4 * i + 3] = shfl_min(f);
}

int main() {
    const int W = 4096;  // waves
    std::mt19937_64 g(7);
    std::normal_distribution<double> nd(0.0, 1.0);
    std::vector<double> xd(64 * W);
    std::vector<float> xf(64 * W);
    for (int i = 0; i < 64 * W; ++i) {
        const int w = i / 64;
        double v = nd(g) * std::ldexp(1.0, (int)(g() % 60) - 30);
        if (w % 7 == 1 && g() % 5 == 0) v = NAN;
        if (w % 11 == 2 && g() % 9 == 0) v = (g() & 1) ? INFINITY : -INFINITY;
        if (w % 13 == 3 && g() % 3 == 0) v = -0.0;
        if (w % 17 == 4) v = NAN;  // whole wave NaN
        xd[i] = v;
        xf[i] = (float)v;
    }
    double *dxd, *dod;
    float *dxf, *dof;
    hipMalloc(&dxd, xd.size() * 8);
    hipMalloc(&dxf, xf.size() * 4);
    hipMalloc(&dod, xd.size() * 6 * 8);
    hipMalloc(&dof, xf.size() * 4 * 4);
    hipMemcpy(dxd, xd.data(), xd.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dxf, xf.data(), xf.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kern, dim3(W), dim3(64), 0, 0, dxd, dxf, dod, dof);
    std::vector<double> od(xd.size() * 6);
    std::vector<float> of(xf.size() * 4);
    if (hipMemcpy(od.data(), dod, od.size() * 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(of.data(), dof, of.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        printf("device error\n");
        return 2;
    }
    long bad[5] = {0, 0, 0, 0, 0};
    for (size_t i = 0; i < xd.size(); ++i) {
        for (int k = 0; k < 3; ++k) {
            const double a = od[6 * i + 2 * k], b = od[6 * i + 2 * k + 1];
            if (std::memcmp(&a, &b, 8) != 0 && !(std::isnan(a) && std::isnan(b))) ++bad[k];
        }
        for (int k = 0; k < 2; ++k) {
            const float a = of[4 * i + 2 * k], b = of[4 * i + 2 * k + 1];
            if (std::memcmp(&a, &b, 4) != 0 && !(std::isnan(a) && std::isnan(b))) ++bad[3 + k];
        }
    }
    printf("VALU butterflies vs __shfl_xor, %d waves x 64 lanes: differing lanes sum_f64 %ld max_f64 %ld min_f64 %ld "
           "max_f32 %ld min_f32 %ld\n", W, bad[0], bad[1], bad[2], bad[3], bad[4]);
    return (bad[0] | bad[1] | bad[2] | bad[3] | bad[4]) ? 1 : 0;
}
