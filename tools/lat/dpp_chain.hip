// Micro-benchmark: cost of dependent v_fmac_f32 chains with and without a DPP row_newbcast
// operand, for one or two waves per SIMD and one or two interleaved chains per wave.
// Workgroup of 4 or 8 waves (waves w and w+4 share a SIMD), one workgroup per CU on every CU.
// Prints wall time per chain step (ns) and the implied cycles at 2.4 GHz.
// Build: hipcc --offload-arch=gfx950 -O3 -o dpp_chain dpp_chain.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kSteps = 4096;  // per chain

#define FMAC_DPP "v_fmac_f32_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
#define FMAC "v_fmac_f32 %0, %1, %2\n\t"
#define X4(s) s s s s
#define X16(s) X4(s) X4(s) X4(s) X4(s)

template <bool DPP, int ILP, int LANES = 64>
__global__ void chain(float* out, float a, int nwaves_active) {
    const int w = threadIdx.x >> 6;
    if (LANES < 64 && (threadIdx.x & 63) >= LANES) {  // partial EXEC: only LANES lanes run the chain
        out[blockIdx.x * blockDim.x + threadIdx.x] = 0.0f;
        return;
    }
    float acc0 = threadIdx.x * 1e-3f, acc1 = threadIdx.x * 2e-3f;
    const float src = a * (threadIdx.x & 15), r = 0.999f;
    if (w < nwaves_active) {
        for (int i = 0; i < kSteps / 16; ++i) {
            if constexpr (ILP == 1) {
                if constexpr (DPP) asm volatile(X16(FMAC_DPP) : "+v"(acc0) : "v"(src), "v"(r));
                else asm volatile(X16(FMAC) : "+v"(acc0) : "v"(src), "v"(r));
            } else {
                if constexpr (DPP)
                    asm volatile(X16("v_fmac_f32_dpp %0, %2, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                                     "v_fmac_f32_dpp %1, %2, %3 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t")
                                 : "+v"(acc0), "+v"(acc1) : "v"(src), "v"(r));
                else
                    asm volatile(X16("v_fmac_f32 %0, %2, %3\n\tv_fmac_f32 %1, %2, %3\n\t")
                                 : "+v"(acc0), "+v"(acc1) : "v"(src), "v"(r));
            }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc0 + acc1;
}

// LDS-broadcast chain: every lane reads the same float4 (ds_read_b128, same address), 4 plain
// v_fmac_f32 per read; ring of R float4 prefetched ahead.  MODE 0: all active waves LDS-broadcast;
// MODE 1: waves 0-3 DPP chain, waves 4-7 LDS-broadcast chain (mixed on every SIMD);
// MODE 2: waves 0-3 DPP, waves 4-7 plain (register operand) chain.
template <int MODE, int R = 4>
__global__ void lds_chain(float* out, float a, int nwaves_active) {
    __shared__ __attribute__((aligned(16))) float v[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) v[i] = a * (i & 7) * 1e-3f;
    __syncthreads();
    const int w = threadIdx.x >> 6;
    float acc = threadIdx.x * 1e-3f;
    const float r = 0.999f, src = a * (threadIdx.x & 15);
    const bool dppwave = MODE >= 1 && w < 4;
    if (w < nwaves_active) {
        if (dppwave) {
            for (int i = 0; i < kSteps / 16; ++i) asm volatile(X16(FMAC_DPP) : "+v"(acc) : "v"(src), "v"(r));
        } else if (MODE == 2) {
            for (int i = 0; i < kSteps / 16; ++i) asm volatile(X16(FMAC) : "+v"(acc) : "v"(src), "v"(r));
        } else {
            float4 ring[R];
#pragma unroll
            for (int q = 0; q < R; ++q) ring[q] = *reinterpret_cast<const float4*>(&v[4 * q]);
            for (int i = 0; i < kSteps / (4 * R); ++i) {
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    const float4 c = ring[q];
                    ring[q] = *reinterpret_cast<const float4*>(&v[(4 * (i * R + q + R)) & 1023]);
                    asm volatile("v_fmac_f32 %0, %1, %5\n\tv_fmac_f32 %0, %2, %5\n\t"
                                 "v_fmac_f32 %0, %3, %5\n\tv_fmac_f32 %0, %4, %5\n\t"
                                 : "+v"(acc) : "v"(c.x), "v"(c.y), "v"(c.z), "v"(c.w), "v"(r));
                }
            }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE, int R = 4>
void run_lds(const char* name, float* out, int grid, int threads, int active) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((lds_chain<MODE, R>), dim3(grid), dim3(threads), 0, 0, out, 1.0f, active);
    const int reps = 20;
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((lds_chain<MODE, R>), dim3(grid), dim3(threads), 0, 0, out, 1.0f, active);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ns_step = ms / reps * 1e6 / kSteps;
    printf("%-44s %7.3f ns/step  (%5.2f cyc @2.4GHz)  waves %d\n", name, ns_step, ns_step * 2.4, active);
}

template <bool DPP, int ILP, int LANES = 64>
void run(const char* name, float* out, int grid, int threads, int active) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((chain<DPP, ILP, LANES>), dim3(grid), dim3(threads), 0, 0, out, 1.0f, active);
    const int reps = 20;
    hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((chain<DPP, ILP, LANES>), dim3(grid), dim3(threads), 0, 0, out, 1.0f, active);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ns_step = ms / reps * 1e6 / kSteps;  // per step of ONE chain
    printf("%-44s %7.3f ns/step  (%5.2f cyc @2.4GHz)  chains/SIMD %d\n", name, ns_step, ns_step * 2.4,
           (active + 3) / 4 * ILP);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int grid = p.multiProcessorCount;
    float* out;
    hipMalloc(&out, (size_t)grid * 1024 * sizeof(float));
    run<false, 1>("plain fmac, 1 wave/SIMD", out, grid, 256, 4);
    run<false, 1>("plain fmac, 2 waves/SIMD", out, grid, 512, 8);
    run<false, 2>("plain fmac, 1 wave/SIMD, ILP2", out, grid, 256, 4);
    run<true, 1>("dpp fmac, 1 wave/SIMD", out, grid, 256, 4);
    run<true, 1>("dpp fmac, 2 waves/SIMD", out, grid, 512, 8);
    run<true, 2>("dpp fmac, 1 wave/SIMD, ILP2", out, grid, 256, 4);
    run<true, 2>("dpp fmac, 2 waves/SIMD, ILP2", out, grid, 512, 8);
    run<true, 1>("dpp fmac, 8 waves, only 4 active", out, grid, 512, 4);
    run_lds<0>("lds-bcast fmac, 1 wave/SIMD", out, grid, 256, 4);
    run_lds<0>("lds-bcast fmac, 2 waves/SIMD", out, grid, 512, 8);
    run_lds<1>("dpp (w0-3) + lds-bcast (w4-7)", out, grid, 512, 8);
    run_lds<2>("dpp (w0-3) + plain (w4-7)", out, grid, 512, 8);
    // prefetch depth: R float4 (4R steps) in flight
    run_lds<0, 8>("lds-bcast R=8, 1 wave/SIMD", out, grid, 256, 4);
    run_lds<0, 16>("lds-bcast R=16, 1 wave/SIMD", out, grid, 256, 4);
    run_lds<0, 16>("lds-bcast R=16, 2 waves/SIMD", out, grid, 512, 8);
    run_lds<0, 16>("lds-bcast R=16, 3 waves/SIMD", out, grid, 768, 12);
    run_lds<0, 16>("lds-bcast R=16, 4 waves/SIMD", out, grid, 1024, 16);
    run_lds<1, 16>("dpp (w0-3) + lds-bcast R=16 (w4-7)", out, grid, 512, 8);
    run<false, 1, 16>("plain fmac, EXEC 16 lanes, 1 wave/SIMD", out, grid, 256, 4);
    run<false, 1, 32>("plain fmac, EXEC 32 lanes, 1 wave/SIMD", out, grid, 256, 4);
    run<false, 1, 16>("plain fmac, EXEC 16 lanes, 4 waves/SIMD", out, grid, 1024, 16);
    run<true, 1, 16>("dpp fmac, EXEC 16 lanes, 1 wave/SIMD", out, grid, 256, 4);
    run<true, 1, 16>("dpp fmac, EXEC 16 lanes, 2 waves/SIMD", out, grid, 512, 8);
    run<false, 2, 16>("plain fmac, EXEC 16 lanes, ILP2", out, grid, 256, 4);
    run<false, 1>("plain fmac, 3 waves/SIMD", out, grid, 768, 12);
    run<false, 1>("plain fmac, 4 waves/SIMD", out, grid, 1024, 16);
    return 0;
}
