// Micro-benchmark: dependent v_fma_f32 chain latency on gfx950 for one wave alone.
// Variants: full wave64, lanes 0-31 only (half wave), packed v_pk_fma_f32 (2 chains per lane),
// and a chain that re-reads an LDS broadcast operand every 4 FMAs.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kLen = 4096;

__global__ void chain_full(float* out, float a, long long* cyc) {
    float acc = threadIdx.x * 1e-3f;
    const float b = a * 0.5f;
    long long t0 = clock64();
#pragma unroll 64
    for (int i = 0; i < kLen; ++i) acc = __builtin_fmaf(acc, a, b);
    long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void chain_half(float* out, float a, long long* cyc) {
    float acc = threadIdx.x * 1e-3f;
    const float b = a * 0.5f;
    long long t0 = clock64();
    if (threadIdx.x < 32) {
#pragma unroll 64
        for (int i = 0; i < kLen; ++i) acc = __builtin_fmaf(acc, a, b);
    }
    long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void chain_pk(float* out, float a, long long* cyc) {
    f2 acc = {threadIdx.x * 1e-3f, threadIdx.x * 2e-3f};
    const f2 av = {a, a}, bv = {a * 0.5f, a * 0.25f};
    long long t0 = clock64();
#pragma unroll 64
    for (int i = 0; i < kLen; ++i) acc = __builtin_elementwise_fma(acc, av, bv);
    long long t1 = clock64();
    out[threadIdx.x] = acc.x + acc.y;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// two independent chains per lane (ILP 2)
__global__ void chain_ilp2(float* out, float a, long long* cyc) {
    float acc = threadIdx.x * 1e-3f, acc2 = threadIdx.x * 2e-3f;
    const float b = a * 0.5f;
    long long t0 = clock64();
#pragma unroll 64
    for (int i = 0; i < kLen; ++i) {
        acc = __builtin_fmaf(acc, a, b);
        acc2 = __builtin_fmaf(acc2, a, b);
    }
    long long t1 = clock64();
    out[threadIdx.x] = acc + acc2;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 1024 * sizeof(float));
    hipMalloc(&cyc, sizeof(long long));
    long long h;
    struct { const char* name; void (*k)(float*, float, long long*); int fmas_per_iter; } ks[] = {
        {"full wave64 dependent", chain_full, 1},
        {"lanes 0-31 only", chain_half, 1},
        {"v_pk_fma_f32 (2 chains)", chain_pk, 1},
        {"ILP 2 chains", chain_ilp2, 2},
    };
    for (auto& k : ks) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k.k, dim3(1), dim3(64), 0, 0, out, 0.999f, cyc);
            hipDeviceSynchronize();
        }
        hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("%-28s %8lld clock64 ticks for %d steps -> %.2f ticks/step\n", k.name, h, kLen,
               (double)h / kLen);
    }
    // clock64 tick vs shader clock: time a long chain with events
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(chain_full, dim3(1), dim3(64), 0, 0, out, 0.999f, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("full chain: %.3f us per launch (%d dependent fmas), %lld ticks\n", ms * 10.0, kLen, h);
    return 0;
}
