// Wave placement probe: where do the waves of 13-wave workgroups land (CU, SIMD), and do two
// such workgroups share a CU, at a given VGPR allocation?  Each wave spins ~200 us so that all
// resident workgroups overlap, then records HW_ID (simd/cu/se) and XCC_ID.
// build: hipcc --offload-arch=gfx950 -O3 -o placement placement.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

template <int V>
__global__ __launch_bounds__(832) void probe(unsigned* out, long long spin) {
    // force the allocation to V VGPRs (next_free_vgpr = V)
    if constexpr (V == 64) asm volatile("v_mov_b32 v63, 0" ::: "v63");
    if constexpr (V == 72) asm volatile("v_mov_b32 v71, 0" ::: "v71");
    if constexpr (V == 80) asm volatile("v_mov_b32 v79, 0" ::: "v79");
    if constexpr (V == 88) asm volatile("v_mov_b32 v87, 0" ::: "v87");
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long rt;
    asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(rt));
    long long t0 = clock64();
    while (clock64() - t0 < spin) {}
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 13 + (threadIdx.x >> 6);
        out[3 * w] = hw;
        out[3 * w + 1] = xcc;
        out[3 * w + 2] = (unsigned)rt;
        // start timestamp (low bits) to tell rounds apart
    }
}

template <int V>
void run(int grid) {
    unsigned* d;
    hipMalloc(&d, sizeof(unsigned) * 3 * 13 * grid);
    hipLaunchKernelGGL(probe<V>, dim3(grid), dim3(832), 0, 0, d, 400000LL);
    hipDeviceSynchronize();
    std::vector<unsigned> h(3 * 13 * grid);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    // per workgroup: (xcc, se, sh, cu) key and simd histogram
    std::map<unsigned long long, std::vector<int>> cu_wgs;
    int simd_hist_first[4] = {0, 0, 0, 0};
    int pattern[5][5][5][5] = {};
    std::map<std::vector<int>, int> patt;
    for (int b = 0; b < grid; ++b) {
        int sc[4] = {0, 0, 0, 0};
        unsigned long long key = 0;
        for (int w = 0; w < 13; ++w) {
            unsigned hw = h[3 * (b * 13 + w)], xcc = h[3 * (b * 13 + w) + 1];
            int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            sc[simd]++;
            key = ((unsigned long long)(xcc & 15) << 16) | (se << 8) | (sh << 4) | cu;
            if (w == 0) simd_hist_first[simd]++;
        }
        cu_wgs[key].push_back(b);
        patt[std::vector<int>(sc, sc + 4)]++;
    }
    (void)pattern;
    int shared = 0, concurrent = 0;
    for (auto& kv : cu_wgs) {
        shared += kv.second.size() > 1;
        if (kv.second.size() > 1) {
            unsigned t0 = h[3 * (kv.second[0] * 13) + 2], t1 = h[3 * (kv.second[1] * 13) + 2];
            int dt = (int)(t1 - t0);
            if (dt < 0) dt = -dt;
            concurrent += dt < 5000;  // 100 MHz ticks: < 50 us apart = overlapping (spin ~170 us)
        }
    }
    printf("[concurrent pairs %d] ", concurrent);
    printf("V=%d grid=%d: distinct CUs %zu, CUs hosting >1 WG %d; per-WG simd patterns:", V, grid,
           cu_wgs.size(), shared);
    for (auto& kv : patt) printf(" [%d %d %d %d]x%d", kv.first[0], kv.first[1], kv.first[2], kv.first[3], kv.second);
    printf("; wave0 simd hist %d %d %d %d\n", simd_hist_first[0], simd_hist_first[1], simd_hist_first[2],
           simd_hist_first[3]);
}

int main() {
    run<64>(512);
    run<72>(512);
    run<80>(512);
    run<88>(512);
    run<64>(256);
    return 0;
}
