// gpad_panel.hip -- shared-matrix batches on the f32 MFMA pipe (gfx950).
//
// When every instance of a batch shares ML and G (one plant, many states: the battery
// scenario batch), the two mat-vecs of a GPAD iteration over 16 instances are two skinny
// GEMMs:  Zhat[n x 16] = (-ML) W[m x 16]  and  Y'[m x 16] = G_L Zhat[n x 16].  One workgroup
// owns a panel of 16 instances for the whole solve (no inter-workgroup traffic at all).
// Both GEMMs are padded to T tiles of 16 rows (T = ceil(max(n, m)/16)) and the workgroup has
// T waves: wave t owns row tile t of BOTH GEMMs (one 4-register accumulator each), so every
// per-row quantity (z, y, u = G_L z, g_P, p_D) of the panel lives in registers, and W / Zhat
// are exchanged through LDS.  Many waves per SIMD hide the 40-cycle MFMA dependency and
// overlap one wave's epilogue with another wave's MFMAs.
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
// Packed operands in HBM/L2 (built once by pack_panel_kernel at setup; T x T tiles each):
//   PA1[b][t][lane][q] = -ML[16t + pi(lane&15)][16b + 4q + (lane>>4)]   (b < TM, t < TN)
//   PA2[b][t][lane][q] = G_L[16t + pi(lane&15)][16b + 4q + (lane>>4)]   (b < TN, t < TM)
// one float4 per lane per (block, tile): 1 KiB per wave-instruction, fully coalesced.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>

#include "gpad_internal.h"

namespace gpad {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int pi16(int rho) { return 4 * (rho & 3) + (rho >> 2); }

// ---------------------------------------------------------------------------------------
// packing
// ---------------------------------------------------------------------------------------
constexpr int kPanelMaxTiles = 16;  // n, m <= 256 (1024-thread workgroups)

static int panel_tiles_for(int n, int m) {
    const int t = ((n > m ? n : m) + 15) / 16;
    return t <= kPanelMaxTiles ? t : 0;
}

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

size_t panel_frag_bytes(int n, int m, int /*batch*/) {
    const int T = panel_tiles_for(n, m);
    return T ? (size_t)2 * T * T * 64 * sizeof(float4) : 0;
}

int panel_tiles(int n, int m, int /*batch*/) { return panel_tiles_for(n, m); }

hipError_t launch_pack_panel(const float* ML, const float* G, int n, int m, int /*batch*/,
                             float mg_sign, double g_scale, void* frag, hipStream_t s) {
    const int T = panel_tiles_for(n, m);
    if (!T) return hipSuccess;
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
// the panel kernel: workgroup = panel of 16 instances, wave t = row tile t
// ---------------------------------------------------------------------------------------
struct PanelSlot {  // per wave (row tile), per instance partials of the Algorithm-1 test
    float violz[16], violh[16], wmin[16];
    double gap[16];
};

// acc = A[tile t] (T k-blocks, streamed from L2 one block ahead) x B (LDS, fragment order).
// The MFMA k-order is ascending (block 0..T-1, step 0..3), i.e. the reference's sequential chain.
// A is read with buffer loads: one 32-bit lane offset (t*1 KiB + lane*16 B) in a VGPR and the
// k-block offset as a compile-time scalar, so the unrolled blocks cost no address registers.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 as_float4(u32x4 v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                       __uint_as_float(v.w));
}

template <int T>
__device__ __forceinline__ f32x4 panel_gemm(__amdgpu_buffer_rsrc_t PA, const float* Bl, int voff,
                                            int lane) {
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    float4 a[2], b[2];
    a[0] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, 0, 0));
    b[0] = *reinterpret_cast<const float4*>(Bl + lane * 4);
#pragma unroll
    for (int kb = 0; kb < T; ++kb) {
        const int cur = kb & 1, nxt = cur ^ 1;
        if (kb + 1 < T) {
            a[nxt] = as_float4(__builtin_amdgcn_raw_buffer_load_b128(PA, voff, (kb + 1) * T * 1024, 0));
            b[nxt] = *reinterpret_cast<const float4*>(Bl + ((kb + 1) * 64 + lane) * 4);
        }
        // the next block's loads issue BEFORE this block's MFMAs (else the scheduler sinks them
        // below and waits on them at once: a full L2 round trip per k-block)
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].x, b[cur].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].y, b[cur].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].z, b[cur].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cur].w, b[cur].w, acc, 0, 0, 0);
        asm volatile("" ::: "memory");  // keep the prefetch one k-block deep
    }
    return acc;
}

// Continuous batching: a workgroup keeps 16 instance "columns" in flight.  A column that
// converges (or reaches N) writes its z*, y* and counts, then pulls the next instance from a
// device-wide queue, so no column and no CU idles while instances remain.  Every column has its
// own iteration counter (theta/beta are per lane); columns are independent in the MFMA, so the
// arithmetic of an instance does not depend on which column or workgroup runs it.
template <int T, bool QUEUE>
__global__ __launch_bounds__(64 * T) void gpad_panel_kernel(SolveArgs<float> a) {
    __shared__ __attribute__((aligned(16))) float Wl[T * 256];  // [T][64][4] w    (B of GEMM 1)
    __shared__ __attribute__((aligned(16))) float Zh[T * 256];  // [T][64][4] zhat (B of GEMM 2)
    __shared__ PanelSlot slots[T];
    __shared__ int next_inst[16];  // refill hand-out per column (-1: none)
    __shared__ int queue_dry;

    const int lane = threadIdx.x & 63;
    const int t = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // row tile of this wave
    const int j = lane >> 4, c = lane & 15;
    const int n = a.n, m = a.m, N = a.N;
    const int abytes = T * T * 1024;  // one packed operand
    const __amdgpu_buffer_rsrc_t PA1 =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.frag), 0, abytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t PA2 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)a.frag + abytes), 0, abytes, 0x00020000);
    const int voff = t * 1024 + lane * 16;
    const int slot = t * 64 + lane;  // this lane's float4 in Wl / Zh
    float4* Wl4 = reinterpret_cast<float4*>(Wl);
    float4* Zh4 = reinterpret_cast<float4*>(Zh);
    const bool use_tol = a.tol > 0.0;
    const int first = gridDim.x * 16;  // instances handed out statically; the queue serves the rest

    // register r <-> row 16t + 4r + j of the lane's current instance (column c)
    float z[4], gp[4], y[4], pd[4], u[4], zh[4];
    int inst = blockIdx.x * 16 + c;
    bool active = inst < a.batch;
    int lc = 0;  // iterations done by this column's instance

    auto load_instance = [&](bool on) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * t + 4 * r + j;
            const bool okn = on && i < n, okm = on && i < m;
            z[r] = okn ? a.z[(size_t)inst * n + i] : 0.0f;
            gp[r] = okn ? a.gP[(size_t)inst * a.ld_gP + i] : 0.0f;
            y[r] = okm ? a.y[(size_t)inst * m + i] : 0.0f;
            pd[r] = okm ? (float)(a.gscale * (double)a.g[(size_t)inst * a.ld_g + i]) : 0.0f;
            u[r] = 0.0f;
        }
        const float b0 = a.beta[0];
        Wl4[slot] = make_float4(__builtin_fmaf(b0, y[0] - y[0], y[0]), __builtin_fmaf(b0, y[1] - y[1], y[1]),
                                __builtin_fmaf(b0, y[2] - y[2], y[2]), __builtin_fmaf(b0, y[3] - y[3], y[3]));
    };
    // u = G_L z_{-1} for the columns in `fresh` (one GEMM for all of them; then the 8c recursion)
    auto seed_u = [&](bool fresh) {
        Zh4[slot] = make_float4(z[0], z[1], z[2], z[3]);
        __syncthreads();
        const f32x4 cz = panel_gemm<T>(PA2, Zh, voff, lane);
        if (fresh) {
#pragma unroll
            for (int r = 0; r < 4; ++r) u[r] = cz[r];
        }
        __syncthreads();
    };

    load_instance(active);
    if (c == 0 && t == 0 && j == 0) queue_dry = first >= a.batch;
    if (use_tol) seed_u(active);
    __syncthreads();

    float th = a.theta[0], bn = a.beta[1];
    int v = 0;  // iterations of this launch (= lc of every active column when there is no queue)
    while (true) {
        // schedule, prefetched one iteration ahead (tables hold N + 2 entries): per column with a
        // queue (columns restart at different times), uniform scalar loads without one
        float th_next, bn_next;
        if constexpr (QUEUE) {
            const int lp = active ? lc : 0;
            th_next = a.theta[lp + 1];
            bn_next = a.beta[lp + 2];
        } else {
            th_next = a.theta[v + 1];
            bn_next = a.beta[v + 2];
        }
        ++v;
        const bool chk = use_tol && active && ((lc + 1) % a.check_every) == 0;
        const float omt = 1.0f - th;
        // ---- GEMM 1 + epilogue: zhat = -ML w - g_P (8b), z = (1-th) z + th zhat (8c) -----
        {
            const f32x4 acc = panel_gemm<T>(PA1, Wl, voff, lane);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                zh[r] = acc[r] - gp[r];
                const float zn = __builtin_fmaf(omt, z[r], th * zh[r]);
                if (active) z[r] = zn;
            }
            Zh4[slot] = make_float4(zh[0], zh[1], zh[2], zh[3]);
        }
        __syncthreads();
        // ---- GEMM 2 + epilogue: y+ = [w + G_L zhat + p_D]+ (8d), next w (8a) --------------
        float violz = -INFINITY, violh = -INFINITY, wmin = INFINITY;
        double gap = 0.0;
        {
            const f32x4 acc = panel_gemm<T>(PA2, Zh, voff, lane);
            const float4 w4 = Wl4[slot];
            const float wv[4] = {w4.x, w4.y, w4.z, w4.w};
            float wn[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float cv = acc[r];
                const float sv = (wv[r] + pd[r]) + cv;
                const float yp = (__builtin_fabsf(sv) + sv) * 0.5f;
                wn[r] = __builtin_fmaf(bn, yp - y[r], yp);
                if (use_tol) {
                    const float un = __builtin_fmaf(omt, u[r], th * cv);
                    if (active) u[r] = un;
                    if (chk && (16 * t + 4 * r + j) < m) {
                        const float tt = cv + pd[r];
                        violh = fmaxf(violh, tt);
                        wmin = fminf(wmin, wv[r]);
                        gap -= (double)wv[r] * (double)tt;
                        violz = fmaxf(violz, u[r] + pd[r]);
                    }
                }
                if (active) y[r] = yp;
            }
            if (active) Wl4[slot] = make_float4(wn[0], wn[1], wn[2], wn[3]);
        }
        if (active) ++lc;
        th = th_next;
        bn = bn_next;
        // Events (a test, or a column at N).  Without a queue every active column has done v
        // iterations, so events are uniform and a plain barrier suffices; with a queue the one
        // barrier per iteration doubles as the event probe (__syncthreads_or: LDS + barriers).
        bool any_chk;
        if constexpr (QUEUE) {
            const bool at_n = active && lc >= N;
            if (!__syncthreads_or((chk || at_n) ? 1 : 0)) continue;
            any_chk = __syncthreads_or(chk ? 1 : 0);
        } else {
            __syncthreads();
            any_chk = use_tol && (v % a.check_every) == 0;
            if (!any_chk && v < N) continue;
        }

        // ---- Algorithm 1 test, per column: lane groups j, then row tiles through LDS ------
        int code = 0;
        if (any_chk) {
#pragma unroll
            for (int o = 16; o < 64; o <<= 1) {
                violz = fmaxf(violz, __shfl_xor(violz, o, 64));
                violh = fmaxf(violh, __shfl_xor(violh, o, 64));
                wmin = fminf(wmin, __shfl_xor(wmin, o, 64));
                gap += __shfl_xor(gap, o, 64);
            }
            if (j == 0) {
                slots[t].violz[c] = violz;
                slots[t].violh[c] = violh;
                slots[t].wmin[c] = wmin;
                slots[t].gap[c] = gap;
            }
            __syncthreads();
            if (chk) {
                double vz = -INFINITY, vh = -INFINITY, wm = INFINITY, gq = 0.0;
#pragma unroll
                for (int s2 = 0; s2 < T; ++s2) {
                    vz = fmax(vz, (double)slots[s2].violz[c]);
                    vh = fmax(vh, (double)slots[s2].violh[c]);
                    wm = fmin(wm, (double)slots[s2].wmin[c]);
                    gq += slots[s2].gap[c];
                }
                if (vz * a.L <= a.tol) code = 1;
                else if ((vh * a.L <= a.tol) && (wm >= 0.0) && (gq * a.L <= a.tol)) code = 2;
            }
        }
        // ---- finished columns: results out -------------------------------------------------
        const bool fin = active && (code != 0 || lc >= N);
        if (fin) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * t + 4 * r + j;
                if (i < n) a.z[(size_t)inst * n + i] = code == 2 ? zh[r] : z[r];  // (B) certifies zhat
                if (i < m) a.y[(size_t)inst * m + i] = y[r];
            }
            if (t == 0 && j == 0) {
                a.iters[inst] = lc;
                a.conv[inst] = code;
            }
            active = false;
        }
        if constexpr (!QUEUE) {
            if (v >= N || !__syncthreads_or(active ? 1 : 0)) break;
            continue;
        }
        // ---- refill idle columns from the queue (one lane per column draws) -----------------
        if (t == 0 && j == 0) {  // -2: did not draw, -1: drew from an empty queue
            int nx = -2;
            if (!active && !queue_dry) {
                const int k = atomicAdd(a.queue, 1);
                nx = first + k < a.batch ? first + k : -1;
            }
            next_inst[c] = nx;
        }
        __syncthreads();
        if (t == 0 && lane == 0) {  // all draws of this round are done: record exhaustion
            bool dry = queue_dry;
            for (int q = 0; q < 16; ++q) dry = dry || next_inst[q] == -1;
            queue_dry = dry;  // read only after the next barrier
        }
        const int nx = next_inst[c];
        const bool fresh = !active && nx >= 0;
        if (fresh) {
            inst = nx;
            active = true;
            lc = 0;
            load_instance(true);
        }
        if (__syncthreads_or(fresh ? 1 : 0)) {
            if (use_tol) seed_u(fresh);
            if (fresh) {
                th = a.theta[0];
                bn = a.beta[1];
            }
        }
        if (!__syncthreads_or(active ? 1 : 0)) break;
    }
}

template <int T>
static hipError_t launch_panel_t(const SolveArgs<float>& a, hipStream_t s) {
    // Persistent grid = as many panels as can be resident (32 waves per CU): per-iteration
    // throughput is highest with two 13-wave panels per CU, and with only ~2 instances per column
    // a smaller grid loses more to the end-of-queue tail than it gains from refills (measured on
    // C4).  Larger batches keep every resident column busy through the queue.
    const int panels = (a.batch + 15) / 16;
    const int resident = a.num_cus * (32 / T > 0 ? 32 / T : 1);
    int grid = panels < resident ? panels : resident;
    if (const char* cap = std::getenv("GPAD_PANEL_MAX_GRID")) {  // test knob: force refills
        const int c = std::atoi(cap);
        if (c > 0 && c < grid) grid = c;
    }
    if (grid < panels)
        hipLaunchKernelGGL((gpad_panel_kernel<T, true>), dim3(grid), dim3(64 * T), 0, s, a);
    else
        hipLaunchKernelGGL((gpad_panel_kernel<T, false>), dim3(grid), dim3(64 * T), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_panel(const SolveArgs<float>& a, hipStream_t s, bool* supported) {
    const int T = panel_tiles_for(a.n, a.m);
    // the fragment image must have been packed for this geometry at setup
    *supported = a.frag != nullptr && T && a.strideA == 0 && a.strideB == 0 && a.frag_tiles == T;
    if (!*supported) return hipSuccess;
    switch (T) {
        case 1: return launch_panel_t<1>(a, s);
        case 2: return launch_panel_t<2>(a, s);
        case 3: return launch_panel_t<3>(a, s);
        case 4: return launch_panel_t<4>(a, s);
        case 5: return launch_panel_t<5>(a, s);
        case 6: return launch_panel_t<6>(a, s);
        case 7: return launch_panel_t<7>(a, s);
        case 8: return launch_panel_t<8>(a, s);
        case 9: return launch_panel_t<9>(a, s);
        case 10: return launch_panel_t<10>(a, s);
        case 11: return launch_panel_t<11>(a, s);
        case 12: return launch_panel_t<12>(a, s);
        case 13: return launch_panel_t<13>(a, s);
        case 14: return launch_panel_t<14>(a, s);
        case 15: return launch_panel_t<15>(a, s);
        default: return launch_panel_t<16>(a, s);
    }
}

}  // namespace gpad
