// gpad_internal.h -- device-side argument blocks and kernel launchers shared by the
// HIP kernels (gpad_kernels.hip, gpad_panel.hip) and the host runtime (gpad_host.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace gpad {

// gpad_last_error() detail for the calling thread; returns code (gpad_host.cpp)
int set_last_error(int code, const std::string& msg);

// Schedule / launch tuning of a handle (gpad_set_option, include/gpad.h GPAD_OPT_*): for tests,
// diagnostics and A/B tools.  None of these changes results -- only launch boundaries, grid
// sizes, work-queue order and where operands are staged.
struct Tuning {
    int phase_len = 0;        // GPAD_OPT_PHASE_LEN: panel phase length, iterations (0: 4 tests)
    int finish_thresh = -1;   // GPAD_OPT_FINISH_THRESH: finisher takeover (-1: 2 per CU)
    int plan = 1;             // GPAD_OPT_PLAN: phase plan from the previous solve
    int phased = 1;           // GPAD_OPT_PHASED: phased compaction of tol > 0 panel solves
    int lpt = 1;              // GPAD_OPT_LPT: longest-predicted-first finisher queue
    int panel_max_grid = 0;   // GPAD_OPT_PANEL_MAX_GRID: cap on the panel grid (0: none)
    int duo_max_grid = 0;     // GPAD_OPT_DUO_MAX_GRID: cap on the finisher grid (0: none)
    int flat_panel_min = -1;  // GPAD_OPT_FLAT_PANEL_MIN: batch from which flat setups use panels
    int flat_panels = 0;      // GPAD_OPT_FLAT_PANELS: panels per flat-panel workgroup (0: auto)
    int flat_waves = 0;       // GPAD_OPT_FLAT_WAVES: 0 auto, 8 or 16 waves per workgroup
    int flat_a_lds = 1;       // GPAD_OPT_FLAT_A_LDS: flat fragment image in LDS when it fits
    int debug_drop_handoff = 0;  // GPAD_OPT_DEBUG_DROP_HANDOFF: test-only fault injection
    int p64_no_relay = 0;     // GPAD_OPT_P64_RELAY = 0: f64 panels without the relay layout
    int p64_no_refill = 0;    // GPAD_OPT_P64_REFILL = 0: f64 panels without column refills
};

// Device error word of a run (SolveArgs::err): kernels OR these bits in with a vector atomic;
// the host turns a non-zero word into GPAD_ERR_DEVICE when it collects or syncs the run.
constexpr int kDevErrHandoff = 1;  // a chain hand-off wait expired (gpad_panel.hip handoff_wait)
// SolveArgs::debug bits (fault injection for tests; 0 in production)
constexpr int kDebugDropHandoff = 1;  // the first hand-off helper skips its first post

// Rounding margin of the Algorithm 1 decisions, in units of max_i(|chain_i| + |pD_i|): a test
// passes when L max(chain + pD) + kViolMargin L max(|chain| + |pD|) <= tol (16 units of 2^-24 /
// 2^-53).  Test (A) is nominated by the recursive u = G_L z and decided on the direct chain
// G_L z (which then also resets u).  Same constants and arithmetic as oracle/gpad_oracle.h.
template <typename T> struct ViolMargin;
template <> struct ViolMargin<float> { static constexpr double value = 0x1p-20; };
template <> struct ViolMargin<double> { static constexpr double value = 0x1p-49; };
// max(acc, |x|) for acc >= 0 that keeps a NaN: as unsigned bit patterns the magnitudes order
// finite < inf < NaN, so a NaN in g reaches the certification floor's max |g| (and the stats flag
// it, GPAD_FLAG_NONFINITE_G) where fmax would drop it
__device__ __forceinline__ float absmax_nan(float acc, float x) {
    const unsigned a = __float_as_uint(acc), b = __float_as_uint(x) & 0x7fffffffu;
    return __uint_as_float(a > b ? a : b);
}
__device__ __forceinline__ double absmax_nan(double acc, double x) {
    const unsigned long long a = (unsigned long long)__double_as_longlong(acc),
                             b = (unsigned long long)__double_as_longlong(x) & 0x7fffffffffffffffull;
    return __longlong_as_double((long long)(a > b ? a : b));
}
// the decision itself, one expression everywhere (no contraction: -ffp-contract=off)
__host__ __device__ inline bool viol_ok(double viol, double mag, double L, double tol, double margin) {
    return viol * L + margin * mag * L <= tol;
}

// Arguments of a fused solve launch (all kernel families).  Every instance b of the batch
// reads its matrices at MGt + b*strideA / GLt + b*strideB (stride 0 = shared).
template <typename T>
struct SolveArgs {
    const T* MGt;          // -ML, k-major: [m][ldn]   (column k of -ML is contiguous)
    const T* GLt;          // G/L, k-major: [n][ldm]
    long long strideA;     // elements between consecutive instances' -ML images (0 = shared)
    long long strideB;     // elements between consecutive instances' G/L images (0 = shared)
    const void* frag;      // panel kernel: fragment-packed matrices (see gpad_panel.hip)
    int frag_tiles;        // tile count the fragment image was packed for
    const T* gP;           // per-instance H^-1 q, [batch][ld_gP]
    const T* g;            // per-instance rhs,    [batch][ld_g]
    long long ld_gP, ld_g;
    double gscale;         // pD = (T)(gscale * g): -1/L, or 1 when g already holds p_D
    T* z;                  // [batch][n]  in z_{-1}, out z*
    T* y;                  // [batch][m]  in y0,     out y*
    int n, m, ldn, ldm;    // ldn = round_up(n,4), ldm = round_up(m,4)
    int batch, N, check_every;
    double tol, L;         // Algorithm 1: stop when L*viol <= tol (tol <= 0: fixed N)
    double tol_gap;        // e_V of test (B)'s duality-gap term (set = tol when the caller gives <= 0)
    const T* theta;        // [N+2] theta_v (two zero pads: kernels prefetch ahead)
    const T* beta;         // [N+2] beta_v
    int* iters;            // [batch] iterations executed
    int* conv;             // [batch] 0 = not converged, 1 = test (A) passed, 2 = test (B) passed
    int num_cus;           // compute units of the device (persistent-grid sizing)
    // panel kernel, phased compaction (set by launch_panel; see gpad_panel.hip)
    void* pwork;           // workspace of panel_work_bytes(m, batch) bytes, or null (one phase)
    int v_begin, v_end;    // iterations [v_begin, v_end) of this phase
    int v_pred;            // flat panels: predicted last iteration (previous solve), 0 = unknown
    const int* idx_in;     // instances of this phase (null: 0..batch-1)
    const int* count_in;   // their number (device; null: batch)
    int* idx_out;          // survivors appended here ...
    int* count_out;        // ... and counted here (device) -- or, with seg_cnt set, listed per panel:
    int* seg_cnt;          // [panel] survivors of panel P of this phase (no same-address atomics)
    int* seg_idx;          // [16 panel + rank] their instances; phase_compact_kernel densifies
    double* gmax_part;     // [kAbsmaxMaxBlocks] per-workgroup max |g| of the run (the certification
                           // floor; null: not wanted): the panel pairs fold it into their loads,
                           // every other path runs launch_absmax.  Not zeroed before the run: its
                           // first writer (the panel pairs' launch at v_begin == 0, or absmax) stores
                           // its slots and zeroes the rest; later phase launches max into them
    int* zero_w;           // panel pairs: words workgroup 0 zeroes at the launch's start (a phased
    int zero_n;            // solve's phase and queue counters, read by later launches only), or null
    float* wc;             // carried w  [batch][m]
    float* uc;             // carried u = G_L z [batch][m]
    int fin_thresh;        // survivors <= this: the resident finisher takes them (0: none)
    int* qctr;             // duo kernel: zeroed device counter of its work-list claims
    const int* pred;       // phased solves: per-instance iteration counts predicted from the
                           // previous solve (or null); orders the finisher's queue longest first
    int n_u;               // flat battery path: cells (n = n_u * horizon), see gpad_flat.hip
    int flat_staged;       // flat path: matrices staged in LDS (set by launch_flat)
    const int* order;      // f64 panels with column refills: instances in start order (the previous
                           // solve's counts, longest first: LPT over the columns), or null (0..batch-1)
    const struct PanelPlan* plan;  // panel phases: host-side plan from the previous solve (or null)
    struct PanelPlan* used;        // panel phases: host-side record of the phases launched (or null)
    const Tuning* tune;    // host-side tuning options (never null on a launch from gpad_host.cpp)
    const T* Hq;           // QP Hessian H, k-major [n][ldn] (gpad_setup_hessian), or null: enables the
                           // value-function branches of the test (stream kernel only)
    long long strideHq;    // elements between consecutive instances' H images (0 = shared)
    const void* hfrag64;   // f64 panels (gpad_panel64.hip): H in their fragment layout, or null (no value
                           // branches)
    int* err;              // device error word (kDevErr* bits), never null on a solve launch
    int debug;             // kDebug* fault-injection bits (tests only)
};

// launchers (return hipError_t of the launch)
template <typename T>
hipError_t launch_stream(const SolveArgs<T>& a, hipStream_t s);
hipError_t launch_resident(const SolveArgs<float>& a, hipStream_t s, bool* supported);
// two-instance ping-pong kernel over a work list (shared matrices; gpad_kernels.hip): the
// list is idx_in/count_in (a no-op unless *count_in <= a.fin_thresh) or 0..batch-1; needs a
// zeroed a.qctr.  Persistent grid of `grid` workgroups (one per CU).
hipError_t launch_duo(const SolveArgs<float>& a, int grid, hipStream_t s);
bool resident_supported(int n, int m);
hipError_t launch_panel(const SolveArgs<float>& a, hipStream_t s, bool* supported);
// f64 panels on the f64 MFMA pipe (gpad_panel64.hip): shared matrices, n, m <= 256, one panel of 16
// instances per workgroup, value-function branches when a.hfrag64 is set; a.frag = the -ML | G_L
// images of launch_pack_panel64, a.frag_tiles = panel64_tiles(n, m)
bool panel64_supported(int n, int m);
int panel64_tiles(int n, int m);
size_t panel64_frag_bytes(int n, int m);  // one T x T operand image
hipError_t launch_pack_panel64(const double* src, int rows, int cols, double scale, int T, void* dst, hipStream_t s);
hipError_t launch_panel64(const SolveArgs<double>& a, hipStream_t s);
// launch_panel at (n, m) runs the panel pairs, which fold max |g| into their loads (gmax_part)
bool panel_folds_gmax(int n, int m);

// Phase end of a panel kernel: list panel P's parked columns.  Called by the wave that speaks for
// the panel, whose lanes 0..15 (j == 0) hold columns 0..15; `park`: this lane's column carries
// over.  With a.seg_cnt the panel writes its own slot -- seg_cnt[P], seg_idx[16 P + rank] -- and
// phase_compact_kernel densifies the list at the boundary: no same-address atomics (hundreds of
// panels appending to one counter serialise at L2, ~25 us per boundary at 512 panels measured).
// Without it (flat panels) the survivors are appended through a.count_out.  Every
// panel of a phase calls it, parked or not, so no slot keeps a stale count.
// A kernel's SolveArgs read afresh from its kernarg segment -- only in kernels whose one argument is
// a SolveArgs<float> (gpad_panel2_kernel, gpad_duo_kernel).  The pointer passes an empty asm, so the
// fields loaded through it at a rare site (refills, results out, park, survivor lists, a panel's
// state loads) are not kept live in SGPRs across the solve loop: loaded once at the top, the dozen
// row-array pointers spilled to VGPR lanes and were reloaded (v_readlane) around every step.
typedef const __attribute__((address_space(4))) SolveArgs<float> KernArgs;
__device__ __forceinline__ KernArgs& kargs() {
    KernArgs* p = (KernArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *p;
}

template <class Args>
__device__ __forceinline__ void list_survivors(const Args& a, int P, bool park, int inst, int lane,
                                               int j) {
    const unsigned long long lv = __ballot(park && j == 0);
    const int rank = (int)__popcll(lv & ((1ull << lane) - 1ull));
    if (a.seg_cnt) {
        if (lane == 0) a.seg_cnt[P] = (int)__popcll(lv);
        if (park && j == 0) a.seg_idx[16 * P + rank] = inst;
    } else {
        int base = 0;
        if (lane == 0 && lv) base = atomicAdd(a.count_out, (int)__popcll(lv));
        base = __shfl(base, 0, 64);
        if (park && j == 0) a.idx_out[base + rank] = inst;
    }
}
// the boundary before phase ph >= 1: the survivors phase ph - 1 listed per panel (seg_cnt / seg_idx)
// -> idx_out[0 .. *count_out), optionally ordered longest-predicted-first (pred: the previous
// solve's counts, when the list is the finisher's: count <= fin_cur).  count_prev / fin_prev:
// phase ph - 1's own input count and finisher threshold (count_prev <= fin_prev: the finisher
// took that list and the panel phase listed nothing).
hipError_t launch_phase_compact(const int* seg_cnt, const int* seg_idx, const int* count_prev, int batch,
                                int fin_prev, int* idx_out, int* count_out, const int* pred, int fin_cur,
                                hipStream_t s);
size_t panel_frag_bytes(int n, int m, int batch);
size_t panel_work_bytes(int m, int batch);
int panel_phase_len(int check_every, const Tuning* t);
int panel_fin_thresh(int n, int m, int num_cus, const Tuning* t);
// phase plan of a phased panel solve, from the previous solve's iteration counts (panel_plan)
constexpr int kPanelMaxPhases = 48;
struct PanelPlan {
    int nph = 0;                  // phases planned (0: the default schedule)
    int N = 0;                    // iteration limit the plan was made for
    int ends[kPanelMaxPhases];    // phase ph covers [ends[ph-1], ends[ph]); the last ends at N
    int fins[kPanelMaxPhases];    // finisher threshold at the start of phase ph (ph >= 1)
    double cost_us = 0.0;         // modelled solve time
};
int panel_plan(const int* iters, int batch, int n, int m, int N, int check_every, int num_cus, const Tuning* t,
               PanelPlan* out);
int panel_tiles(int n, int m, int batch);
// gpad_bigpanel.hip: shared f32 matrices with n or m in (256, 1024]
bool bigpanel_supported(int n, int m);
size_t bigpanel_frag_bytes(int n, int m);
hipError_t launch_pack_bigpanel(const float* ML, const float* G, int n, int m, float mg_sign, double g_scale,
                                void* frag, hipStream_t s);
hipError_t launch_bigpanel(const SolveArgs<float>& a, int grid, hipStream_t s);
hipError_t launch_pack_panel(const float* ML, const float* G, int n, int m, int batch, float mg_sign,
                             double g_scale, void* frag, hipStream_t s);

// layout: out[k*ld + i] = (T)(scale * in[i*cols + k]) for i < rows, k < cols; zero pad i >= rows
template <typename T>
hipError_t launch_pack_kmajor(const T* in, T* out, int rows, int cols, int ld, double scale,
                              int batch, long long in_stride, long long out_stride, hipStream_t s);

// gpad_plant.hip: out1 = c1 + P1 x (rows1), out2 = c2 + P2 x (rows2) per instance; c may be null
template <typename T>
hipError_t launch_affine2(const T* P1, const T* c1, int rows1, T* out1, const T* P2, const T* c2,
                          int rows2, T* out2, const T* x, int nx, int batch, hipStream_t s);
// xn = A x + B z[:, 0:nu]; xs/us (nullable) receive x and z[:, 0:nu]
template <typename T>
hipError_t launch_plant_step(const T* A, const T* B, const T* x, const T* z, long long ldz, T* xn, int nx,
                             int nu, int batch, T* xs, T* us, hipStream_t s);

// gpad_flat.hip (flat battery path; MGt = flat -ML [Nh][m], GLt = flat G_L t-major [Nh][m])
hipError_t launch_flat(const SolveArgs<float>& a, hipStream_t s);
// register-resident flat variant (gpad_kernels.hip): a.MGt = flat -ML (Nh x m), a.GLt = the
// flat G_L expanded to the full k-major image [n][ldm]
bool flat_resident_supported(int n, int m, int n_u);
hipError_t launch_flat_resident(const SolveArgs<float>& a, hipStream_t s);
// one-time QP precompute (gpad_precompute.hip): Gauss-Jordan on [H | A' | f'] per instance
size_t precompute_work_bytes(int n, int m, int nf, int count);
bool precompute_supported(int n, int m, int nf);
hipError_t launch_precompute(int n, int m, int nf, const double* H, long long sH, const double* A, long long sA,
                             const double* f, long long sF, double* work, double* ML, double* gP, double* L, int b0,
                             int count, hipStream_t s);
hipError_t launch_apply_inv(int n, int batch, const double* Hinv, const double* f, double* gP, hipStream_t s);
hipError_t launch_accumulate_iters(const int* iters, long long count, long long* acc, hipStream_t s);
// part[b] = max |g_i| over workgroup b's share, b < absmax_blocks(count), the remaining slots zeroed:
// per-workgroup maxima, no atomics (the host reduces them when it reads the stats)
constexpr int kAbsmaxMaxBlocks = 1024;
// gpad_release_cached: this thread's gpad_solve_sharded group (gpad_group.cpp)
void release_sharded_cache();
inline int absmax_blocks(long long count) {
    const long long b = (count + 4095) / 4096;
    return b < 1 ? 1 : (b > kAbsmaxMaxBlocks ? kAbsmaxMaxBlocks : (int)b);
}
template <typename T>
hipError_t launch_absmax(const T* g, long long count, double* part, hipStream_t s);
// flat battery data on the MFMA pipe (gpad_flatpanel.hip): per-cell skinny GEMMs over panels
bool flatpanel_supported(int n, int m, int n_u);
size_t flatpanel_frag_bytes(int n, int m, int n_u);
hipError_t launch_pack_flatpanel(const float* MGf, const float* GLT, int n, int m, int n_u, void* frag,
                                 hipStream_t s);
// tol > 0 with a.pwork (panel_work_bytes): phased compaction, phases of flat_phase_len iterations
hipError_t launch_flatpanel(const SolveArgs<float>& a, hipStream_t s);
int flat_phase_len(int v0, int check_every, const Tuning* t);
// flat G_L (m x Nh) -> full k-major image out[k*ld + r] (k < n), zero off the structure
hipError_t launch_expand_flat_gl(const float* GLf, float* out, int Nh, int n_u, int m, int ld, hipStream_t s);
hipError_t launch_step2_flat(const float* MGf, const float* w, const float* gP, float* zhat, int Nh, int n_u,
                             int m, hipStream_t s);
hipError_t launch_step4_flat(const float* GLf, float* yp1, const float* w, const float* pD, const float* zhat,
                             int Nh, int n_u, int m, hipStream_t s);
hipError_t launch_transpose_flat(const float* in, float* out, int rows, int cols, hipStream_t s);

hipError_t launch_step1(const float* y, const float* ym1, float* w, float beta, int m, hipStream_t s);
hipError_t launch_step2(const float* MGneg, const float* w, const float* gP, float* zhat, int n,
                        int m, hipStream_t s);
hipError_t launch_step3(float theta, const float* zm1, const float* zhat, float* z, int n,
                        hipStream_t s);
hipError_t launch_step4(const float* GL, float* yp1, const float* w, const float* pD,
                        const float* zhat, int n, int m, hipStream_t s);

}  // namespace gpad
