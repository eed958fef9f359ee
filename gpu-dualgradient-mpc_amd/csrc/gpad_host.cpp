// gpad_host.cpp -- host runtime behind the C-ABI of include/gpad.h.
//
// Owns, per handle: the packed device copies of the constant matrices (k-major -ML and G/L,
// and the MFMA fragment image for shared-matrix batches), the theta/beta table, per-instance
// workspaces for host-memory callers, per-instance iteration/convergence counters and the
// HIP events that time the solve launch.  Replaces the host driver of the reference
// (main.cu:79-203: file read, 9 cudaMallocs, H2D copies, 100 x (6 launches + 3 syncs), D2H).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/gpad.h"
#include "gpad_abi.h"
#include "gpad_internal.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

// "<what>: hipErrorName (code N): description" -- the name and number of the HIP status, so a
// failure report says which runtime error it was (include/gpad.h gpad_last_error)
std::string hip_detail(const std::string& what, hipError_t e) {
    return what + ": " + hipGetErrorName(e) + " (code " + std::to_string((int)e) + "): " + hipGetErrorString(e);
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) {                                                              \
            return fail(_e == hipErrorOutOfMemory ? GPAD_ERR_NOMEM : GPAD_ERR_HIP,           \
                        hip_detail(#expr, _e));                                              \
        }                                                                                    \
    } while (0)

size_t esize(int dtype) { return dtype == GPAD_DTYPE_F64 ? sizeof(double) : sizeof(float); }
int round4(int x) { return (x + 3) & ~3; }

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t want) {
        if (want <= bytes && p) return GPAD_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (want == 0) return GPAD_OK;
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(e == hipErrorOutOfMemory ? GPAD_ERR_NOMEM : GPAD_ERR_HIP,
                        hip_detail("hipMalloc(" + std::to_string(want) + " bytes)", e));
        }
        bytes = want;
        return GPAD_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

void host_schedule(int N, int kind, double* theta, double* beta) {
    // acceldualgrad.m:18,27,55-56 (MATLAB: beta lagged one iteration) / paper eq. (8e)
    double th = 1.0, thm1 = 1.0, b = 0.0;
    for (int v = 0; v < N; ++v) {
        const double thn = (std::sqrt(std::pow(th, 4.0) + 4.0 * std::pow(th, 2.0)) - std::pow(th, 2.0)) / 2.0;
        theta[v] = th;
        if (kind == GPAD_SCHEDULE_PAPER) {
            beta[v] = th * (1.0 / thm1 - 1.0);
        } else {
            beta[v] = b;
            b = th * (1.0 / thm1 - 1.0);
        }
        thm1 = th;
        th = thn;
    }
}

}  // namespace

int gpad::set_last_error(int code, const std::string& msg) { return fail(code, msg); }

// Run status block (gpad_handle_s::status): the device error word, then the per-workgroup maxima
// of |g| (launch_absmax) from which the host takes gmax.  The maxima are zeroed before each run's
// first launch; the error word is sticky -- zeroed only when the block is created and right after
// gpad_sync / the stats collection copied it out -- so a fault of an asynchronous run still
// reaches the next sync when further runs were queued behind it.
struct RunStatus {
    int err;
    int pad;
    double part[gpad::kAbsmaxMaxBlocks];
};

struct gpad_handle_s {
    int device = 0;
    hipStream_t stream = nullptr;
    bool ready = false;
    bool flat = false;   // gpad_setup_flat: the flat battery path (gpad_flat.hip)
    int n_u = 0;
    gpad_dims_t dims{};
    double L = 1.0;
    bool scaled = false;
    int ldn = 0, ldm = 0;
    DevBuf MGt, GLt, frag, stage;
    bool frag_ok = false;      // frag holds the fragment image of the bound matrices
    bool keep_stage = false;   // gpad_solve's cached handle keeps its staging buffer
    // gpad_solve: host copy of the last bound (ML, G, L, dims) so a repeated one-shot call on
    // the same host matrices skips the H2D copy and repack
    std::vector<unsigned char> shadow;
    gpad_dims_t shadow_dims{};
    double shadow_L = 0.0;
    bool shadow_ok = false;
    DevBuf GLx;  // flat path: flat G_L expanded to the full k-major image (flat resident kernel)
    DevBuf Hq;           // gpad_setup_hessian: H, k-major [n][ldn] per matrix (value-function branches)
    bool hess_ok = false;
    DevBuf frag64;       // f64 panels (gpad_panel64.hip): -ML | G_L fragment images, shared f64 matrices
    bool frag64_ok = false;
    int frag64_tiles = 0;
    DevBuf hfrag64;      // ... and H's, bound by gpad_setup_hessian (value branches on the f64 panels)
    DevBuf q64;          // f64 panels: the refill queue counter (one int, zeroed per launch)
    // f64 panels with refills: the start order of the next solve -- the previous solve's instances by
    // its counts, longest first (SolveArgs::order; GPAD_OPT_LPT), rebuilt whenever counts arrive
    DevBuf p64_order;
    std::vector<int> p64_order_host;
    int p64_order_batch = 0;
    bool p64_order_dirty = false;
    bool last_p64 = false;  // the last run was an f64 panel solve with a tolerance (its counts order the next)
    bool hfrag64_ok = false;
    int frag_tiles = 0;
    DevBuf theta, beta;
    int sched_len = 0, sched_kind = -1, sched_dtype = -1;
    DevBuf work, counters, pwork;
    std::vector<int> h_counts;
    // run status block on the device, zeroed per run: {int error bits (gpad::kDevErr*), pad,
    // double max |g|} -- the error word the kernels report into and the certification floor's
    // data term (include/gpad.h gpad_run)
    DevBuf status;             // RunStatus
    RunStatus h_status;        // ... its host copy for the stats
    double last_tol = 0.0;          // tol of the last run
    double last_floor_scale = 0.0;  // tol_floor = this * max |g| (margin * L * |gscale|)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int last_kernel = 0, last_batch = 0, last_steps = 1;
    // phased panel solves: the plan made from the previous solve (gpad::panel_plan)
    bool last_phased = false;
    int last_N = 0;
    gpad::PanelPlan plan;
    unsigned long long plan_key = 0;    // fingerprint of the counts the plan was built from
    gpad::PanelPlan prior;              // a handle without its own plan: the shape's last plan (plan_prior)
    bool last_prior = false;            // the last run followed `prior`
    gpad::PanelPlan last_phases;        // the phases the last phased panel solve launched (gpad_last_phases)
    int flat_vpred = 0;                 // flat panels: last iteration of the previous phased solve
    // asynchronous runs (no stats): the counts of each phased solve are copied to pinned host
    // memory behind it; the next run re-plans from them once that copy has landed, so a pipeline
    // of back-to-back solves plans from its most recent completed solve without a host sync
    int* plan_pin = nullptr;
    size_t plan_pin_cap = 0;
    hipEvent_t plan_ev = nullptr;
    bool plan_pending = false;
    int plan_pending_N = 0, plan_pending_batch = 0;
    bool plan_pending_p64 = false;      // ... the pending counts are an f64 panel solve's (build_p64_order)
    // plant binding (gpad_setup_plant): affine state maps and dynamics, device copies
    int nx = 0, nu = 0;
    bool plant_ready = false, plant_dyn = false;
    DevBuf plant;                       // [PM n*nx | M0 n | Pg m*nx | g0 m | A nx*nx | B nx*nu]
    bool has_M0 = false, has_g0 = false;
    int plant_n = 0, plant_m = 0, plant_dtype = -1;
    DevBuf state;                       // per-state workspaces (M(x), g(x), x ping-pong, ...)
    int num_cus = 256;
    bool timed = false;
    gpad::Tuning tune;                  // gpad_set_option
    bool failed_run = false;            // the last run's device error was reported (fetch_status
                                        // clears the device word): later stats calls for that
                                        // run keep returning GPAD_ERR_DEVICE until the next run
};


static int reset_status(gpad_handle_t h, double tol, double floor_scale) {
    const bool fresh = h->status.p == nullptr;
    int rc = h->status.ensure(sizeof(RunStatus));
    if (rc) return rc;
    // the error word once (fetch_status clears it behind each read); the |g| slots are stored by
    // the run's first writer (SolveArgs::gmax_part), so a solve enqueues no memset here
    if (fresh) HIP_TRY(hipMemsetAsync(h->status.p, 0, sizeof(RunStatus), h->stream));
    h->last_tol = tol;
    h->last_floor_scale = floor_scale;
    h->failed_run = false;
    return GPAD_OK;
}

// Enqueue the copy of the status block to *rs (the caller synchronises the stream): the error word,
// and with `maxima` the per-workgroup |g| maxima of the run (RunStatus::part).  The error word is
// cleared behind the copy: every error bit is reported exactly once.
static int fetch_status(gpad_handle_t h, RunStatus* rs, bool maxima = false) {
    rs->err = 0;
    if (!h->status.p) return GPAD_OK;
    const size_t bytes = maxima ? sizeof(RunStatus) : offsetof(RunStatus, part);
    HIP_TRY(hipMemcpyAsync(rs, h->status.p, bytes, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipMemsetAsync(h->status.p, 0, sizeof(int), h->stream));
    return GPAD_OK;
}

static double status_gmax(gpad_handle_t h, const RunStatus& rs) {
    double g = 0.0;
    for (int b = 0; b < gpad::kAbsmaxMaxBlocks; ++b) {
        if (std::isnan(rs.part[b])) return rs.part[b];  // a NaN in g (absmax_nan keeps it)
        g = std::max(g, rs.part[b]);
    }
    return g;
}

static int status_error(gpad_handle_t h, const RunStatus& rs) {
    if (rs.err == 0 && !h->failed_run) return GPAD_OK;
    if (rs.err == 0)
        return fail(GPAD_ERR_DEVICE, "the run failed on the device (reported by an earlier call; its results "
                                     "are invalid)");
    h->failed_run = true;
    return fail(GPAD_ERR_DEVICE, std::string("device error bits 0x") + std::to_string(rs.err) +
                                     ((rs.err & gpad::kDevErrHandoff) ? ": a chain hand-off wait expired "
                                                                        "(the run's results are invalid)"
                                                                      : ""));
}

extern "C" {

const char* gpad_version(void) { return "gpad-mi355x 0.5 (gfx950)"; }

int gpad_device_count(void) {
    return gpad::abi_guard("gpad_device_count", [&]() -> int {
        int count = 0;
        const hipError_t e = hipGetDeviceCount(&count);
        if (e != hipSuccess) return fail(GPAD_ERR_NO_DEVICE, hip_detail("gpad_device_count: hipGetDeviceCount", e));
        return count;
    });
}

const char* gpad_strerror(int status) {
    switch (status) {
        case GPAD_OK: return "ok";
        case GPAD_ERR_INVALID: return "invalid argument";
        case GPAD_ERR_HIP: return "HIP runtime error";
        case GPAD_ERR_NOMEM: return "device out of memory";
        case GPAD_ERR_UNSUPPORTED: return "unsupported shape/kernel combination";
        case GPAD_ERR_NOT_SETUP: return "gpad_run before gpad_setup";
        case GPAD_ERR_NO_DEVICE: return "no HIP device";
        case GPAD_ERR_DEVICE: return "device-side failure (results invalid)";
        default: return "unknown status";
    }
}

const char* gpad_last_error(void) { return g_last_error.c_str(); }

int gpad_create(gpad_handle_t* out, int device, void* stream) {
    return gpad::abi_guard("gpad_create", [&]() -> int {
        if (!out) return fail(GPAD_ERR_INVALID, "gpad_create: null handle pointer");
        *out = nullptr;
        int count = 0;
        const hipError_t e = hipGetDeviceCount(&count);
        if (e != hipSuccess) return fail(GPAD_ERR_NO_DEVICE, hip_detail("gpad_create: hipGetDeviceCount", e));
        if (count <= 0) return fail(GPAD_ERR_NO_DEVICE, "gpad_create: hipGetDeviceCount reported 0 devices");
        if (device < 0 || device >= count)
            return fail(GPAD_ERR_INVALID, "gpad_create: bad device index " + std::to_string(device) + " (" +
                                              std::to_string(count) + " visible)");
        HIP_TRY(hipSetDevice(device));
        auto h = std::make_unique<gpad_handle_s>();
        h->device = device;
        h->stream = static_cast<hipStream_t>(stream);  // NULL = the device's default (null) stream
        {
            hipDeviceProp_t prop;
            if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
                h->num_cus = prop.multiProcessorCount;
        }
        HIP_TRY(hipEventCreate(&h->ev0));
        HIP_TRY(hipEventCreate(&h->ev1));
        *out = h.release();
        return GPAD_OK;
    });
}

int gpad_destroy(gpad_handle_t h) {
    return gpad::abi_guard("gpad_destroy", [&]() -> int {
        if (!h) return GPAD_OK;
        (void)hipSetDevice(h->device);
        (void)hipStreamSynchronize(h->stream);
        h->MGt.release();
        h->GLt.release();
        h->GLx.release();
        h->Hq.release();
        h->frag64.release();
        h->hfrag64.release();
        h->q64.release();
        h->p64_order.release();
        h->frag.release();
        h->stage.release();
        h->theta.release();
        h->beta.release();
        h->work.release();
        h->counters.release();
        h->pwork.release();
        h->status.release();
        h->plant.release();
        h->state.release();
        if (h->ev0) (void)hipEventDestroy(h->ev0);
        if (h->ev1) (void)hipEventDestroy(h->ev1);
        if (h->plan_ev) (void)hipEventDestroy(h->plan_ev);
        if (h->plan_pin) (void)hipHostFree(h->plan_pin);
        delete h;
        return GPAD_OK;
    });
}

int gpad_set_stream(gpad_handle_t h, void* stream) {
    return gpad::abi_guard("gpad_set_stream", [&]() -> int {
        if (!h) return fail(GPAD_ERR_INVALID, "gpad_set_stream: null handle");
        HIP_TRY(hipSetDevice(h->device));
        HIP_TRY(hipStreamSynchronize(h->stream));  // work queued on the old stream completes first
        h->stream = static_cast<hipStream_t>(stream);
        return GPAD_OK;
    });
}

int gpad_set_option(gpad_handle_t h, int option, int value) {
    return gpad::abi_guard("gpad_set_option", [&]() -> int {
        if (!h) return fail(GPAD_ERR_INVALID, "gpad_set_option: null handle");
        gpad::Tuning& t = h->tune;
        const gpad::Tuning def{};
        auto set = [&](int& field, int lo, int hi, int dflt) -> int {
            if (value == GPAD_OPT_DEFAULT) {
                field = dflt;
                return GPAD_OK;
            }
            if (value < lo || value > hi) return fail(GPAD_ERR_INVALID, "gpad_set_option: value out of range");
            field = value;
            return GPAD_OK;
        };
        const int big = 1 << 30;
        switch (option) {
            case GPAD_OPT_PHASE_LEN: return set(t.phase_len, 0, big, def.phase_len);
            case GPAD_OPT_FINISH_THRESH: return set(t.finish_thresh, 0, big, def.finish_thresh);
            case GPAD_OPT_PLAN: h->plan.nph = 0; h->plan_key = 0; return set(t.plan, 0, 1, def.plan);
            case GPAD_OPT_PHASED: return set(t.phased, 0, 2, def.phased);
            case GPAD_OPT_LPT: return set(t.lpt, 0, 1, def.lpt);
            case GPAD_OPT_PANEL_MAX_GRID: return set(t.panel_max_grid, 0, big, def.panel_max_grid);
            case GPAD_OPT_DUO_MAX_GRID: return set(t.duo_max_grid, 0, big, def.duo_max_grid);
            case GPAD_OPT_FLAT_PANEL_MIN: return set(t.flat_panel_min, 0, big, def.flat_panel_min);
            case GPAD_OPT_FLAT_PANELS: return set(t.flat_panels, 0, 4, def.flat_panels);
            case GPAD_OPT_FLAT_WAVES:
                if (value != GPAD_OPT_DEFAULT && value != 0 && value != 8 && value != 16)
                    return fail(GPAD_ERR_INVALID, "gpad_set_option: flat waves must be 0, 8 or 16");
                return set(t.flat_waves, 0, 16, def.flat_waves);
            case GPAD_OPT_FLAT_A_LDS: return set(t.flat_a_lds, 0, 1, def.flat_a_lds);
            case GPAD_OPT_DEBUG_DROP_HANDOFF: return set(t.debug_drop_handoff, 0, 1, def.debug_drop_handoff);
            case GPAD_OPT_P64_REFILL: {
                int on = 1 - t.p64_no_refill;
                const int rc = set(on, 0, 1, 1);
                t.p64_no_refill = 1 - on;
                return rc;
            }
            case GPAD_OPT_P64_RELAY: {
                int on = 1 - t.p64_no_relay;
                const int rc = set(on, 0, 1, 1);
                t.p64_no_relay = 1 - on;
                return rc;
            }
            default: return fail(GPAD_ERR_INVALID, "gpad_set_option: unknown option");
        }
    });
}

int gpad_sync(gpad_handle_t h) {
    return gpad::abi_guard("gpad_sync", [&]() -> int {
        if (!h) return fail(GPAD_ERR_INVALID, "gpad_sync: null handle");
        HIP_TRY(hipSetDevice(h->device));
        RunStatus& rs = h->h_status;
        int rc = fetch_status(h, &rs);
        if (rc) return rc;
        HIP_TRY(hipStreamSynchronize(h->stream));
        return status_error(h, rs);
    });
}

int gpad_schedule(int N, int kind, double* theta, double* beta) {
    return gpad::abi_guard("gpad_schedule", [&]() -> int {
        if (N < 0 || !theta || !beta) return fail(GPAD_ERR_INVALID, "gpad_schedule: bad arguments");
        host_schedule(N, kind, theta, beta);
        return GPAD_OK;
    });
}

static int validate_dims(const gpad_dims_t* d) {
    if (!d) return fail(GPAD_ERR_INVALID, "null dims");
    if (d->n <= 0 || d->m <= 0 || d->batch <= 0)
        return fail(GPAD_ERR_INVALID, "dims: n, m, batch must be positive");
    if (d->dtype != GPAD_DTYPE_F32 && d->dtype != GPAD_DTYPE_F64)
        return fail(GPAD_ERR_INVALID, "dims: bad dtype");
    if (d->memory != GPAD_MEM_HOST && d->memory != GPAD_MEM_DEVICE)
        return fail(GPAD_ERR_INVALID, "dims: bad memory kind");
    if (d->schedule != GPAD_SCHEDULE_MATLAB && d->schedule != GPAD_SCHEDULE_PAPER)
        return fail(GPAD_ERR_INVALID, "dims: bad schedule");
    if (d->kernel < GPAD_KERNEL_AUTO || d->kernel > GPAD_KERNEL_PANEL)
        return fail(GPAD_ERR_INVALID, "dims: bad kernel");
    if (!std::isfinite(d->tol_gap)) return fail(GPAD_ERR_INVALID, "dims: tol_gap must be finite");
    if (d->reserved != 0) return fail(GPAD_ERR_INVALID, "dims: reserved must be 0");
    return GPAD_OK;
}

static int setup_impl(gpad_handle_t h, const gpad_dims_t* d, const void* A, const void* B, double L,
                      bool scaled) {
    if (!h) return fail(GPAD_ERR_INVALID, "gpad_setup: null handle");
    int rc = validate_dims(d);
    if (rc) return rc;
    if (!A || !B) return fail(GPAD_ERR_INVALID, "gpad_setup: null matrix");
    if (!(L > 0.0) || !std::isfinite(L)) return fail(GPAD_ERR_INVALID, "gpad_setup: L must be > 0");
    HIP_TRY(hipSetDevice(h->device));
    h->ready = false;
    h->flat = false;
    h->shadow_ok = false;
    h->hess_ok = false;
    h->frag64_ok = false;
    h->hfrag64_ok = false;
    h->plan.nph = 0;
    h->p64_order_batch = 0;  // (a new problem: the previous counts order nothing)
    h->flat_vpred = 0;
    h->plan_pending = false;
    h->last_phased = false;
    h->dims = *d;
    if (h->dims.check_every <= 0) h->dims.check_every = 10;
    h->L = L;
    h->scaled = scaled;
    const int n = d->n, m = d->m;
    h->ldn = round4(n);
    h->ldm = round4(m);
    const size_t es = esize(d->dtype);
    const int nmats = d->shared ? 1 : d->batch;
    const size_t a_elems = (size_t)m * h->ldn, b_elems = (size_t)n * h->ldm;
    if ((rc = h->MGt.ensure(es * a_elems * nmats))) return rc;
    if ((rc = h->GLt.ensure(es * b_elems * nmats))) return rc;
    const size_t raw = (size_t)n * m * nmats * es;
    const void* dA = A;
    const void* dB = B;
    if (d->memory == GPAD_MEM_HOST) {
        if ((rc = h->stage.ensure(2 * raw))) return rc;
        HIP_TRY(hipMemcpyAsync(h->stage.p, A, raw, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipMemcpyAsync((char*)h->stage.p + raw, B, raw, hipMemcpyHostToDevice, h->stream));
        dA = h->stage.p;
        dB = (char*)h->stage.p + raw;
    }
    // -ML -> k-major [m][ldn];  G/L -> k-major [n][ldm]   (acceldualgrad.m:20,22)
    const double sa = scaled ? 1.0 : -1.0;
    const double sb = scaled ? 1.0 : 1.0 / L;
    const long long in_stride = d->shared ? 0 : (long long)n * m;
    if (d->dtype == GPAD_DTYPE_F32) {
        HIP_TRY(gpad::launch_pack_kmajor<float>((const float*)dA, (float*)h->MGt.p, n, m, h->ldn, sa,
                                                nmats, in_stride, (long long)a_elems, h->stream));
        HIP_TRY(gpad::launch_pack_kmajor<float>((const float*)dB, (float*)h->GLt.p, m, n, h->ldm, sb,
                                                nmats, in_stride, (long long)b_elems, h->stream));
    } else {
        HIP_TRY(gpad::launch_pack_kmajor<double>((const double*)dA, (double*)h->MGt.p, n, m, h->ldn, sa,
                                                 nmats, in_stride, (long long)a_elems, h->stream));
        HIP_TRY(gpad::launch_pack_kmajor<double>((const double*)dB, (double*)h->GLt.p, m, n, h->ldm, sb,
                                                 nmats, in_stride, (long long)b_elems, h->stream));
    }
    // fragment image for the MFMA panel kernel (shared f32 matrices only); the buffer is kept
    // across setups and only grows
    // f64 panels: -ML | G_L in the f64 MFMA fragment layout (gpad_panel64.hip)
    if (d->shared && d->dtype == GPAD_DTYPE_F64 && gpad::panel64_supported(n, m)) {
        const int T = gpad::panel64_tiles(n, m);
        const size_t ob = gpad::panel64_frag_bytes(n, m);
        if ((rc = h->frag64.ensure(2 * ob))) return rc;
        HIP_TRY(gpad::launch_pack_panel64((const double*)dA, n, m, sa, T, h->frag64.p, h->stream));
        HIP_TRY(gpad::launch_pack_panel64((const double*)dB, m, n, sb, T, (char*)h->frag64.p + ob, h->stream));
        h->frag64_tiles = T;
        h->frag64_ok = true;
    }
    h->frag_ok = false;
    h->frag_tiles = 0;
    if (d->shared && d->dtype == GPAD_DTYPE_F32) {
        const size_t fb = gpad::panel_frag_bytes(n, m, d->batch);
        if (fb > 0) {
            if ((rc = h->frag.ensure(fb))) return rc;
            HIP_TRY(gpad::launch_pack_panel((const float*)dA, (const float*)dB, n, m, d->batch,
                                            (float)sa, sb, h->frag.p, h->stream));
            h->frag_tiles = gpad::panel_tiles(n, m, d->batch);
            h->frag_ok = true;
        }
    }
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (d->memory == GPAD_MEM_HOST && !h->keep_stage) h->stage.release();
    h->ready = true;
    return GPAD_OK;
}

int gpad_setup(gpad_handle_t h, const gpad_dims_t* d, const void* ML, const void* G, double L) {
    return gpad::abi_guard("gpad_setup", [&]() -> int {
        return setup_impl(h, d, ML, G, L, false);
    });
}

int gpad_setup_scaled(gpad_handle_t h, const gpad_dims_t* d, const void* MGneg, const void* GL,
                      double L) {
    return gpad::abi_guard("gpad_setup_scaled", [&]() -> int {
        return setup_impl(h, d, MGneg, GL, L, true);
    });
}

int gpad_setup_hessian(gpad_handle_t h, const void* H) {
    return gpad::abi_guard("gpad_setup_hessian", [&]() -> int {
        if (!h) return fail(GPAD_ERR_INVALID, "gpad_setup_hessian: null handle");
        if (!h->ready) return fail(GPAD_ERR_NOT_SETUP, "gpad_setup_hessian: call gpad_setup first");
        if (h->flat) return fail(GPAD_ERR_UNSUPPORTED, "gpad_setup_hessian: not on the flat battery path");
        h->hess_ok = false;
        h->hfrag64_ok = false;
        if (!H) return GPAD_OK;
        HIP_TRY(hipSetDevice(h->device));
        const gpad_dims_t& d = h->dims;
        const int n = d.n, nmats = d.shared ? 1 : d.batch;
        const size_t es = esize(d.dtype), raw = (size_t)n * n * nmats * es;
        int rc;
        if ((rc = h->Hq.ensure(es * (size_t)n * h->ldn * nmats))) return rc;
        const void* dH = H;
        DevBuf stage;
        if (d.memory == GPAD_MEM_HOST) {
            if ((rc = stage.ensure(raw))) return rc;
            HIP_TRY(hipMemcpyAsync(stage.p, H, raw, hipMemcpyHostToDevice, h->stream));
            dH = stage.p;
        }
        const long long in_stride = d.shared ? 0 : (long long)n * n, out_stride = (long long)n * h->ldn;
        if (d.dtype == GPAD_DTYPE_F32)
            HIP_TRY(gpad::launch_pack_kmajor<float>((const float*)dH, (float*)h->Hq.p, n, n, h->ldn, 1.0, nmats, in_stride,
                                                    out_stride, h->stream));
        else
            HIP_TRY(gpad::launch_pack_kmajor<double>((const double*)dH, (double*)h->Hq.p, n, n, h->ldn, 1.0, nmats,
                                                     in_stride, out_stride, h->stream));
        if (h->frag64_ok) {  // shared f64: H for the f64 panels' value branches
            if ((rc = h->hfrag64.ensure(gpad::panel64_frag_bytes(n, d.m)))) return rc;
            HIP_TRY(gpad::launch_pack_panel64((const double*)dH, n, n, 1.0, h->frag64_tiles, h->hfrag64.p, h->stream));
            h->hfrag64_ok = true;
        }
        HIP_TRY(hipStreamSynchronize(h->stream));
        h->hess_ok = true;
        return GPAD_OK;
    });
}

int gpad_setup_flat(gpad_handle_t h, const gpad_dims_t* d, int n_u, const float* MGf, const float* GLf,
                    double L) {
    return gpad::abi_guard("gpad_setup_flat", [&]() -> int {
        if (!h) return fail(GPAD_ERR_INVALID, "gpad_setup_flat: null handle");
        int rc = validate_dims(d);
        if (rc) return rc;
        if (!MGf || !GLf) return fail(GPAD_ERR_INVALID, "gpad_setup_flat: null matrix");
        if (!(L > 0.0) || !std::isfinite(L)) return fail(GPAD_ERR_INVALID, "gpad_setup_flat: L must be > 0");
        if (d->dtype != GPAD_DTYPE_F32 || !d->shared)
            return fail(GPAD_ERR_UNSUPPORTED, "gpad_setup_flat: f32 and shared matrices only");
        if (n_u <= 0 || d->n % n_u != 0 || d->m < 4 * d->n)
            return fail(GPAD_ERR_INVALID, "gpad_setup_flat: need n = n_u*N and m >= 4 n_u N");
        HIP_TRY(hipSetDevice(h->device));
        h->ready = false;
        h->flat = false;
        h->shadow_ok = false;
        h->hess_ok = false;
        h->plan.nph = 0;
        h->p64_order_batch = 0;  // (a new problem: the previous counts order nothing)
        h->flat_vpred = 0;
        h->plan_pending = false;
        h->last_phased = false;
        h->dims = *d;
        if (h->dims.check_every <= 0) h->dims.check_every = 10;
        h->L = L;
        h->scaled = true;
        const int Nh = d->n / n_u, m = d->m;
        const size_t bytes = sizeof(float) * (size_t)Nh * m;
        h->ldn = round4(d->n);
        h->ldm = round4(m);
        if ((rc = h->MGt.ensure(bytes)) || (rc = h->GLt.ensure(bytes))) return rc;
        const void* dG = GLf;
        if (d->memory == GPAD_MEM_HOST) {
            if ((rc = h->stage.ensure(bytes))) return rc;
            HIP_TRY(hipMemcpyAsync(h->MGt.p, MGf, bytes, hipMemcpyHostToDevice, h->stream));
            HIP_TRY(hipMemcpyAsync(h->stage.p, GLf, bytes, hipMemcpyHostToDevice, h->stream));
            dG = h->stage.p;
        } else {
            HIP_TRY(hipMemcpyAsync(h->MGt.p, MGf, bytes, hipMemcpyDeviceToDevice, h->stream));
        }
        HIP_TRY(gpad::launch_transpose_flat((const float*)dG, (float*)h->GLt.p, m, Nh, h->stream));
        h->GLx.release();
        if (gpad::flat_resident_supported(d->n, m, n_u)) {
            if ((rc = h->GLx.ensure(sizeof(float) * (size_t)d->n * h->ldm))) return rc;
            HIP_TRY(gpad::launch_expand_flat_gl((const float*)dG, (float*)h->GLx.p, Nh, n_u, m, h->ldm,
                                                h->stream));
        }
        h->frag_ok = false;
        h->frag_tiles = 0;
        {  // MFMA panels over the flat data (gpad_flatpanel.hip)
            const size_t fb = gpad::flatpanel_frag_bytes(d->n, m, n_u);
            if (fb) {
                if ((rc = h->frag.ensure(fb))) return rc;
                HIP_TRY(gpad::launch_pack_flatpanel((const float*)h->MGt.p, (const float*)h->GLt.p, d->n, m, n_u,
                                                    h->frag.p, h->stream));
                h->frag_ok = true;
            }
        }
        HIP_TRY(hipStreamSynchronize(h->stream));
        if (d->memory == GPAD_MEM_HOST && !h->keep_stage) h->stage.release();
        h->n_u = n_u;
        h->flat = true;
        h->ready = true;
        return GPAD_OK;
    });
}

static int ensure_schedule(gpad_handle_t h, int N, const void* theta_in, const void* beta_in) {
    const int dt = h->dims.dtype;
    const size_t es = esize(dt);
    const bool custom = theta_in != nullptr || beta_in != nullptr;
    if (!custom && h->sched_len >= N + 2 && h->sched_kind == h->dims.schedule && h->sched_dtype == dt)
        return GPAD_OK;
    const int len = N + 2;  // kernels prefetch theta[v+1], beta[v+2]
    std::vector<double> th(len, 0.0), be(len, 0.0);
    host_schedule(N, h->dims.schedule, th.data(), be.data());
    if (custom) {
        if (!theta_in || !beta_in) return fail(GPAD_ERR_INVALID, "run_scaled: give both theta and beta");
        for (int v = 0; v < N; ++v) {
            th[v] = dt == GPAD_DTYPE_F64 ? ((const double*)theta_in)[v] : ((const float*)theta_in)[v];
            be[v] = dt == GPAD_DTYPE_F64 ? ((const double*)beta_in)[v] : ((const float*)beta_in)[v];
        }
    }
    th[N] = th[N + 1] = 0.0;  // pads: read by the prefetch, never used
    be[N] = be[N + 1] = 0.0;
    int rc;
    if ((rc = h->theta.ensure(es * len))) return rc;
    if ((rc = h->beta.ensure(es * len))) return rc;
    if (dt == GPAD_DTYPE_F64) {
        HIP_TRY(hipMemcpyAsync(h->theta.p, th.data(), es * len, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipMemcpyAsync(h->beta.p, be.data(), es * len, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
    } else {
        std::vector<float> tf(len), bf(len);
        for (int i = 0; i < len; ++i) {
            tf[i] = (float)th[i];
            bf[i] = (float)be[i];
        }
        HIP_TRY(hipMemcpyAsync(h->theta.p, tf.data(), es * len, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipMemcpyAsync(h->beta.p, bf.data(), es * len, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
    }
    h->sched_len = custom ? 0 : len;  // custom tables are never reused
    h->sched_kind = h->dims.schedule;
    h->sched_dtype = dt;
    return GPAD_OK;
}

// Shape-keyed plan prior.  A handle plans a phased solve from its OWN previous
// solve's counts, so its first solve ran the default schedule -- ~15 % slower on fresh C4 inputs
// (3.86 vs 3.3-3.4 ms, a second handle's first solve in a warm process), which every new
// gpad_solve caller thread paid once.  The last plan any handle of the process made is kept per
// (n, m, batch, check_every, N, CUs, finisher threshold option), and a handle with no plan of its
// own follows it.  A plan only moves launch boundaries and the finisher takeover (results are
// bit-identical under any plan), so a stale prior costs time, never correctness.
using PlanShape = std::tuple<int, int, int, int, int, int, int>;
static std::mutex g_prior_mu;
static std::map<PlanShape, gpad::PanelPlan>& prior_plans() {
    static std::map<PlanShape, gpad::PanelPlan> m;
    return m;
}
static PlanShape plan_shape(gpad_handle_t h, int batch, int N) {
    return PlanShape{h->dims.n, h->dims.m, batch, h->dims.check_every, N, h->num_cus, h->tune.finish_thresh};
}
static void plan_prior_store(gpad_handle_t h, int batch, int N) {
    if (h->plan.nph <= 0) return;
    std::lock_guard<std::mutex> lk(g_prior_mu);
    auto& m = prior_plans();
    if (m.size() >= 64 && !m.count(plan_shape(h, batch, N))) m.clear();  // (bounded: a handful of shapes)
    m[plan_shape(h, batch, N)] = h->plan;
}
// the plan a phased solve of this handle follows: its own, else the shape's prior (or none)
static const gpad::PanelPlan* plan_for(gpad_handle_t h, int batch, int N) {
    h->last_prior = false;
    if (!h->tune.plan) return nullptr;
    if (h->plan.nph > 0 && h->plan.N == N) return &h->plan;
    std::lock_guard<std::mutex> lk(g_prior_mu);
    auto it = prior_plans().find(plan_shape(h, batch, N));
    if (it == prior_plans().end()) return nullptr;
    h->prior = it->second;
    h->last_prior = true;
    return &h->prior;
}

// The phase plan is a pure function of the per-instance counts (and the shape): rebuild it only
// when they changed (repeated solves of one batch skip the DP).
static void update_plan(gpad_handle_t h, const int* counts, int batch, int N) {
    if (h->flat) {  // the flat panels' phases run to the previous solve's last iteration
        int mx = 0;
        for (int b = 0; b < batch; ++b) mx = std::max(mx, counts[b]);
        h->flat_vpred = mx;
        return;
    }
    unsigned long long key = 1469598103934665603ull ^ (unsigned long long)N;
    for (int b = 0; b < batch; ++b) key = (key ^ (unsigned)counts[b]) * 1099511628211ull;
    if (key != h->plan_key || h->plan.nph == 0) {
        gpad::panel_plan(counts, batch, h->dims.n, h->dims.m, N, h->dims.check_every, h->num_cus, &h->tune,
                         &h->plan);
        h->plan_key = key;
        plan_prior_store(h, batch, N);
    }
}

// f64 panels: the next solve starts its instances longest-predicted-first, so
// the column refills pair long instances with short ones (greedy list scheduling over the columns)
// instead of in batch order -- each column's two-or-more instances then end together.  Predicted =
// the previous solve's counts on the same batch size (an MPC stream's statistics, or the same batch
// re-solved); ties keep batch order (stable).  Only the schedule changes: every instance runs the same
// arithmetic in any column (bit-identical results, tests/test_panel64.py).
static void build_p64_order(gpad_handle_t h, const int* counts, int batch) {
    h->p64_order_host.resize(batch);
    for (int b = 0; b < batch; ++b) h->p64_order_host[b] = b;
    std::stable_sort(h->p64_order_host.begin(), h->p64_order_host.end(),
                     [&](int x, int y) { return counts[x] > counts[y]; });
    h->p64_order_batch = batch;
    h->p64_order_dirty = true;
}

// Counters are laid out [steps][iters[batch] | conv[batch]].
static int collect_stats(gpad_handle_t h, gpad_stats_t* st) {
    const int batch = h->last_batch;
    const size_t entries = (size_t)batch * h->last_steps;
    h->h_counts.resize(2 * entries);
    HIP_TRY(hipMemcpyAsync(h->h_counts.data(), h->counters.p, sizeof(int) * 2 * entries,
                           hipMemcpyDeviceToHost, h->stream));
    RunStatus& rs = h->h_status;
    int rc = fetch_status(h, &rs, true);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    st->iterations = 0;
    st->converged = 0;
    st->total_iterations = 0;
    for (int t = 0; t < h->last_steps; ++t) {
        const int* it = h->h_counts.data() + (size_t)2 * batch * t;
        const int* cv = it + batch;
        for (int b = 0; b < batch; ++b) {
            st->iterations = std::max(st->iterations, it[b]);
            st->converged += cv[b] != 0;
            st->total_iterations += it[b];
            if (st->iters) st->iters[(size_t)t * batch + b] = it[b];
            if (st->codes) st->codes[(size_t)t * batch + b] = cv[b];
        }
    }
    if (h->last_phased && h->last_steps == 1) {
        update_plan(h, h->h_counts.data(), batch, h->last_N);
        h->plan_pending = false;  // these counts are at least as recent as any copy in flight
    }
    if (h->last_p64 && h->last_steps == 1) {
        build_p64_order(h, h->h_counts.data(), batch);
        h->plan_pending = false;
    }
    st->kernel = h->last_kernel;
    float ms = 0.0f;
    st->kernel_ms = 0.0;
    if (h->timed && hipEventElapsedTime(&ms, h->ev0, h->ev1) == hipSuccess) st->kernel_ms = ms;
    st->tol_floor = h->last_tol > 0.0 ? h->last_floor_scale * status_gmax(h, rs) : 0.0;
    st->flags = (h->last_tol > 0.0 && h->last_tol < st->tol_floor) ? GPAD_FLAG_TOL_FLOOR : 0;
    if (h->last_tol > 0.0 && !std::isfinite(st->tol_floor))  // NaN / inf in g: nothing certifies
        st->flags |= GPAD_FLAG_TOL_FLOOR | GPAD_FLAG_NONFINITE_G;
    return status_error(h, rs);
}

int gpad_accumulate_iterations(gpad_handle_t h, long long* acc) {
    return gpad::abi_guard("gpad_accumulate_iterations", [&]() -> int {
        if (!h || !acc) return fail(GPAD_ERR_INVALID, "gpad_accumulate_iterations: null argument");
        if (h->last_batch <= 0) return fail(GPAD_ERR_NOT_SETUP, "gpad_accumulate_iterations: no run yet");
        HIP_TRY(hipSetDevice(h->device));
        // counters: [steps][iters[batch] | conv[batch]]; each solve's iteration block in turn
        for (int t = 0; t < h->last_steps; ++t)
            HIP_TRY(gpad::launch_accumulate_iters((const int*)h->counters.p + (size_t)2 * h->last_batch * t,
                                                  h->last_batch, acc, h->stream));
        return GPAD_OK;
    });
}

int gpad_last_stats(gpad_handle_t h, gpad_stats_t* st) {
    return gpad::abi_guard("gpad_last_stats", [&]() -> int {
        if (!h || !st) return fail(GPAD_ERR_INVALID, "gpad_last_stats: null argument");
        if (h->last_batch <= 0) return fail(GPAD_ERR_NOT_SETUP, "gpad_last_stats: no run yet");
        HIP_TRY(hipSetDevice(h->device));
        return collect_stats(h, st);
    });
}

int gpad_phase_plan(gpad_handle_t h, int* ends, int* fins, int cap, double* cost_us) {
    return gpad::abi_guard("gpad_phase_plan", [&]() -> int {
        if (!h) return fail(GPAD_ERR_INVALID, "gpad_phase_plan: null handle");
        const int n = h->plan.nph;
        for (int i = 0; i < n && i < cap; ++i) {
            if (ends) ends[i] = h->plan.ends[i];
            if (fins) fins[i] = h->plan.fins[i];
        }
        if (cost_us) *cost_us = h->plan.cost_us;
        return n;
    });
}

int gpad_last_phases(gpad_handle_t h, int* ends, int* fins, int* counts, int cap, int* prior) {
    return gpad::abi_guard("gpad_last_phases", [&]() -> int {
        if (!h || cap < 0) return fail(GPAD_ERR_INVALID, "gpad_last_phases: bad argument");
        if (prior) *prior = h->last_prior ? 1 : 0;
        if (!h->last_phased || !h->pwork.p || h->flat) return 0;
        const int k = std::min(cap, h->last_phases.nph);
        for (int i = 0; i < k; ++i) {
            if (ends) ends[i] = h->last_phases.ends[i];
            if (fins) fins[i] = h->last_phases.fins[i];
        }
        if (counts && k > 0) {
            HIP_TRY(hipSetDevice(h->device));
            const int* dev = reinterpret_cast<const int*>(h->pwork.p) + 2 * (size_t)h->last_batch;  // panel_work_bytes
            HIP_TRY(hipMemcpyAsync(counts, dev, sizeof(int) * (size_t)k, hipMemcpyDeviceToHost, h->stream));
            HIP_TRY(hipStreamSynchronize(h->stream));
        }
        return k;
    });
}

int gpad_phase_counts(gpad_handle_t h, int* counts, int cap) {
    return gpad::abi_guard("gpad_phase_counts", [&]() -> int {
        if (!h || !counts || cap < 0) return fail(GPAD_ERR_INVALID, "gpad_phase_counts: bad argument");
        if (!h->last_phased || !h->pwork.p) return 0;
        HIP_TRY(hipSetDevice(h->device));
        const int k = cap < gpad::kPanelMaxPhases ? cap : gpad::kPanelMaxPhases;
        const int* dev = reinterpret_cast<const int*>(h->pwork.p) + 2 * (size_t)h->last_batch;  // panel_work_bytes
        HIP_TRY(hipMemcpyAsync(counts, dev, sizeof(int) * (size_t)k, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        return k;
    });
}

#ifdef GPAD_STAMP
}  // extern "C"
namespace gpad {
hipError_t read_stamps(unsigned long long* out, size_t bytes);      // gpad_panel.hip (diagnostic builds)
hipError_t read_res_stamps(unsigned long long* out, size_t bytes);  // gpad_kernels.hip
hipError_t read_duo_stamps(unsigned long long* out, size_t bytes);  // gpad_duo.hip
}
extern "C" {
int gpad_debug_res_stamps(unsigned long long* out, size_t bytes) {
    return gpad::abi_guard("gpad_debug_res_stamps", [&]() -> int {
        HIP_TRY(gpad::read_res_stamps(out, bytes));
        return GPAD_OK;
    });
}
int gpad_debug_duo_stamps(unsigned long long* out, size_t bytes) {
    return gpad::abi_guard("gpad_debug_duo_stamps", [&]() -> int {
        HIP_TRY(gpad::read_duo_stamps(out, bytes));
        return GPAD_OK;
    });
}
// diagnostic builds only (not declared in gpad.h): the phase-anatomy stamps of the last panel-pair run
int gpad_debug_stamps(unsigned long long* out, size_t bytes) {
    return gpad::abi_guard("gpad_debug_stamps", [&]() -> int {
        HIP_TRY(gpad::read_stamps(out, bytes));
        return GPAD_OK;
    });
}
#endif

int gpad_plan_phases(const int* iters, int batch, int n, int m, int N, int check_every, int num_cus,
                     int* ends, int* fins, int cap, double* cost_us) {
    return gpad::abi_guard("gpad_plan_phases", [&]() -> int {
        if (!iters || batch <= 0 || n <= 0 || m <= 0 || N <= 0 || num_cus <= 0)
            return fail(GPAD_ERR_INVALID, "gpad_plan_phases: bad argument");
        gpad::PanelPlan p;
        gpad::panel_plan(iters, batch, n, m, N, check_every, num_cus, nullptr, &p);
        for (int i = 0; i < p.nph && i < cap; ++i) {
            if (ends) ends[i] = p.ends[i];
            if (fins) fins[i] = p.fins[i];
        }
        if (cost_us) *cost_us = p.cost_us;
        return p.nph;
    });
}

}  // extern "C"

// Enqueue one fused solve on device buffers (no staging, no sync).  Counters: iters/conv
// [batch] each.  *kernel_out = the family that ran.
template <typename T>
static int launch_solve(gpad_handle_t h, T* dz, T* dy, const T* dM, const T* dg, int N, double tol,
                        bool scaled_vec, int* iters, int* conv, int* kernel_out) {
    const gpad_dims_t& d = h->dims;
    const int n = d.n, m = d.m, batch = d.batch;
    gpad::SolveArgs<T> a{};
    a.MGt = (const T*)h->MGt.p;
    a.GLt = (const T*)h->GLt.p;
    a.strideA = d.shared ? 0 : (long long)m * h->ldn;
    a.strideB = d.shared ? 0 : (long long)n * h->ldm;
    a.frag = h->frag_ok ? h->frag.p : nullptr;
    a.frag_tiles = h->frag_tiles;
    a.gP = dM;
    a.g = dg;
    a.ld_gP = n;
    a.ld_g = m;
    a.gscale = scaled_vec ? 1.0 : -1.0 / h->L;
    a.z = dz;
    a.y = dy;
    a.n = n;
    a.m = m;
    a.ldn = h->ldn;
    a.ldm = h->ldm;
    a.batch = batch;
    a.N = N;
    a.check_every = d.check_every;
    a.tol = tol;
    a.tol_gap = d.tol_gap > 0.0 ? d.tol_gap : tol;
    a.L = h->L;
    a.theta = (const T*)h->theta.p;
    a.beta = (const T*)h->beta.p;
    a.iters = iters;
    a.conv = conv;
    a.num_cus = h->num_cus;
    a.tune = &h->tune;
    a.Hq = (h->hess_ok && tol > 0.0) ? (const T*)h->Hq.p : nullptr;
    a.strideHq = d.shared ? 0 : (long long)n * h->ldn;
    a.err = (int*)h->status.p;
    a.debug = h->tune.debug_drop_handoff ? gpad::kDebugDropHandoff : 0;
    // the certification floor's data term max |g| (stats: tol_floor, GPAD_FLAG_TOL_FLOOR): folded
    // into the panel pairs' own loads, else one launch_absmax after the solve's launches
    double* gpart = tol > 0.0 ? reinterpret_cast<double*>((char*)h->status.p + offsetof(RunStatus, part)) : nullptr;
    bool gmax_done = false;
    if constexpr (sizeof(T) == sizeof(float)) a.gmax_part = gpart;
    auto finish = [&](int rc) {
        if (rc == GPAD_OK && gpart && !gmax_done) {
            const hipError_t ea = gpad::launch_absmax<T>(dg, (long long)batch * m, gpart, h->stream);
            if (ea != hipSuccess) return fail(GPAD_ERR_HIP, std::string("absmax: ") + hipGetErrorString(ea));
        }
        return rc;
    };
    int kernel = d.kernel;
    const bool prev_phased = h->last_phased;  // the previous launch's counts are still in `iters`
    h->last_phased = false;  // set again below when this launch is a phased panel solve
    h->last_p64 = false;
    h->last_N = N;
    hipError_t e = hipSuccess;
    bool ok = false;
    if (N == 0) {  // nothing to iterate: outputs are the inputs, zero counts
        HIP_TRY(hipMemsetAsync(a.iters, 0, sizeof(int) * (size_t)batch, h->stream));
        HIP_TRY(hipMemsetAsync(a.conv, 0, sizeof(int) * (size_t)batch, h->stream));
        *kernel_out = d.kernel == GPAD_KERNEL_AUTO ? GPAD_KERNEL_STREAM : d.kernel;
        return finish(GPAD_OK);
    }
    if constexpr (sizeof(T) == sizeof(double)) {
        // f64 panels on the f64 MFMA pipe (shared matrices, n, m <= 256; value branches included):
        // forced, or from one panel per CU on (below that the one-instance-per-workgroup stream
        // kernel has the shorter iteration)
        if (h->frag64_ok && (kernel == GPAD_KERNEL_PANEL || (kernel == GPAD_KERNEL_AUTO && batch >= 16 * h->num_cus))) {
            a.frag = h->frag64.p;
            a.frag_tiles = h->frag64_tiles;
            if (int rq = h->q64.ensure(sizeof(int))) return rq;
            a.qctr = static_cast<int*>(h->q64.p);
            a.hfrag64 = (a.Hq && h->hfrag64_ok) ? h->hfrag64.p : nullptr;
            a.Hq = nullptr;
            if (tol > 0.0 && h->tune.lpt && h->p64_order_batch == batch && (int)h->p64_order_host.size() == batch) {
                if (h->p64_order_dirty) {
                    if (int ro = h->p64_order.ensure(sizeof(int) * (size_t)batch)) return ro;
                    HIP_TRY(hipMemcpyAsync(h->p64_order.p, h->p64_order_host.data(), sizeof(int) * (size_t)batch,
                                           hipMemcpyHostToDevice, h->stream));
                    h->p64_order_dirty = false;
                }
                a.order = static_cast<const int*>(h->p64_order.p);
            }
            e = gpad::launch_panel64(a, h->stream);
            if (e != hipSuccess) return fail(GPAD_ERR_HIP, hip_detail("f64 panel", e));
            h->last_p64 = tol > 0.0;
            *kernel_out = GPAD_KERNEL_PANEL;
            return finish(GPAD_OK);
        }
    }
    if (a.Hq) {  // value-function branches: the stream kernel family (and the f64 panels, above)
        if (kernel != GPAD_KERNEL_AUTO && kernel != GPAD_KERNEL_STREAM)
            return fail(GPAD_ERR_UNSUPPORTED, "the value-function test (gpad_setup_hessian) runs on the stream kernel "
                                              "(f32) or the stream / f64 panel kernels (f64)");
        kernel = GPAD_KERNEL_STREAM;
    }
    if constexpr (sizeof(T) == sizeof(float)) {
        if (kernel == GPAD_KERNEL_STREAM && !h->flat) {
            // forced stream kernel (or the value-function test): none of the f32 families below
        } else if (h->flat) {  // (flat data with STREAM forced: the LDS flat kernel)  // structure-exploiting battery path (gpad_setup_flat)
            a.n_u = h->n_u;
            // flat panels from 8 instances per CU when the register-resident flat chains exist
            // (their per-CU cost grows with the batch, a panel's does not until every CU holds
            // one: crossover ~2048 at C1, tools/fp_cross.py); always when only the LDS flat
            // kernel would be left (several times slower at any batch)
            const int fpm = h->tune.flat_panel_min >= 0 ? h->tune.flat_panel_min : (h->GLx.p ? 8 * h->num_cus : 0);
            if (h->frag_ok && (kernel == GPAD_KERNEL_PANEL || (kernel == GPAD_KERNEL_AUTO && batch >= fpm))) {
                if (tol > 0.0) {  // phased compaction workspace (gpad_flatpanel.hip)
                    int rc = h->pwork.ensure(gpad::panel_work_bytes(m, batch));
                    if (rc) return rc;
                    a.pwork = h->pwork.p;
                    a.v_pred = h->flat_vpred;  // the previous solve's last iteration (0: unknown)
                }
                e = gpad::launch_flatpanel(a, h->stream);
                h->last_phased = a.pwork != nullptr;
            } else if (h->GLx.p && kernel != GPAD_KERNEL_STREAM) {  // register-resident flat chains
                a.GLt = (const T*)h->GLx.p;
                a.strideA = a.strideB = 0;
                e = gpad::launch_flat_resident(a, h->stream);
            } else {
                e = gpad::launch_flat(a, h->stream);
            }
            if (e != hipSuccess)
                return fail(e == hipErrorInvalidValue ? GPAD_ERR_UNSUPPORTED : GPAD_ERR_HIP,
                            std::string("flat kernel: ") + hipGetErrorString(e));
            *kernel_out = GPAD_KERNEL_FLAT;
            return finish(GPAD_OK);
        }
        // shared matrices: panels once there are more instances than the latency kernel can
        // run at ~one round (4 per CU: 4 x its 1/6-panel iteration time < one panel iteration)
        const int panel_min = gpad::resident_supported(n, m) ? 4 * h->num_cus : 64;
        if (kernel == GPAD_KERNEL_PANEL || (kernel == GPAD_KERNEL_AUTO && d.shared && batch > panel_min)) {
            if (tol > 0.0 && h->frag_ok) {  // phased compaction workspace (gpad_panel.hip)
                int rc = h->pwork.ensure(gpad::panel_work_bytes(m, batch));
                if (rc) return rc;
                a.pwork = h->pwork.p;
                a.plan = plan_for(h, batch, N);
                a.used = &h->last_phases;
                // the previous phased solve's counts are still in `iters` for every instance this
                // solve has not finished yet: the finisher orders its queue by them
                if (prev_phased && h->last_batch == batch && h->last_steps == 1) a.pred = iters;
            }
            e = gpad::launch_panel(a, h->stream, &ok);
            if (e != hipSuccess) return fail(GPAD_ERR_HIP, std::string("panel: ") + hipGetErrorString(e));
            if (ok) kernel = GPAD_KERNEL_PANEL;
            else if (kernel == GPAD_KERNEL_PANEL)
                return fail(GPAD_ERR_UNSUPPORTED, "panel kernel: needs shared f32 matrices");
            gmax_done = ok && gpad::panel_folds_gmax(n, m);
        }
        if (!ok && (kernel == GPAD_KERNEL_RESIDENT || kernel == GPAD_KERNEL_AUTO)) {
            e = gpad::launch_resident(a, h->stream, &ok);
            if (e != hipSuccess) return fail(GPAD_ERR_HIP, std::string("resident: ") + hipGetErrorString(e));
            if (ok) kernel = GPAD_KERNEL_RESIDENT;
            else if (kernel == GPAD_KERNEL_RESIDENT)
                return fail(GPAD_ERR_UNSUPPORTED, "resident kernel: needs n, m <= 208");
        }
    } else {
        if (kernel == GPAD_KERNEL_PANEL || kernel == GPAD_KERNEL_RESIDENT)
            return fail(GPAD_ERR_UNSUPPORTED, "f64: the resident kernel is f32 only; the f64 panels need shared "
                                              "matrices with n, m <= 256");
    }
    if (!ok) {
        kernel = GPAD_KERNEL_STREAM;
        e = gpad::launch_stream<T>(a, h->stream);
        if (e != hipSuccess)
            return fail(e == hipErrorInvalidValue ? GPAD_ERR_UNSUPPORTED : GPAD_ERR_HIP,
                        std::string("stream kernel: ") + hipGetErrorString(e) +
                            " (n+m beyond the LDS budget?)");
    }
    *kernel_out = kernel;
    h->last_phased = kernel == GPAD_KERNEL_PANEL && a.pwork != nullptr;
    return finish(GPAD_OK);
}

template <typename T>
static int run_typed(gpad_handle_t h, T* z, T* y, const T* M, const T* g, int N, double tol,
                     const void* theta_in, const void* beta_in, bool scaled_vec, gpad_stats_t* st) {
    const gpad_dims_t& d = h->dims;
    const int n = d.n, m = d.m, batch = d.batch;
    int rc = ensure_schedule(h, N, theta_in, beta_in);
    if (rc) return rc;
    // [iters | conv]
    if ((rc = h->counters.ensure(sizeof(int) * 2 * (size_t)batch))) return rc;
    T *dz = z, *dy = y;
    const T *dM = M, *dg = g;
    const size_t zb = sizeof(T) * (size_t)batch * n, yb = sizeof(T) * (size_t)batch * m;
    if (d.memory == GPAD_MEM_HOST) {
        if ((rc = h->work.ensure(2 * zb + 2 * yb))) return rc;
        char* base = (char*)h->work.p;
        dz = (T*)base;
        dy = (T*)(base + zb);
        T* wM = (T*)(base + zb + yb);
        T* wg = (T*)(base + 2 * zb + yb);
        HIP_TRY(hipMemcpyAsync(dz, z, zb, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipMemcpyAsync(dy, y, yb, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipMemcpyAsync(wM, M, zb, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipMemcpyAsync(wg, g, yb, hipMemcpyHostToDevice, h->stream));
        dM = wM;
        dg = wg;
    }
    int* iters = (int*)h->counters.p;
    int kernel = 0;
    const double margin = sizeof(T) == sizeof(float) ? gpad::ViolMargin<float>::value : gpad::ViolMargin<double>::value;
    if ((rc = reset_status(h, tol, margin * h->L * (scaled_vec ? 1.0 : 1.0 / h->L)))) return rc;
    if (h->plan_pending && hipEventQuery(h->plan_ev) == hipSuccess) {  // a previous solve's counts landed
        if (h->plan_pending_batch == batch) {
            if (h->plan_pending_p64) build_p64_order(h, h->plan_pin, batch);
            else update_plan(h, h->plan_pin, batch, h->plan_pending_N);
        }
        h->plan_pending = false;
    }
    HIP_TRY(hipEventRecord(h->ev0, h->stream));
    if ((rc = launch_solve<T>(h, dz, dy, dM, dg, N, tol, scaled_vec, iters, iters + batch, &kernel)))
        return rc;
    HIP_TRY(hipEventRecord(h->ev1, h->stream));
    h->timed = true;
    h->last_kernel = kernel;
    h->last_batch = batch;
    h->last_steps = 1;
    if (!st && ((h->last_phased && h->tune.plan) || (h->last_p64 && h->tune.lpt))) {  // asynchronous run: counts
        // to the host behind it
        const size_t want = sizeof(int) * (size_t)batch;
        if (h->plan_pin_cap < want) {
            if (h->plan_pending) {  // the previous run's copy into the old buffer must land first
                HIP_TRY(hipEventSynchronize(h->plan_ev));
                h->plan_pending = false;
            }
            if (h->plan_pin) (void)hipHostFree(h->plan_pin);
            h->plan_pin = nullptr;
            h->plan_pin_cap = 0;
            HIP_TRY(hipHostMalloc((void**)&h->plan_pin, want, hipHostMallocDefault));
            h->plan_pin_cap = want;
        }
        if (!h->plan_ev) HIP_TRY(hipEventCreateWithFlags(&h->plan_ev, hipEventDisableTiming));
        HIP_TRY(hipMemcpyAsync(h->plan_pin, iters, want, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipEventRecord(h->plan_ev, h->stream));
        h->plan_pending = true;
        h->plan_pending_N = N;
        h->plan_pending_batch = batch;
        h->plan_pending_p64 = h->last_p64;
    }
    if (st) {
        if (d.memory == GPAD_MEM_HOST) {
            HIP_TRY(hipMemcpyAsync(z, dz, zb, hipMemcpyDeviceToHost, h->stream));
            HIP_TRY(hipMemcpyAsync(y, dy, yb, hipMemcpyDeviceToHost, h->stream));
        }
        return collect_stats(h, st);  // synchronises; a device error fails the run
    }
    if (d.memory == GPAD_MEM_HOST) {
        HIP_TRY(hipMemcpyAsync(z, dz, zb, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipMemcpyAsync(y, dy, yb, hipMemcpyDeviceToHost, h->stream));
        return gpad_sync(h);
    }
    return GPAD_OK;
}

extern "C" {

static int run_impl(gpad_handle_t h, void* z0, void* y0, const void* M, const void* g, int N,
                    double tol, const void* theta, const void* beta, bool scaled_vec,
                    gpad_stats_t* st) {
    if (!h) return fail(GPAD_ERR_INVALID, "gpad_run: null handle");
    if (!h->ready) return fail(GPAD_ERR_NOT_SETUP, "gpad_run: call gpad_setup first");
    if (!z0 || !y0 || !M || !g) return fail(GPAD_ERR_INVALID, "gpad_run: null vector");
    if (N < 0) return fail(GPAD_ERR_INVALID, "gpad_run: N < 0");
    if (!(tol <= 0.0) && !std::isfinite(tol)) return fail(GPAD_ERR_INVALID, "gpad_run: bad tol");
    HIP_TRY(hipSetDevice(h->device));
    if (h->dims.dtype == GPAD_DTYPE_F64)
        return run_typed<double>(h, (double*)z0, (double*)y0, (const double*)M, (const double*)g, N,
                                 tol, theta, beta, scaled_vec, st);
    return run_typed<float>(h, (float*)z0, (float*)y0, (const float*)M, (const float*)g, N, tol, theta,
                            beta, scaled_vec, st);
}

int gpad_run(gpad_handle_t h, void* z0, void* y0, const void* M, const void* g, int N, double tol,
             gpad_stats_t* st) {
    return gpad::abi_guard("gpad_run", [&]() -> int {
        return run_impl(h, z0, y0, M, g, N, tol, nullptr, nullptr, false, st);
    });
}

int gpad_run_scaled(gpad_handle_t h, void* z0, void* y0, const void* gP, const void* pD, int N,
                    double tol, const void* theta, const void* beta, gpad_stats_t* st) {
    return gpad::abi_guard("gpad_run_scaled", [&]() -> int {
        return run_impl(h, z0, y0, gP, pD, N, tol, theta, beta, true, st);
    });
}

// field by field: a stack-built dims may carry different padding bytes on every call
static bool same_dims(const gpad_dims_t& a, const gpad_dims_t& b) {
    return a.n == b.n && a.m == b.m && a.batch == b.batch && a.shared == b.shared && a.dtype == b.dtype &&
           a.memory == b.memory && a.schedule == b.schedule && a.check_every == b.check_every &&
           a.kernel == b.kernel && a.reserved == b.reserved && a.tol_gap == b.tol_gap;
}

}  // extern "C"

// gpad_solve's per-thread handle: freed by gpad_release_cached(), not by a thread-exit destructor
// (at process exit that may run after the HIP runtime tore down; the OS reclaims it then).
namespace {
struct SolveCache {
    gpad_handle_t h = nullptr;
    int device = -1;
};
thread_local SolveCache t_solve_cache;
}  // namespace

extern "C" {

void gpad_release_cached(void) {
    if (t_solve_cache.h) gpad_destroy(t_solve_cache.h);
    t_solve_cache.h = nullptr;
    t_solve_cache.device = -1;
    gpad::release_sharded_cache();
}

int gpad_solve(void* z0, void* y0, const void* ML, const void* M, const void* G, const void* g, int N,
               double L, double tol, const gpad_dims_t* dims, gpad_stats_t* st) {
    return gpad::abi_guard("gpad_solve", [&]() -> int {
        // One handle per thread and device, kept between calls: a per-MPC-step caller (gpad.m:90)
        // pays the handle, the workspaces and -- when the host matrices are unchanged -- the H2D
        // copy and repack of ML/G once, not per call.  gpad_release_cached() frees it.
        SolveCache& cache = t_solve_cache;
        int rc = validate_dims(dims);
        if (rc) return rc;
        if (!ML || !G) return fail(GPAD_ERR_INVALID, "gpad_solve: null matrix");
        int dev = 0;
        HIP_TRY(hipGetDevice(&dev));
        if (!cache.h || cache.device != dev) {
            if (cache.h) gpad_destroy(cache.h);
            cache.h = nullptr;
            if ((rc = gpad_create(&cache.h, dev, nullptr))) return rc;
            cache.device = dev;
            cache.h->keep_stage = true;
        }
        gpad_handle_t h = cache.h;
        // host matrices: reuse the bound problem when (dims, L, ML, G) equal the last call's; the
        // comparison is the full contents (a caller may rewrite its buffers in place).  Device
        // matrices are always repacked (two stream-ordered pack kernels, no copy).
        const bool host = dims->memory == GPAD_MEM_HOST;
        const size_t bytes = (size_t)dims->n * dims->m * esize(dims->dtype) * (dims->shared ? 1 : dims->batch);
        bool same = false;
        if (host && h->ready && h->shadow_ok && L == h->shadow_L && same_dims(h->shadow_dims, *dims) &&
            h->shadow.size() == 2 * bytes)
            same = std::memcmp(h->shadow.data(), ML, bytes) == 0 && std::memcmp(h->shadow.data() + bytes, G, bytes) == 0;
        if (!same) {
            if ((rc = gpad_setup(h, dims, ML, G, L))) return rc;
            if (host) {
                h->shadow.resize(2 * bytes);
                std::memcpy(h->shadow.data(), ML, bytes);
                std::memcpy(h->shadow.data() + bytes, G, bytes);
                h->shadow_dims = *dims;
                h->shadow_L = L;
                h->shadow_ok = true;
            }
        }
        if ((rc = gpad_run(h, z0, y0, M, g, N, tol, st))) return rc;
        return gpad_sync(h);
    });
}

// ---- per-state QP data and closed-loop MPC (gpad.m:79-95) --------
}  // extern "C"

namespace {
struct PlantOffsets {
    size_t PM, M0, Pg, g0, A, B, total;
};
PlantOffsets plant_offsets(int n, int m, int nx, int nu) {
    PlantOffsets o{};
    o.PM = 0;
    o.M0 = o.PM + (size_t)n * nx;
    o.Pg = o.M0 + (size_t)n;
    o.g0 = o.Pg + (size_t)m * nx;
    o.A = o.g0 + (size_t)m;
    o.B = o.A + (size_t)nx * nx;
    o.total = o.B + (size_t)nx * nu;
    return o;
}
}  // namespace

extern "C" int gpad_precompute(gpad_handle_t h, int n, int m, int batch, int shared, int memory, const double* H,
                               const double* A, const double* f, double* ML, double* gP, double* L) {
    return gpad::abi_guard("gpad_precompute", [&]() -> int {
        if (!h) return fail(GPAD_ERR_INVALID, "gpad_precompute: null handle");
        if (n <= 0 || m < 0 || batch <= 0 || !H || !A || !ML || !L || (f == nullptr) != (gP == nullptr) ||
            (memory != GPAD_MEM_HOST && memory != GPAD_MEM_DEVICE))
            return fail(GPAD_ERR_INVALID, "gpad_precompute: bad arguments");
        HIP_TRY(hipSetDevice(h->device));
        const bool host = memory == GPAD_MEM_HOST;
        const int nmat = shared ? 1 : batch;  // eliminations
        const size_t nH = (size_t)nmat * n * n, nA = (size_t)nmat * m * n, nML = (size_t)nmat * n * m;
        const size_t nF = f ? (size_t)batch * n : 0;
        // shared: one elimination of [H | A' | I] gives ML and inv(H); gP = inv(H) f' per row after
        const int fchunk = shared ? (f ? n : 0) : (f ? 1 : 0);
        if (!gpad::precompute_supported(n, m, fchunk))
            return fail(GPAD_ERR_UNSUPPORTED, "gpad_precompute: 2n + m too large for the LDS pivot row");
        // device views of the operands (host memory: staged copies)
        DevBuf stage, work;
        const double *dH = H, *dA = A, *df = f;
        double *dML = ML, *dgP = gP, *dL = L;
        const size_t tot = nH + nA + nF + nML + nF + nmat;
        int rc;
        if (host) {
            if ((rc = stage.ensure(sizeof(double) * tot))) return rc;
            double* b = (double*)stage.p;
            double* sH = b;
            double* sA = sH + nH;
            double* sf = sA + nA;
            dML = sf + nF;
            dgP = f ? dML + nML : nullptr;
            dL = dML + nML + nF;
            HIP_TRY(hipMemcpyAsync(sH, H, sizeof(double) * nH, hipMemcpyHostToDevice, h->stream));
            HIP_TRY(hipMemcpyAsync(sA, A, sizeof(double) * nA, hipMemcpyHostToDevice, h->stream));
            if (f) HIP_TRY(hipMemcpyAsync(sf, f, sizeof(double) * nF, hipMemcpyHostToDevice, h->stream));
            dH = sH;
            dA = sA;
            df = f ? sf : nullptr;
        }
        if (shared) {
            const size_t wb = gpad::precompute_work_bytes(n, m, fchunk, 1);
            if ((rc = work.ensure(wb + (f ? sizeof(double) * (size_t)n * n : 0)))) return rc;
            double* Hinv = f ? (double*)((char*)work.p + wb) : nullptr;
            HIP_TRY(gpad::launch_precompute(n, m, fchunk, dH, 0, dA, 0, nullptr, 0, (double*)work.p, dML, Hinv, dL, 0, 1,
                                            h->stream));
            if (f) HIP_TRY(gpad::launch_apply_inv(n, batch, Hinv, df, dgP, h->stream));
        } else {
            const size_t per = gpad::precompute_work_bytes(n, m, fchunk, 1);
            int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)batch, ((size_t)1 << 30) / per));
            chunk = std::min(chunk, 4 * h->num_cus);
            if ((rc = work.ensure(per * chunk))) return rc;
            for (int b0 = 0; b0 < batch; b0 += chunk) {
                const int cnt = std::min(chunk, batch - b0);
                HIP_TRY(gpad::launch_precompute(n, m, fchunk, dH, (long long)n * n, dA, (long long)m * n, df, n,
                                                (double*)work.p, dML, dgP, dL, b0, cnt, h->stream));
            }
        }
        if (host) {
            HIP_TRY(hipMemcpyAsync(ML, dML, sizeof(double) * nML, hipMemcpyDeviceToHost, h->stream));
            if (f) HIP_TRY(hipMemcpyAsync(gP, dgP, sizeof(double) * nF, hipMemcpyDeviceToHost, h->stream));
            HIP_TRY(hipMemcpyAsync(L, dL, sizeof(double) * nmat, hipMemcpyDeviceToHost, h->stream));
        }
        HIP_TRY(hipStreamSynchronize(h->stream));
        return GPAD_OK;
    });
}

extern "C" int gpad_setup_plant(gpad_handle_t h, int nx, int nu, const void* PM, const void* M0,
                                const void* Pg, const void* g0, const void* A, const void* B) {
    return gpad::abi_guard("gpad_setup_plant", [&]() -> int {
        if (!h) return fail(GPAD_ERR_INVALID, "gpad_setup_plant: null handle");
        if (!h->ready) return fail(GPAD_ERR_NOT_SETUP, "gpad_setup_plant: call gpad_setup first");
        if (nx <= 0 || nu < 0 || !PM || !Pg) return fail(GPAD_ERR_INVALID, "gpad_setup_plant: bad arguments");
        if ((A == nullptr) != (B == nullptr) || (A && nu == 0))
            return fail(GPAD_ERR_INVALID, "gpad_setup_plant: give A and B together (nu >= 1)");
        if (nu > h->dims.n) return fail(GPAD_ERR_INVALID, "gpad_setup_plant: nu > n");
        HIP_TRY(hipSetDevice(h->device));
        const int n = h->dims.n, m = h->dims.m;
        const size_t es = esize(h->dims.dtype);
        const PlantOffsets o = plant_offsets(n, m, nx, nu);
        int rc;
        if ((rc = h->plant.ensure(es * o.total))) return rc;
        char* base = (char*)h->plant.p;
        const hipMemcpyKind kind = h->dims.memory == GPAD_MEM_HOST ? hipMemcpyHostToDevice
                                                                    : hipMemcpyDeviceToDevice;
        auto put = [&](size_t off, const void* src, size_t elems) -> int {
            if (!src || elems == 0) return GPAD_OK;
            HIP_TRY(hipMemcpyAsync(base + es * off, src, es * elems, kind, h->stream));
            return GPAD_OK;
        };
        if ((rc = put(o.PM, PM, (size_t)n * nx)) || (rc = put(o.M0, M0, n)) ||
            (rc = put(o.Pg, Pg, (size_t)m * nx)) || (rc = put(o.g0, g0, m)) ||
            (rc = put(o.A, A, (size_t)nx * nx)) || (rc = put(o.B, B, (size_t)nx * nu)))
            return rc;
        HIP_TRY(hipStreamSynchronize(h->stream));
        h->nx = nx;
        h->nu = nu;
        h->has_M0 = M0 != nullptr;
        h->has_g0 = g0 != nullptr;
        h->plant_dyn = A != nullptr;
        h->plant_ready = true;
        h->plant_n = n;
        h->plant_m = m;
        h->plant_dtype = h->dims.dtype;
        return GPAD_OK;
    });
}

template <typename T>
static int state_typed(gpad_handle_t h, T* x, T* z, T* y, int steps, int N, double tol, int warm,
                       T* xs, T* us, gpad_stats_t* st) {
    // steps == 0: one solve at x (gpad_run_state); steps >= 1: closed loop (gpad_closed_loop)
    const gpad_dims_t& d = h->dims;
    const int n = d.n, m = d.m, batch = d.batch, nx = h->nx, nu = h->nu;
    const bool loop = steps > 0;
    const int nsolve = loop ? steps : 1;
    int rc = ensure_schedule(h, N, nullptr, nullptr);
    if (rc) return rc;
    if ((rc = h->counters.ensure(sizeof(int) * 2 * (size_t)batch * nsolve))) return rc;
    const bool host = d.memory == GPAD_MEM_HOST;
    const size_t zn = (size_t)batch * n, yn = (size_t)batch * m, xn = (size_t)batch * nx;
    const size_t xsn = loop && xs ? (size_t)steps * xn : 0, usn = loop && us ? (size_t)steps * batch * nu : 0;
    // workspace: M(x) | g(x) | x ping | x pong | (host) z | y | xs | us
    size_t elems = zn + yn + 2 * xn;
    if (host) elems += zn + yn + xsn + usn;
    if ((rc = h->state.ensure(sizeof(T) * elems))) return rc;
    T* Mx = (T*)h->state.p;
    T* gx = Mx + zn;
    T* xa = gx + yn;
    T* xb = xa + xn;
    T *dz = z, *dy = y, *dxs = xs, *dus = us;
    if (host) {
        dz = xb + xn;
        dy = dz + zn;
        dxs = xsn ? dy + yn : nullptr;
        dus = usn ? dy + yn + xsn : nullptr;
    }
    const hipMemcpyKind in_kind = host ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    const hipMemcpyKind out_kind = host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    HIP_TRY(hipMemcpyAsync(xa, x, sizeof(T) * xn, in_kind, h->stream));
    if (host && (!loop || warm)) {
        HIP_TRY(hipMemcpyAsync(dz, z, sizeof(T) * zn, hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipMemcpyAsync(dy, y, sizeof(T) * yn, hipMemcpyHostToDevice, h->stream));
    }
    const PlantOffsets o = plant_offsets(n, m, nx, nu);
    const T* P = (const T*)h->plant.p;
    int* counters = (int*)h->counters.p;
    int kernel = 0;
    const double margin = sizeof(T) == sizeof(float) ? gpad::ViolMargin<float>::value : gpad::ViolMargin<double>::value;
    if ((rc = reset_status(h, tol, margin))) return rc;  // g(x) unscaled: margin * L * (1/L)
    HIP_TRY(hipEventRecord(h->ev0, h->stream));
    T* xc = xa;
    T* xnext = xb;
    for (int t = 0; t < nsolve; ++t) {
        HIP_TRY(gpad::launch_affine2<T>(P + o.PM, h->has_M0 ? P + o.M0 : nullptr, n, Mx, P + o.Pg,
                                        h->has_g0 ? P + o.g0 : nullptr, m, gx, xc, nx, batch, h->stream));
        if (loop && !warm) {  // acceldualgrad.m:16-17: every MPC step starts from z = y = 0
            HIP_TRY(hipMemsetAsync(dz, 0, sizeof(T) * zn, h->stream));
            HIP_TRY(hipMemsetAsync(dy, 0, sizeof(T) * yn, h->stream));
        }
        int* it = counters + 2 * (size_t)batch * t;
        if ((rc = launch_solve<T>(h, dz, dy, Mx, gx, N, tol, false, it, it + batch, &kernel)))
            return rc;
        if (loop) {  // gpad.m:91-94: u = z*(1:nu); x <- A x + B u
            HIP_TRY(gpad::launch_plant_step<T>(P + o.A, P + o.B, xc, dz, n, xnext, nx, nu, batch,
                                               dxs ? dxs + (size_t)t * xn : nullptr,
                                               dus ? dus + (size_t)t * batch * nu : nullptr, h->stream));
            std::swap(xc, xnext);
        }
    }
    HIP_TRY(hipEventRecord(h->ev1, h->stream));
    h->timed = true;
    h->last_kernel = kernel;
    h->last_batch = batch;
    h->last_steps = nsolve;
    if (loop) HIP_TRY(hipMemcpyAsync(x, xc, sizeof(T) * xn, out_kind, h->stream));
    if (host) {
        HIP_TRY(hipMemcpyAsync(z, dz, sizeof(T) * zn, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipMemcpyAsync(y, dy, sizeof(T) * yn, hipMemcpyDeviceToHost, h->stream));
        if (xsn) HIP_TRY(hipMemcpyAsync(xs, dxs, sizeof(T) * xsn, hipMemcpyDeviceToHost, h->stream));
        if (usn) HIP_TRY(hipMemcpyAsync(us, dus, sizeof(T) * usn, hipMemcpyDeviceToHost, h->stream));
        if (!st) return gpad_sync(h);
    }
    if (st) return collect_stats(h, st);
    return GPAD_OK;
}

static int state_impl(gpad_handle_t h, void* x, void* z, void* y, int steps, int N, double tol, int warm,
                      void* xs, void* us, gpad_stats_t* st, const char* where) {
    if (!h) return fail(GPAD_ERR_INVALID, std::string(where) + ": null handle");
    if (!h->ready) return fail(GPAD_ERR_NOT_SETUP, std::string(where) + ": call gpad_setup first");
    if (!h->plant_ready || h->plant_n != h->dims.n || h->plant_m != h->dims.m ||
        h->plant_dtype != h->dims.dtype)
        return fail(GPAD_ERR_NOT_SETUP, std::string(where) + ": call gpad_setup_plant after gpad_setup");
    if (steps > 0 && !h->plant_dyn)
        return fail(GPAD_ERR_NOT_SETUP, std::string(where) + ": plant bound without A, B");
    if (!x || !z || !y) return fail(GPAD_ERR_INVALID, std::string(where) + ": null vector");
    if (N < 0 || steps < 0) return fail(GPAD_ERR_INVALID, std::string(where) + ": N, steps must be >= 0");
    if (!(tol <= 0.0) && !std::isfinite(tol)) return fail(GPAD_ERR_INVALID, std::string(where) + ": bad tol");
    HIP_TRY(hipSetDevice(h->device));
    if (h->dims.dtype == GPAD_DTYPE_F64)
        return state_typed<double>(h, (double*)x, (double*)z, (double*)y, steps, N, tol, warm, (double*)xs,
                                   (double*)us, st);
    return state_typed<float>(h, (float*)x, (float*)z, (float*)y, steps, N, tol, warm, (float*)xs,
                              (float*)us, st);
}

extern "C" {

int gpad_run_state(gpad_handle_t h, const void* x, void* z0, void* y0, int N, double tol,
                   gpad_stats_t* st) {
    return gpad::abi_guard("gpad_run_state", [&]() -> int {
        return state_impl(h, const_cast<void*>(x), z0, y0, 0, N, tol, 1, nullptr, nullptr, st,
                          "gpad_run_state");
    });
}

int gpad_closed_loop(gpad_handle_t h, void* x, void* z, void* y, int steps, int N, double tol, int warm,
                     void* xs, void* us, gpad_stats_t* st) {
    return gpad::abi_guard("gpad_closed_loop", [&]() -> int {
        if (steps == 0) return GPAD_OK;
        return state_impl(h, x, z, y, steps, N, tol, warm, xs, us, st, "gpad_closed_loop");
    });
}

// ---- per-step entry points ---------------------------------------------------------------
int gpad_step1_extrapolate(gpad_handle_t h, const float* y, const float* ym1, float* w, float beta,
                           int m) {
    return gpad::abi_guard("gpad_step1_extrapolate", [&]() -> int {
        if (!h || !y || !ym1 || !w || m < 0) return fail(GPAD_ERR_INVALID, "gpad_step1: bad arguments");
        if (m == 0) return GPAD_OK;
        HIP_TRY(hipSetDevice(h->device));
        HIP_TRY(gpad::launch_step1(y, ym1, w, beta, m, h->stream));
        return GPAD_OK;
    });
}

int gpad_step2_primal(gpad_handle_t h, const float* MGneg, const float* w, const float* gP,
                      float* zhat, int n, int m) {
    return gpad::abi_guard("gpad_step2_primal", [&]() -> int {
        if (!h || !MGneg || !w || !gP || !zhat || n <= 0 || m <= 0)
            return fail(GPAD_ERR_INVALID, "gpad_step2: bad arguments");
        if ((size_t)m * sizeof(float) > 64 * 1024) return fail(GPAD_ERR_UNSUPPORTED, "gpad_step2: m too large");
        HIP_TRY(hipSetDevice(h->device));
        HIP_TRY(gpad::launch_step2(MGneg, w, gP, zhat, n, m, h->stream));
        return GPAD_OK;
    });
}

int gpad_step2_primal_flat(gpad_handle_t h, const float* MGf, const float* w, const float* gP,
                           float* zhat, int N, int n_u, int m) {
    return gpad::abi_guard("gpad_step2_primal_flat", [&]() -> int {
        if (!h || !MGf || !w || !gP || !zhat || N <= 0 || n_u <= 0 || m < 4 * n_u * N)
            return fail(GPAD_ERR_INVALID, "gpad_step2_flat: bad arguments");
        HIP_TRY(hipSetDevice(h->device));
        HIP_TRY(gpad::launch_step2_flat(MGf, w, gP, zhat, N, n_u, m, h->stream));
        return GPAD_OK;
    });
}

int gpad_step4_project_flat(gpad_handle_t h, const float* GLf, float* yp1, const float* w,
                            const float* pD, const float* zhat, int N, int n_u, int m) {
    return gpad::abi_guard("gpad_step4_project_flat", [&]() -> int {
        if (!h || !GLf || !yp1 || !w || !pD || !zhat || N <= 0 || n_u <= 0 || m < 4 * n_u * N)
            return fail(GPAD_ERR_INVALID, "gpad_step4_flat: bad arguments");
        HIP_TRY(hipSetDevice(h->device));
        HIP_TRY(gpad::launch_step4_flat(GLf, yp1, w, pD, zhat, N, n_u, m, h->stream));
        return GPAD_OK;
    });
}

int gpad_step3_average(gpad_handle_t h, float theta, const float* zm1, const float* zhat, float* z,
                       int n) {
    return gpad::abi_guard("gpad_step3_average", [&]() -> int {
        if (!h || !zm1 || !zhat || !z || n < 0) return fail(GPAD_ERR_INVALID, "gpad_step3: bad arguments");
        if (n == 0) return GPAD_OK;
        HIP_TRY(hipSetDevice(h->device));
        HIP_TRY(gpad::launch_step3(theta, zm1, zhat, z, n, h->stream));
        return GPAD_OK;
    });
}

int gpad_step4_project(gpad_handle_t h, const float* GL, float* yp1, const float* w,
                       const float* pD, const float* zhat, int n, int m) {
    return gpad::abi_guard("gpad_step4_project", [&]() -> int {
        if (!h || !GL || !yp1 || !w || !pD || !zhat || n <= 0 || m <= 0)
            return fail(GPAD_ERR_INVALID, "gpad_step4: bad arguments");
        if ((size_t)n * sizeof(float) > 64 * 1024) return fail(GPAD_ERR_UNSUPPORTED, "gpad_step4: n too large");
        HIP_TRY(hipSetDevice(h->device));
        HIP_TRY(gpad::launch_step4(GL, yp1, w, pD, zhat, n, m, h->stream));
        return GPAD_OK;
    });
}

}  // extern "C"
