// gpad_group.cpp -- several devices from one C caller: instance-sharded solves with an RCCL
// scatter/gather (north_star: "partition across the 8 GPUs of one node by
// sharding independent MPC problem instances with a single RCCL gather of solutions").
//
// A group owns one libgpad handle and one HIP stream per device and, when the devices are
// distinct, one RCCL communicator clique over them (ncclCommInitAll: single process, one rank
// per device -- the reference's caller is a single C process, main.cu:79-203).  The batch is
// split into contiguous shards (sizes differ by at most one, larger first, as
// gpad_mpc/parallel.shard_range).  Per run there is no communication between the shards'
// solves; the data movement is:
//   host memory   : each device copies its own shard in and its solution out (no collective)
//   device memory : the caller's buffers live on devices[0] (the root); one grouped
//                   ncclSend/ncclRecv moves every non-root shard of (M, g, z0, y0) out, and one
//                   more brings (z*, y*) back into the caller's root buffers.  Shared matrices are
//                   broadcast once at setup (ncclBroadcast), per-instance matrices sent per shard.
// A device listed twice (one GPU standing in for several, e.g. the 1-GPU test box) has no RCCL
// clique (RCCL refuses duplicate devices): the same moves are then peer copies
// (hipMemcpyPeerAsync), ordered by events exactly where the RCCL calls are.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>  // types only: librccl is loaded on first use (current_rccl() below), not linked

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gpad.h"
#include "gpad_abi.h"
#include "gpad_internal.h"

namespace {

int gfail(int code, const std::string& msg) { return gpad::set_last_error(code, msg); }

#define G_HIP(expr)                                                                                   \
    do {                                                                                              \
        hipError_t _e = (expr);                                                                       \
        if (_e != hipSuccess)                                                                         \
            return gfail(_e == hipErrorOutOfMemory ? GPAD_ERR_NOMEM : GPAD_ERR_HIP,                   \
                         std::string(#expr) + ": " + hipGetErrorString(_e));                          \
    } while (0)
// RCCL entry points, resolved from librccl on the first group over distinct devices, so that
// single-GPU users of libgpad (gpad_solve, the handle API) never need RCCL installed.  Without it a
// group falls back to the peer-copy transport (gpad_group_transport reports which).
// gpad_group_rccl_library swaps the library (tests: a stub that moves the same bytes with HIP copies
// and accepts a repeated device, so the RCCL branch runs with several ranks on a one-GPU box); a
// group keeps the entry points it was created with.
struct Rccl {
    bool ok = false;
    bool force = false;  // RCCL transport even for a repeated device (gpad_group_rccl_library)
    std::string path;    // (empty: the default librccl)
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

std::shared_ptr<const Rccl> load_rccl(const std::string& path, bool force) {
    auto r = std::make_shared<Rccl>();
    r->path = path;
    void* lib = nullptr;
    if (!path.empty()) {
        lib = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    } else {
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((lib = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
    }
    if (!lib) return r;  // (never dlclose'd: groups created from it may outlive a swap)
    auto sym = [&](auto& fn, const char* name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(lib, name));
        return fn != nullptr;
    };
    r->ok = sym(r->CommInitAll, "ncclCommInitAll") && sym(r->CommDestroy, "ncclCommDestroy") &&
            sym(r->GroupStart, "ncclGroupStart") && sym(r->GroupEnd, "ncclGroupEnd") && sym(r->Send, "ncclSend") &&
            sym(r->Recv, "ncclRecv") && sym(r->Broadcast, "ncclBroadcast") &&
            sym(r->GetErrorString, "ncclGetErrorString");
    r->force = r->ok && force;
    return r;
}

std::mutex g_rccl_mu;
std::shared_ptr<const Rccl> g_rccl;  // loaded on first use (default librccl), or set by gpad_group_rccl_library
unsigned g_rccl_gen = 0;             // bumped by every gpad_group_rccl_library (the sharded cache re-creates)

std::shared_ptr<const Rccl> current_rccl(unsigned* gen = nullptr) {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!g_rccl) g_rccl = load_rccl(std::string(), false);
    if (gen) *gen = g_rccl_gen;
    return g_rccl;
}

#define G_NCCL(expr)                                                                                  \
    do {                                                                                              \
        ncclResult_t _r = g->r->expr;                                                                 \
        if (_r != ncclSuccess)                                                                        \
            return gfail(GPAD_ERR_HIP, std::string("nccl" #expr) + ": " + g->r->GetErrorString(_r));   \
    } while (0)

size_t esz(int dtype) { return dtype == GPAD_DTYPE_F64 ? sizeof(double) : sizeof(float); }

}  // namespace

struct gpad_group_s {
    int ndev = 0;
    std::vector<int> dev;
    std::vector<gpad_handle_t> h;
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> ev;      // one per device: ordering of the peer-copy transport
    std::vector<ncclComm_t> comm;    // empty: peer-copy transport (a device listed twice)
    std::shared_ptr<const Rccl> r;   // the RCCL entry points the clique was created with
    gpad_dims_t dims{};              // the whole batch
    double L = 0.0;
    bool ready = false;
    std::vector<int> start, count;   // shard of device d: [start, start + count)
    std::vector<void*> vec;          // per device: M | g | z | y of its shard (device memory)
    std::vector<size_t> vec_bytes;
    std::vector<void*> mat;          // per device: raw ML | G before packing
    std::vector<size_t> mat_bytes;
    hipStream_t caller = nullptr;    // the caller's stream on devices[0] (gpad_group_set_stream;
                                     // NULL = the device's null stream)
    hipEvent_t caller_ev = nullptr;  // recorded on it before the group touches device buffers
};

namespace {

int release(gpad_group_s* g) {
    for (int d = 0; d < g->ndev; ++d) {
        (void)hipSetDevice(g->dev[d]);
        if (d < (int)g->st.size() && g->st[d]) (void)hipStreamSynchronize(g->st[d]);
        if (d < (int)g->h.size() && g->h[d]) gpad_destroy(g->h[d]);
        if (d < (int)g->vec.size() && g->vec[d]) (void)hipFree(g->vec[d]);
        if (d < (int)g->mat.size() && g->mat[d]) (void)hipFree(g->mat[d]);
        if (d < (int)g->ev.size() && g->ev[d]) (void)hipEventDestroy(g->ev[d]);
        if (d < (int)g->st.size() && g->st[d]) (void)hipStreamDestroy(g->st[d]);
    }
    if (g->caller_ev) {
        (void)hipSetDevice(g->dev[0]);
        (void)hipEventDestroy(g->caller_ev);
    }
    for (ncclComm_t c : g->comm) (void)g->r->CommDestroy(c);
    delete g;
    return GPAD_OK;
}

int ensure(gpad_group_s* g, std::vector<void*>& bufs, std::vector<size_t>& sizes, int d, size_t want) {
    if (sizes[d] >= want && bufs[d]) return GPAD_OK;
    G_HIP(hipSetDevice(g->dev[d]));
    if (bufs[d]) (void)hipFree(bufs[d]);
    bufs[d] = nullptr;
    sizes[d] = 0;
    if (want == 0) return GPAD_OK;
    G_HIP(hipMalloc(&bufs[d], want));
    sizes[d] = want;
    return GPAD_OK;
}

// Root -> device d moves: (dst on device d, src on the root) pairs, all in one RCCL group (or
// peer copies on the root stream, with every destination stream waiting on it).
struct Move {
    int d;
    void* dst;
    const void* src;
    size_t bytes;
};

int scatter(gpad_group_s* g, const std::vector<Move>& mv) {
    if (mv.empty()) return GPAD_OK;
    if (!g->comm.empty()) {
        G_NCCL(GroupStart());
        for (const Move& x : mv) {
            G_NCCL(Send(x.src, x.bytes, ncclChar, x.d, g->comm[0], g->st[0]));
            G_NCCL(Recv(x.dst, x.bytes, ncclChar, 0, g->comm[x.d], g->st[x.d]));
        }
        G_NCCL(GroupEnd());
        return GPAD_OK;
    }
    G_HIP(hipSetDevice(g->dev[0]));
    for (const Move& x : mv)
        G_HIP(hipMemcpyPeerAsync(x.dst, g->dev[x.d], x.src, g->dev[0], x.bytes, g->st[0]));
    G_HIP(hipEventRecord(g->ev[0], g->st[0]));
    for (int d = 1; d < g->ndev; ++d) {
        G_HIP(hipSetDevice(g->dev[d]));
        G_HIP(hipStreamWaitEvent(g->st[d], g->ev[0], 0));
    }
    return GPAD_OK;
}

// Device d -> root moves (dst on the root, src on device d): the gather of the solutions.
int gather(gpad_group_s* g, const std::vector<Move>& mv) {
    if (mv.empty()) return GPAD_OK;
    if (!g->comm.empty()) {
        G_NCCL(GroupStart());
        for (const Move& x : mv) {
            G_NCCL(Send(x.src, x.bytes, ncclChar, 0, g->comm[x.d], g->st[x.d]));
            G_NCCL(Recv(x.dst, x.bytes, ncclChar, x.d, g->comm[0], g->st[0]));
        }
        G_NCCL(GroupEnd());
        return GPAD_OK;
    }
    for (int d = 1; d < g->ndev; ++d) {  // the root copies once every shard's solve is done
        G_HIP(hipSetDevice(g->dev[d]));
        G_HIP(hipEventRecord(g->ev[d], g->st[d]));
        G_HIP(hipSetDevice(g->dev[0]));
        G_HIP(hipStreamWaitEvent(g->st[0], g->ev[d], 0));
    }
    G_HIP(hipSetDevice(g->dev[0]));
    for (const Move& x : mv)
        G_HIP(hipMemcpyPeerAsync(x.dst, g->dev[0], x.src, g->dev[x.d], x.bytes, g->st[0]));
    return GPAD_OK;
}

// Device-memory callers produce their buffers on their own stream of devices[0]; the group's
// streams are non-blocking, so every one of them first waits for the work queued there so far
// (else a producer kernel still in flight could race with the scatter or the root's solve).
int order_after_caller(gpad_group_s* g) {
    G_HIP(hipSetDevice(g->dev[0]));
    G_HIP(hipEventRecord(g->caller_ev, g->caller));
    for (int d = 0; d < g->ndev; ++d) {
        G_HIP(hipSetDevice(g->dev[d]));
        G_HIP(hipStreamWaitEvent(g->st[d], g->caller_ev, 0));
    }
    return GPAD_OK;
}

int sync_all(gpad_group_s* g) {
    for (int d = 0; d < g->ndev; ++d) {
        G_HIP(hipSetDevice(g->dev[d]));
        G_HIP(hipStreamSynchronize(g->st[d]));
    }
    return GPAD_OK;
}

}  // namespace

extern "C" {

int gpad_group_create(gpad_group_t* out, int ndev, const int* devices) {
    return gpad::abi_guard("gpad_group_create", [&]() -> int {
        if (!out || ndev <= 0 || !devices) return gfail(GPAD_ERR_INVALID, "gpad_group_create: bad arguments");
        *out = nullptr;
        int visible = 0;
        if (hipGetDeviceCount(&visible) != hipSuccess || visible <= 0)
            return gfail(GPAD_ERR_NO_DEVICE, "gpad_group_create: no HIP device visible");
        for (int d = 0; d < ndev; ++d)
            if (devices[d] < 0 || devices[d] >= visible)
                return gfail(GPAD_ERR_INVALID, "gpad_group_create: bad device index");
        auto* g = new gpad_group_s;
        g->ndev = ndev;
        g->dev.assign(devices, devices + ndev);
        g->h.assign(ndev, nullptr);
        g->st.assign(ndev, nullptr);
        g->ev.assign(ndev, nullptr);
        g->vec.assign(ndev, nullptr);
        g->vec_bytes.assign(ndev, 0);
        g->mat.assign(ndev, nullptr);
        g->mat_bytes.assign(ndev, 0);
        for (int d = 0; d < ndev; ++d) {
            int rc;
            if (hipSetDevice(g->dev[d]) != hipSuccess || hipStreamCreateWithFlags(&g->st[d], hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&g->ev[d], hipEventDisableTiming) != hipSuccess) {
                release(g);
                return gfail(GPAD_ERR_HIP, "gpad_group_create: stream/event creation failed");
            }
            if ((rc = gpad_create(&g->h[d], g->dev[d], g->st[d]))) {
                release(g);
                return rc;
            }
        }
        if (hipSetDevice(g->dev[0]) != hipSuccess ||
            hipEventCreateWithFlags(&g->caller_ev, hipEventDisableTiming) != hipSuccess) {
            release(g);
            return gfail(GPAD_ERR_HIP, "gpad_group_create: event creation failed");
        }
        std::vector<int> sorted(g->dev);
        std::sort(sorted.begin(), sorted.end());
        const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
        g->r = current_rccl();
        if ((distinct || g->r->force) && g->r->ok) {  // one RCCL clique, rank d on devices[d]
            g->comm.assign(ndev, nullptr);
            const ncclResult_t r = g->r->CommInitAll(g->comm.data(), ndev, g->dev.data());
            if (r != ncclSuccess) {
                g->comm.clear();
                release(g);
                return gfail(GPAD_ERR_HIP, std::string("ncclCommInitAll: ") + g->r->GetErrorString(r));
            }
        }
        *out = g;
        return GPAD_OK;
    });
}

int gpad_group_destroy(gpad_group_t g) {
    return gpad::abi_guard("gpad_group_destroy", [&]() -> int {
        if (!g) return GPAD_OK;
        return release(g);
    });
}

int gpad_group_rccl_library(const char* path, int force_rccl) {
    return gpad::abi_guard("gpad_group_rccl_library", [&]() -> int {
        auto r = load_rccl(path ? std::string(path) : std::string(), force_rccl != 0);
        {
            std::lock_guard<std::mutex> lk(g_rccl_mu);
            g_rccl = r;
            ++g_rccl_gen;
        }
        if (!r->ok)
            return gfail(GPAD_ERR_UNSUPPORTED, std::string("gpad_group_rccl_library: cannot load the RCCL entry points from ") +
                                                   (path ? path : "librccl") + " (groups use peer copies)");
        return GPAD_OK;
    });
}

int gpad_group_transport(gpad_group_t g) {
    return gpad::abi_guard("gpad_group_transport", [&]() -> int {
        if (!g) return gfail(GPAD_ERR_INVALID, "gpad_group_transport: null group");
        return g->comm.empty() ? GPAD_GROUP_PEER : GPAD_GROUP_RCCL;
    });
}

int gpad_group_set_stream(gpad_group_t g, void* hip_stream) {
    return gpad::abi_guard("gpad_group_set_stream", [&]() -> int {
        if (!g) return gfail(GPAD_ERR_INVALID, "gpad_group_set_stream: null group");
        g->caller = static_cast<hipStream_t>(hip_stream);
        return GPAD_OK;
    });
}

int gpad_group_setup(gpad_group_t g, const gpad_dims_t* dims, const void* ML, const void* G, double L) {
    return gpad::abi_guard("gpad_group_setup", [&]() -> int {
        if (!g || !dims || !ML || !G) return gfail(GPAD_ERR_INVALID, "gpad_group_setup: bad arguments");
        if (dims->batch < 1 || dims->n <= 0 || dims->m <= 0)
            return gfail(GPAD_ERR_INVALID, "gpad_group_setup: dims: n, m, batch must be positive");
        g->ready = false;
        const int nd = g->ndev, B = dims->batch;
        g->start.assign(nd, 0);
        g->count.assign(nd, 0);
        for (int d = 0, s = 0; d < nd; ++d) {  // contiguous shards, larger first
            g->count[d] = B / nd + (d < B % nd ? 1 : 0);
            g->start[d] = s;
            s += g->count[d];
        }
        const bool host = dims->memory == GPAD_MEM_HOST;
        const size_t es = esz(dims->dtype), nm = (size_t)dims->n * dims->m * es;
        std::vector<Move> mv;
        std::vector<const void*> mlp(nd), gp(nd);
        int rc;
        if (!host && (rc = order_after_caller(g))) return rc;
        for (int d = 0; d < nd; ++d) {
            const int c = std::max(g->count[d], 1);
            const size_t per = dims->shared ? nm : nm * (size_t)c;  // each of ML and G
            const size_t off = dims->shared ? 0 : nm * (size_t)g->start[d];
            if (g->count[d] == 0 && !dims->shared) {  // more devices than instances: an idle shard
                if ((rc = ensure(g, g->mat, g->mat_bytes, d, 2 * per))) return rc;
                G_HIP(hipSetDevice(g->dev[d]));
                G_HIP(hipMemsetAsync(g->mat[d], 0, 2 * per, g->st[d]));
                mlp[d] = g->mat[d];
                gp[d] = (char*)g->mat[d] + per;
                continue;
            }
            if (!host && d == 0) {  // the root's shard reads the caller's buffers in place
                mlp[d] = (const char*)ML + off;
                gp[d] = (const char*)G + off;
                continue;
            }
            if ((rc = ensure(g, g->mat, g->mat_bytes, d, 2 * per))) return rc;
            void* dml = g->mat[d];
            void* dg = (char*)g->mat[d] + per;
            mlp[d] = dml;
            gp[d] = dg;
            if (host) {
                G_HIP(hipSetDevice(g->dev[d]));
                G_HIP(hipMemcpyAsync(dml, (const char*)ML + off, per, hipMemcpyHostToDevice, g->st[d]));
                G_HIP(hipMemcpyAsync(dg, (const char*)G + off, per, hipMemcpyHostToDevice, g->st[d]));
            } else if (!dims->shared || g->comm.empty()) {
                mv.push_back({d, dml, (const char*)ML + off, per});
                mv.push_back({d, dg, (const char*)G + off, per});
            }
        }
        if (!host && dims->shared && !g->comm.empty() && nd > 1) {  // shared matrices: one broadcast each
            G_NCCL(GroupStart());
            for (int d = 0; d < nd; ++d) {
                G_NCCL(Broadcast(d == 0 ? ML : nullptr, const_cast<void*>(mlp[d]), nm, ncclChar, 0, g->comm[d], g->st[d]));
                G_NCCL(Broadcast(d == 0 ? G : nullptr, const_cast<void*>(gp[d]), nm, ncclChar, 0, g->comm[d], g->st[d]));
            }
            G_NCCL(GroupEnd());
        }
        if ((rc = scatter(g, mv))) return rc;
        for (int d = 0; d < nd; ++d) {  // pack on every device (each handle orders on its stream)
            gpad_dims_t dd = *dims;
            dd.batch = std::max(g->count[d], 1);
            dd.memory = GPAD_MEM_DEVICE;
            if ((rc = gpad_setup(g->h[d], &dd, mlp[d], gp[d], L))) return rc;
        }
        if ((rc = sync_all(g))) return rc;
        g->dims = *dims;
        g->L = L;
        g->ready = true;
        return GPAD_OK;
    });
}

int gpad_group_run(gpad_group_t g, void* z0, void* y0, const void* M, const void* gv, int N, double tol,
                   gpad_stats_t* st) {
    return gpad::abi_guard("gpad_group_run", [&]() -> int {
        if (!g) return gfail(GPAD_ERR_INVALID, "gpad_group_run: null group");
        if (!g->ready) return gfail(GPAD_ERR_NOT_SETUP, "gpad_group_run: call gpad_group_setup first");
        if (!z0 || !y0 || !M || !gv) return gfail(GPAD_ERR_INVALID, "gpad_group_run: null vector");
        const gpad_dims_t& D = g->dims;
        const bool host = D.memory == GPAD_MEM_HOST;
        const size_t es = esz(D.dtype), nb = (size_t)D.n * es, mb = (size_t)D.m * es;
        const int nd = g->ndev;
        std::vector<char*> Mp(nd), gp(nd), zp(nd), yp(nd);
        std::vector<Move> in, out;
        int rc;
        if (!host && (rc = order_after_caller(g))) return rc;
        for (int d = 0; d < nd; ++d) {
            const size_t c = (size_t)g->count[d], s0 = (size_t)g->start[d];
            if (!host && d == 0) {  // root shard in place
                Mp[d] = (char*)M;
                gp[d] = (char*)gv;
                zp[d] = (char*)z0;
                yp[d] = (char*)y0;
                continue;
            }
            if ((rc = ensure(g, g->vec, g->vec_bytes, d, std::max<size_t>(1, 2 * c * (nb + mb))))) return rc;
            Mp[d] = (char*)g->vec[d];
            gp[d] = Mp[d] + c * nb;
            zp[d] = gp[d] + c * mb;
            yp[d] = zp[d] + c * nb;
            if (c == 0) continue;
            if (host) {
                G_HIP(hipSetDevice(g->dev[d]));
                G_HIP(hipMemcpyAsync(Mp[d], (const char*)M + s0 * nb, c * nb, hipMemcpyHostToDevice, g->st[d]));
                G_HIP(hipMemcpyAsync(gp[d], (const char*)gv + s0 * mb, c * mb, hipMemcpyHostToDevice, g->st[d]));
                G_HIP(hipMemcpyAsync(zp[d], (const char*)z0 + s0 * nb, c * nb, hipMemcpyHostToDevice, g->st[d]));
                G_HIP(hipMemcpyAsync(yp[d], (const char*)y0 + s0 * mb, c * mb, hipMemcpyHostToDevice, g->st[d]));
            } else {
                in.push_back({d, Mp[d], (const char*)M + s0 * nb, c * nb});
                in.push_back({d, gp[d], (const char*)gv + s0 * mb, c * mb});
                in.push_back({d, zp[d], (const char*)z0 + s0 * nb, c * nb});
                in.push_back({d, yp[d], (const char*)y0 + s0 * mb, c * mb});
                out.push_back({d, (char*)z0 + s0 * nb, zp[d], c * nb});
                out.push_back({d, (char*)y0 + s0 * mb, yp[d], c * mb});
            }
        }
        if ((rc = scatter(g, in))) return rc;
        for (int d = 0; d < nd; ++d) {  // every shard's solve, asynchronous on its device's stream
            if (g->count[d] == 0) continue;
            if ((rc = gpad_run(g->h[d], zp[d], yp[d], Mp[d], gp[d], N, tol, nullptr))) return rc;
        }
        if ((rc = gather(g, out))) return rc;
        if (host) {
            for (int d = 0; d < nd; ++d) {
                const size_t c = (size_t)g->count[d], s0 = (size_t)g->start[d];
                if (c == 0) continue;
                G_HIP(hipSetDevice(g->dev[d]));
                G_HIP(hipMemcpyAsync((char*)z0 + s0 * nb, zp[d], c * nb, hipMemcpyDeviceToHost, g->st[d]));
                G_HIP(hipMemcpyAsync((char*)y0 + s0 * mb, yp[d], c * mb, hipMemcpyDeviceToHost, g->st[d]));
            }
        }
        if ((rc = sync_all(g))) return rc;
        for (int d = 0; d < nd; ++d)  // device-side failures of any shard fail the run (GPAD_ERR_DEVICE)
            if (g->count[d] > 0 && (rc = gpad_sync(g->h[d]))) return rc;
        if (st) {  // per-shard counters (host copies), aggregated; st->iters [batch] in global order
            gpad_stats_t tot{};
            for (int d = 0; d < nd; ++d) {
                if (g->count[d] == 0) continue;
                gpad_stats_t sd{};
                sd.iters = st->iters ? st->iters + g->start[d] : nullptr;
                sd.codes = st->codes ? st->codes + g->start[d] : nullptr;
                if ((rc = gpad_last_stats(g->h[d], &sd))) return rc;
                tot.iterations = std::max(tot.iterations, sd.iterations);
                tot.converged += sd.converged;
                tot.total_iterations += sd.total_iterations;
                tot.kernel = sd.kernel;
                tot.kernel_ms = std::max(tot.kernel_ms, sd.kernel_ms);
                tot.tol_floor = std::max(tot.tol_floor, sd.tol_floor);
                tot.flags |= sd.flags;
            }
            int* keep = st->iters;
            int* keep_codes = st->codes;
            *st = tot;
            st->iters = keep;
            st->codes = keep_codes;
        }
        return GPAD_OK;
    });
}

}  // extern "C"

// One group per thread and device list, kept between gpad_solve_sharded calls (communicator set-up
// is the expensive part).  Freed by gpad_release_cached(), never from a thread-exit destructor: at
// process exit that can run after the HIP / RCCL runtimes tore down (the OS reclaims it instead).
namespace {
struct ShardCache {
    gpad_group_t grp = nullptr;
    std::vector<int> devs;
    unsigned rccl_gen = 0;  // the RCCL configuration the group was created under
};
thread_local ShardCache t_shard_cache;
}  // namespace

void gpad::release_sharded_cache() {
    if (t_shard_cache.grp) gpad_group_destroy(t_shard_cache.grp);
    t_shard_cache.grp = nullptr;
    t_shard_cache.devs.clear();
}

extern "C" {

int gpad_solve_sharded(int ndev, const int* devices, void* z0, void* y0, const void* ML, const void* M,
                       const void* G, const void* g, int N, double L, double tol, const gpad_dims_t* dims,
                       gpad_stats_t* st) {
    return gpad::abi_guard("gpad_solve_sharded", [&]() -> int {
        ShardCache& cache = t_shard_cache;
        if (ndev <= 0 || !devices) return gfail(GPAD_ERR_INVALID, "gpad_solve_sharded: bad device list");
        std::vector<int> want(devices, devices + ndev);
        unsigned gen = 0;
        (void)current_rccl(&gen);
        if (!cache.grp || cache.devs != want || cache.rccl_gen != gen) {
            if (cache.grp) gpad_group_destroy(cache.grp);
            cache.grp = nullptr;
            int rc = gpad_group_create(&cache.grp, ndev, devices);
            if (rc) return rc;
            cache.devs = want;
            cache.rccl_gen = gen;
        }
        int rc = gpad_group_setup(cache.grp, dims, ML, G, L);
        if (rc) return rc;
        return gpad_group_run(cache.grp, z0, y0, M, g, N, tol, st);
    });
}

}  // extern "C"
