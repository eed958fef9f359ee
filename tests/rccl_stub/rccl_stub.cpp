// rccl_stub.cpp -- TEST INFRASTRUCTURE (never part of libgpad): the eight RCCL entry points libgpad's
// group transport binds (csrc/gpad_group.cpp, loaded through gpad_group_rccl_library), implemented
// with HIP copies so the RCCL branch of the grouped scatter / gather / broadcast runs with several
// ranks on a one-GPU box: a clique may list a device more than once (real RCCL refuses that).
//
// Semantics kept from NCCL: operations issued between ncclGroupStart / ncclGroupEnd are matched at
// the outermost ncclGroupEnd -- ncclSend(peer) on rank r with ncclRecv(from r) on rank peer (FIFO per
// pair, equal sizes), the k-th ncclBroadcast of every rank of a clique as one collective.  Each move
// is ordered like the real thing: the receiving stream waits for the sender's stream, copies, and the
// sending stream then waits for that copy (the send "completes" once the bytes landed).  Unmatched
// operations fail the group (ncclInvalidUsage).  rccl_stub_moves() counts the byte moves performed,
// so a test can prove the RCCL branch really moved data.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <memory>
#include <vector>

namespace {
struct Clique {
    int n = 0;
};
struct Op {
    int kind;  // 0 send, 1 recv, 2 broadcast
    const void* sbuf;
    void* rbuf;
    size_t bytes;
    int peer;  // send: to, recv: from, broadcast: root
    ncclComm_t comm;
    hipStream_t st;
    bool done;
};
thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;
std::atomic<long long> g_moves{0};

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}
}  // namespace

struct ncclComm {
    std::shared_ptr<Clique> clique;
    int rank;
    int dev;
};

namespace {
// dst on device dd (ordered on stream ds) <- src on device sd (stream ss)
ncclResult_t move(void* dst, int dd, hipStream_t ds, const void* src, int sd, hipStream_t ss, size_t bytes) {
    hipEvent_t e1 = nullptr, e2 = nullptr;
    if (hipSetDevice(sd) != hipSuccess || hipEventCreateWithFlags(&e1, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(e1, ss) != hipSuccess)
        return ncclUnhandledCudaError;
    if (hipSetDevice(dd) != hipSuccess || hipStreamWaitEvent(ds, e1, 0) != hipSuccess) return ncclUnhandledCudaError;
    const hipError_t c = dd == sd ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ds)
                                  : hipMemcpyPeerAsync(dst, dd, src, sd, bytes, ds);
    if (c != hipSuccess || hipEventCreateWithFlags(&e2, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(e2, ds) != hipSuccess)
        return ncclUnhandledCudaError;
    if (hipSetDevice(sd) != hipSuccess || hipStreamWaitEvent(ss, e2, 0) != hipSuccess) return ncclUnhandledCudaError;
    (void)hipEventDestroy(e1);  // (released once complete)
    (void)hipEventDestroy(e2);
    g_moves.fetch_add(1);
    return ncclSuccess;
}

ncclResult_t flush() {
    int dev0 = 0;
    (void)hipGetDevice(&dev0);
    std::vector<Op> ops;
    ops.swap(t_ops);
    ncclResult_t res = ncclSuccess;
    for (Op& s : ops) {  // point to point: each send with the first unmatched recv of its pair
        if (s.kind != 0) continue;
        for (Op& r : ops) {
            if (r.kind != 1 || r.done || r.comm->clique != s.comm->clique || r.comm->rank != s.peer ||
                r.peer != s.comm->rank)
                continue;
            if (r.bytes != s.bytes) return ncclInvalidUsage;
            if (s.bytes && (res = move(r.rbuf, r.comm->dev, r.st, s.sbuf, s.comm->dev, s.st, s.bytes)) != ncclSuccess)
                return res;
            r.done = s.done = true;
            break;
        }
        if (!s.done) return ncclInvalidUsage;
    }
    for (const Op& r : ops)
        if (r.kind == 1 && !r.done) return ncclInvalidUsage;
    // broadcasts: the k-th broadcast of each rank of a clique together
    for (size_t i = 0; i < ops.size(); ++i) {
        if (ops[i].kind != 2 || ops[i].done) continue;
        std::vector<Op*> coll;  // this collective: one op per rank, in issue order
        std::vector<int> seen(ops[i].comm->clique->n, 0);
        for (size_t j = i; j < ops.size(); ++j) {
            Op& o = ops[j];
            if (o.kind != 2 || o.done || o.comm->clique != ops[i].comm->clique || seen[o.comm->rank]) continue;
            seen[o.comm->rank] = 1;
            coll.push_back(&o);
        }
        if ((int)coll.size() != ops[i].comm->clique->n) return ncclInvalidUsage;
        Op* root = nullptr;
        for (Op* o : coll)
            if (o->comm->rank == o->peer) root = o;
        if (!root) return ncclInvalidArgument;
        for (Op* o : coll) {
            if (o->bytes != root->bytes || o->peer != root->peer) return ncclInvalidUsage;
            if (o->rbuf != root->sbuf && o->bytes &&
                (res = move(o->rbuf, o->comm->dev, o->st, root->sbuf, root->comm->dev, root->st, o->bytes)) != ncclSuccess)
                return res;
            o->done = true;
        }
    }
    (void)hipSetDevice(dev0);
    return ncclSuccess;
}

ncclResult_t issue(const Op& op) {
    if (!op.comm) return ncclInvalidArgument;
    t_ops.push_back(op);
    return t_depth == 0 ? flush() : ncclSuccess;
}
}  // namespace

extern "C" {

long long rccl_stub_moves(void) { return g_moves.load(); }

ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist) {
    if (!comm || ndev <= 0) return ncclInvalidArgument;
    auto c = std::make_shared<Clique>();
    c->n = ndev;
    for (int r = 0; r < ndev; ++r) comm[r] = new ncclComm{c, r, devlist ? devlist[r] : r};
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    ++t_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    return --t_depth == 0 ? flush() : ncclSuccess;
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    const size_t es = type_size(datatype);
    if (!es || !comm || peer < 0 || peer >= comm->clique->n) return ncclInvalidArgument;
    return issue(Op{0, sendbuff, nullptr, count * es, peer, comm, stream, false});
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    const size_t es = type_size(datatype);
    if (!es || !comm || peer < 0 || peer >= comm->clique->n) return ncclInvalidArgument;
    return issue(Op{1, nullptr, recvbuff, count * es, peer, comm, stream, false});
}

ncclResult_t ncclBroadcast(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, int root,
                           ncclComm_t comm, hipStream_t stream) {
    const size_t es = type_size(datatype);
    if (!es || !comm || root < 0 || root >= comm->clique->n) return ncclInvalidArgument;
    return issue(Op{2, sendbuff, recvbuff, count * es, root, comm, stream, false});
}

const char* ncclGetErrorString(ncclResult_t result) {
    switch (result) {
        case ncclSuccess: return "no error (rccl_stub)";
        case ncclUnhandledCudaError: return "unhandled HIP error (rccl_stub)";
        case ncclInvalidArgument: return "invalid argument (rccl_stub)";
        case ncclInvalidUsage: return "invalid usage: unmatched operation in a group (rccl_stub)";
        default: return "error (rccl_stub)";
    }
}

}  // extern "C"
