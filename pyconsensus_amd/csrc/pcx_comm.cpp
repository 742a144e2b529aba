// pcx_comm.cpp -- cross-rank exchange of the sharded single-matrix consensus.
//
// The reference has no distribution; these are the collectives of the
// row-sharded design: all-reduce SUM / MIN / MAX of u64 selection
// histograms and of the f64 covariance, all-gather of per-rank dd partial blocks.
//
//   * RCCL (one process per GPU over xGMI): ncclAllReduce / ncclAllGather on the
//     context's stream;
//   * group: virtual ranks as threads of one process (any devices), exchanging through
//     host memory in rank order -- the 1-GPU rehearsal of the multi-GPU path;
//   * custom: caller callbacks on host buffers (e.g. torch.distributed gloo).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "pcx_internal.h"
#include "pcx_sync.h"

namespace pcx {
namespace {

size_t dtype_size(int) { return 8; }

template <class T>
void reduce_into(T* acc, const T* x, int64_t n, int op) {
    for (int64_t i = 0; i < n; i++) {
        if (op == PCX_SUM)
            acc[i] = acc[i] + x[i];
        else if (op == PCX_MIN)
            acc[i] = x[i] < acc[i] ? x[i] : acc[i];
        else
            acc[i] = x[i] > acc[i] ? x[i] : acc[i];
    }
}

void host_reduce(void* acc, const void* x, int64_t n, int dtype, int op) {
    if (dtype == PCX_F64)
        reduce_into((double*)acc, (const double*)x, n, op);
    else
        reduce_into((uint64_t*)acc, (const uint64_t*)x, n, op);
}

int hip_err(hipError_t e, const char* what, std::string& err) {
    if (e == hipSuccess) return 0;
    err = std::string(what) + ": " + hipGetErrorString(e);
    return PCX_EHIP;
}

// ------------------------------------------------------------------ RCCL
// AbortOnce (pcx_sync.h): the handle, its bounded-wait abort and the overlap it may leave.
struct RcclComm : Comm {
    AbortOnce<ncclComm_t> handle;
    static constexpr int ABORT_WAIT_MS = 2000;
    ~RcclComm() override {
        if (ncclComm_t c = handle.h.exchange(nullptr)) ncclCommDestroy(c);
    }
    void abort() override {
        aborted = true;
        handle.abort([](ncclComm_t c) { ncclCommAbort(c); }, ABORT_WAIT_MS);
    }
    static ncclDataType_t dt(int d) { return d == PCX_F64 ? ncclFloat64 : ncclUint64; }
    static ncclRedOp_t op_of(int o) { return o == PCX_SUM ? ncclSum : (o == PCX_MIN ? ncclMin : ncclMax); }
    static constexpr int GONE = 1;  // (positive: never a PCX_ status)
    static int gone(std::string& err) {
        err = "RCCL communicator aborted after a failed call: recreate the context";
        return PCX_ECOMM;
    }
    int allreduce(void* buf, int64_t count, int dtype, int op, hipStream_t st, std::string& err) override {
        if (count <= 0) return 0;
        const int rc = handle.use(
            [&](ncclComm_t c) {
                ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, dt(dtype), op_of(op), c, st);
                if (r == ncclSuccess) return 0;
                err = std::string("ncclAllReduce: ") + ncclGetErrorString(r);
                return (int)PCX_ECOMM;
            },
            GONE);
        return rc == GONE ? gone(err) : rc;
    }
    int allgather(const void* send, void* recv, int64_t bytes, hipStream_t st, std::string& err) override {
        if (bytes <= 0) return 0;
        const int rc = handle.use(
            [&](ncclComm_t c) {
                ncclResult_t r = ncclAllGather(send, recv, (size_t)bytes, ncclUint8, c, st);
                if (r == ncclSuccess) return 0;
                err = std::string("ncclAllGather: ") + ncclGetErrorString(r);
                return (int)PCX_ECOMM;
            },
            GONE);
        return rc == GONE ? gone(err) : rc;
    }
    const char* kind() const override { return "rccl"; }
};

// ------------------------------------------------------------------ host-staged backends
struct StagedComm : Comm {
    std::vector<char> h0, h1;
    int stage_out(const void* dev, int64_t bytes, std::vector<char>& h, hipStream_t st, std::string& err) {
        if ((int64_t)h.size() < bytes) h.resize(bytes);
        int rc = hip_err(hipMemcpyAsync(h.data(), dev, bytes, hipMemcpyDeviceToHost, st), "exchange D2H", err);
        if (!rc) rc = hip_err(hipStreamSynchronize(st), "exchange sync", err);
        return rc;
    }
    int stage_in(void* dev, const void* h, int64_t bytes, hipStream_t st, std::string& err) {
        int rc = hip_err(hipMemcpyAsync(dev, h, bytes, hipMemcpyHostToDevice, st), "exchange H2D", err);
        if (!rc) rc = hip_err(hipStreamSynchronize(st), "exchange sync", err);
        return rc;
    }
};

struct GroupComm : StagedComm {
    pcx_group* g = nullptr;
    static int aborted(std::string& err) {
        err = "exchange aborted: another rank of the group failed";
        return PCX_ECOMM;
    }
    int allreduce(void* buf, int64_t count, int dtype, int op, hipStream_t st, std::string& err) override {
        if (count <= 0) return 0;
        const int64_t bytes = count * (int64_t)dtype_size(dtype);
        int rc = stage_out(buf, bytes, g->slot[rank], st, err);
        if (!g->barrier()) return aborted(err);
        if (rc == 0) {
            // every rank reduces in rank order: identical results everywhere
            std::vector<char>& acc = h1;
            if ((int64_t)acc.size() < bytes) acc.resize(bytes);
            memcpy(acc.data(), g->slot[0].data(), bytes);
            for (int w = 1; w < world; w++) host_reduce(acc.data(), g->slot[w].data(), count, dtype, op);
        }
        if (!g->barrier()) return aborted(err);
        if (rc == 0) rc = stage_in(buf, h1.data(), bytes, st, err);
        return rc;
    }
    int allgather(const void* send, void* recv, int64_t bytes, hipStream_t st, std::string& err) override {
        if (bytes <= 0) return 0;
        int rc = stage_out(send, bytes, g->slot[rank], st, err);
        if (!g->barrier()) return aborted(err);
        if (rc == 0) {
            if ((int64_t)h1.size() < bytes * world) h1.resize(bytes * world);
            for (int w = 0; w < world; w++) memcpy(h1.data() + (int64_t)w * bytes, g->slot[w].data(), bytes);
        }
        if (!g->barrier()) return aborted(err);
        if (rc == 0) rc = stage_in(recv, h1.data(), bytes * world, st, err);
        return rc;
    }
    const char* kind() const override { return "group"; }
};

struct CustomComm : StagedComm {
    pcx_comm_ops ops{};
    int allreduce(void* buf, int64_t count, int dtype, int op, hipStream_t st, std::string& err) override {
        if (count <= 0) return 0;
        const int64_t bytes = count * (int64_t)dtype_size(dtype);
        int rc = stage_out(buf, bytes, h0, st, err);
        if (rc) return rc;
        if (ops.allreduce(ops.user, h0.data(), count, dtype, op) != 0) {
            err = "custom allreduce callback failed";
            return PCX_ECOMM;
        }
        return stage_in(buf, h0.data(), bytes, st, err);
    }
    int allgather(const void* send, void* recv, int64_t bytes, hipStream_t st, std::string& err) override {
        if (bytes <= 0) return 0;
        int rc = stage_out(send, bytes, h0, st, err);
        if (rc) return rc;
        if ((int64_t)h1.size() < bytes * world) h1.resize(bytes * world);
        if (ops.allgather(ops.user, h0.data(), h1.data(), bytes) != 0) {
            err = "custom allgather callback failed";
            return PCX_ECOMM;
        }
        return stage_in(recv, h1.data(), bytes * world, st, err);
    }
    const char* kind() const override { return "custom"; }
};

}  // namespace

// The RCCL that serves libpcx's calls is whichever librccl the process loaded first: with
// torch imported, torch's bundled copy (2.26.x next to /opt/rocm's 2.27.x headers).
// libpcx calls only the version-2 core API (unique id, CommInitRank / InitAll, AllReduce,
// AllGather, CommAbort / Destroy, GetErrorString), whose signatures and 128-byte ncclUniqueId
// are fixed across 2.x; a runtime of another major version, or older than the 2.18 this was
// validated against, is refused with both versions named.
int rccl_version(int* runtime, int* compiled) {
    int v = 0;
    if (ncclGetVersion(&v) != ncclSuccess) v = 0;
    if (runtime) *runtime = v;
    if (compiled) *compiled = NCCL_VERSION_CODE;
    return v;
}

int rccl_check_version(std::string& err) {
    int rt = 0, ct = 0;
    rccl_version(&rt, &ct);
    const int rt_major = rt >= 10000 ? rt / 10000 : rt / 1000;
    const int ct_major = ct >= 10000 ? ct / 10000 : ct / 1000;
    if (rt_major != ct_major || rt < 21800) {
        err = "RCCL runtime " + std::to_string(rt) + " is incompatible with the headers libpcx was built against (" +
              std::to_string(ct) + "): need the same major version and >= 2.18 (version code 21800)";
        return PCX_ECOMM;
    }
    return 0;
}

int comm_rccl_unique_id(pcx_comm_id* out, std::string& err) {
    static_assert(sizeof(pcx_comm_id) == sizeof(ncclUniqueId), "pcx_comm_id mirrors ncclUniqueId");
    if (const int rc = rccl_check_version(err)) return rc;
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return PCX_ECOMM;
    }
    memcpy(out, &id, sizeof(id));
    return 0;
}

Comm* comm_rccl(int device, int world, int rank, const pcx_comm_id* id, std::string& err) {
    if (rccl_check_version(err)) return nullptr;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        err = std::string("hipSetDevice: ") + hipGetErrorString(e);
        return nullptr;
    }
    RcclComm* c = new (std::nothrow) RcclComm;
    if (!c) return nullptr;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t h = nullptr;
    ncclResult_t r = ncclCommInitRank(&h, world, uid, rank);
    if (r != ncclSuccess) {
        err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        delete c;
        return nullptr;
    }
    c->handle.h = h;
    c->world = world;
    c->rank = rank;
    return c;
}

int comm_rccl_all(int n, const int* devices, std::vector<Comm*>& out, std::string& err) {
    if (const int rc = rccl_check_version(err)) return rc;
    std::vector<ncclComm_t> comms(n, nullptr);
    ncclResult_t r = ncclCommInitAll(comms.data(), n, devices);
    if (r != ncclSuccess) {
        err = std::string("ncclCommInitAll: ") + ncclGetErrorString(r);
        return PCX_ECOMM;
    }
    for (int k = 0; k < n; k++) {
        RcclComm* c = new (std::nothrow) RcclComm;
        if (!c) {
            for (int j = k; j < n; j++) ncclCommDestroy(comms[j]);
            err = "out of host memory";
            return PCX_ENOMEM;
        }
        c->handle.h = comms[k];
        c->world = n;
        c->rank = k;
        out.push_back(c);
    }
    return 0;
}

pcx_group* group_create(int world) {
    if (world < 1) return nullptr;
    pcx_group* g = new (std::nothrow) pcx_group;
    if (!g) return nullptr;
    g->world = world;
    g->slot.resize(world);
    return g;
}

void group_destroy(pcx_group* g) { delete g; }

void group_abort(pcx_group* g) {
    if (g) g->abort();
}

void group_reset(pcx_group* g) {
    if (g) g->reset();
}

Comm* comm_group(pcx_group* g, int rank, std::string& err) {
    if (!g || rank < 0 || rank >= g->world) {
        err = "pcx_create_grouped: bad group or rank";
        return nullptr;
    }
    GroupComm* c = new (std::nothrow) GroupComm;
    if (!c) return nullptr;
    c->g = g;
    c->world = g->world;
    c->rank = rank;
    return c;
}

Comm* comm_custom(int world, int rank, const pcx_comm_ops* ops, std::string& err) {
    if (!ops || !ops->allreduce || !ops->allgather || world < 1 || rank < 0 || rank >= world) {
        err = "pcx_create_custom: bad ops / world / rank";
        return nullptr;
    }
    CustomComm* c = new (std::nothrow) CustomComm;
    if (!c) return nullptr;
    c->ops = *ops;
    c->world = world;
    c->rank = rank;
    return c;
}

}  // namespace pcx
