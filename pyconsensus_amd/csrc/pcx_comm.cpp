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
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "pcx_internal.h"

struct pcx_group {
    int world = 1;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t generation = 0;
    std::vector<std::vector<char>> slot;  // per rank host staging
    std::vector<char> result;             // reduced data (written by the last arriver)

    bool aborted = false;                 // a rank failed: every waiting and later exchange fails

    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return false;
        const int64_t g = generation;
        if (++arrived == world) {
            arrived = 0;
            generation++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != g || aborted; });
        }
        return !aborted;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

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
struct RcclComm : Comm {
    // the handle is swapped out atomically by abort(): ncclCommAbort runs exactly once even
    // when several failing worker threads abort the same communicator, and an exchange that
    // starts after the abort sees nullptr and fails instead of using a freed communicator
    std::atomic<ncclComm_t> comm{nullptr};
    ~RcclComm() override {
        if (ncclComm_t c = comm.exchange(nullptr)) ncclCommDestroy(c);
    }
    void abort() override {
        aborted = true;
        if (ncclComm_t c = comm.exchange(nullptr)) ncclCommAbort(c);
    }
    static ncclDataType_t dt(int d) { return d == PCX_F64 ? ncclFloat64 : ncclUint64; }
    static ncclRedOp_t op_of(int o) { return o == PCX_SUM ? ncclSum : (o == PCX_MIN ? ncclMin : ncclMax); }
    static int gone(std::string& err) {
        err = "RCCL communicator aborted after a failed call: recreate the context";
        return PCX_ECOMM;
    }
    int allreduce(void* buf, int64_t count, int dtype, int op, hipStream_t st, std::string& err) override {
        if (count <= 0) return 0;
        ncclComm_t c = comm.load();
        if (!c || aborted) return gone(err);
        ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, dt(dtype), op_of(op), c, st);
        if (r != ncclSuccess) {
            err = std::string("ncclAllReduce: ") + ncclGetErrorString(r);
            return PCX_ECOMM;
        }
        return 0;
    }
    int allgather(const void* send, void* recv, int64_t bytes, hipStream_t st, std::string& err) override {
        if (bytes <= 0) return 0;
        ncclComm_t c = comm.load();
        if (!c || aborted) return gone(err);
        ncclResult_t r = ncclAllGather(send, recv, (size_t)bytes, ncclUint8, c, st);
        if (r != ncclSuccess) {
            err = std::string("ncclAllGather: ") + ncclGetErrorString(r);
            return PCX_ECOMM;
        }
        return 0;
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

int comm_rccl_unique_id(pcx_comm_id* out, std::string& err) {
    static_assert(sizeof(pcx_comm_id) == sizeof(ncclUniqueId), "pcx_comm_id mirrors ncclUniqueId");
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
    c->comm = h;
    c->world = world;
    c->rank = rank;
    return c;
}

int comm_rccl_all(int n, const int* devices, std::vector<Comm*>& out, std::string& err) {
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
        c->comm = comms[k];
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
    if (!g) return;
    std::lock_guard<std::mutex> lk(g->mu);
    g->aborted = false;
    g->arrived = 0;
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
