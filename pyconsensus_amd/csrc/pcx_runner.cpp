// pcx_runner.cpp -- the single-matrix consensus as ONE library call.
//
// Sequences the stages of pcx_matrix.hip for Oracle.consensus() (__init__.py:502-611)
// and for the reference's stage methods (interpolate / wpca / lie_detector /
// nonconformity(_rank), :260-500); owns the scratch (cached per context) and the
// cross-rank exchange between stages (pcx_comm.cpp: RCCL, in-process group, callbacks).
//
// Exchange discipline:
//   * per-rank double-double partial sums live in slot [rank] of [world][...] buffers and
//     are ALL-GATHERED; kernels then combine the ranks in rank order, so every rank gets
//     bit-identical event vectors whatever the collective's internal order;
//   * exact integer selection state (weight limbs, counts) is all-reduced with SUM, key
//     ranges and minimum weights with MIN / MAX -- order-independent by construction;
//   * the covariance partial (E x E) is the one floating-point SUM all-reduce.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <thread>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "pcx_internal.h"
#include "pcx_sync.h"

namespace {
constexpr int BT = 256;
constexpr int CS = 16;  // dd slots per column in cstat
constexpr int CM = 8;   // doubles per column in mpart / cmax
constexpr int EV_SLOTS = 19;  // E-sized rows of ev (pcx_matrix.hip ev_slot)
constexpr int SS = 16;  // dd slots in scal
constexpr int SC_BIGTOK_SLOT = 10;  // scal slot: count of tokens outside [0, 63] (pcx_matrix.hip SC_BIGTOK)
constexpr int COV_TILE = 128;
constexpr int COV_STAGE = 64 * PCX_GEMM_KS > 128 ? 64 * PCX_GEMM_KS : 128;  // wcd rows: whole stages of the int8 GEMM
constexpr int SELS = 40;
// k-slice cost model of the covariance products (calibrated on C5, profiles/r3): one 64-row
// stage of one 256 x 256 int8 tile, one 8-row stage of one 128 x 128 fp64 tile (3 per CU), and
// the effective rate at which a slab is written and read back by k_cov_reduce
constexpr double GEMM_I8_STAGE_S = 0.55e-6, SYRK_STAGE_S = 2.8e-6, SLAB_BW = 4.0e12;
constexpr int MAX_SEL_PASSES = 12;  // 64-bit keys, >= 8 bits resolved per pass

template <class T>
T* at(void* base, size_t off) {
    return reinterpret_cast<T*>(static_cast<char*>(base) + off);
}
}  // namespace

// one rank's scratch for an (n_rows x E) shard with n_scaled scaled events
struct pcx_workspace {
    int64_t n_rows = -1, E = -1, n_total = -1;
    int n_scaled = -1, world = -1;
    int64_t col_blocks = 0, cov_tiles = 0, cov_kslices = 0, wcd_rows = 0, wcd_ld = 0;
    std::vector<void*> blocks;
    size_t bytes = 0;
    // zeroed before every call
    void* zero_base = nullptr;
    size_t zero_bytes = 0;
    // buffers
    double *rep, *tok, *T, *part, *mpart, *cstat, *cmax, *scal, *spart, *ev, *cslab, *C, *Mw, *pvec, *rowv;
    uint32_t* rowstat;
    uint64_t* skey;
    int64_t* info;
    uint64_t *sel_state, *sel_isum, *hist_w, *hist_min, *sel_arg;
    int32_t *sel_act, *hard, *hard_cols, *hard_modes, *scols, *sidx;
    double *wcd, *tokp, *scalars, *xsend, *xrecv;
    uint32_t* rowpart;
    int32_t *cov_perm, *cov_pos;
    int8_t *zA, *zB;
    int64_t* zsum;
    double* dscale;
    uint64_t* cbuf;
    uint64_t* vsave;
    int64_t* ccount;
    int64_t ccap = 0;
    // sized by the data (the grid / general split), grown on demand
    struct Grow {
        void* p = nullptr;
        size_t bytes = 0;
    } pgg, zd, pmx, clw, fg, nam, dtok, ze, pgx, wdig, zbg;
    bool grow(Grow& g, size_t need) {
        if (g.bytes >= need) return true;
        if (g.p) (void)hipFree(g.p);
        g.p = nullptr;
        g.bytes = 0;
        if (hipMalloc(&g.p, need) != hipSuccess) return false;
        g.bytes = need;
        return true;
    }
    int64_t xcap = 0;  // doubles per rank in xsend

    ~pcx_workspace() {
        for (void* p : blocks) (void)hipFree(p);
        for (Grow* g : {&pgg, &zd, &pmx, &clw, &fg, &nam, &dtok, &ze, &pgx, &wdig, &zbg})
            if (g->p) (void)hipFree(g->p);
    }
};

namespace pcx {
namespace {

struct Fail {
    int code;
};

struct Run {
    pcx_ctx* c;
    hipStream_t st;
    std::string& err;
    Comm* comm;
    int world, rank;
    std::vector<hipEvent_t> evs;
    std::vector<int> ev_stage;
    double comm_bytes = 0.0;

    void hip(hipError_t e, const char* what) {
        if (e != hipSuccess) {
            err = std::string(what) + ": " + hipGetErrorString(e);
            throw Fail{PCX_EHIP};
        }
    }
    void check_err(hipError_t e, const char* what) {
        if (!err.empty()) throw Fail{PCX_EINVAL};
        hip(e, what);
    }
    void comm_rc(int rc) {
        if (rc) throw Fail{rc};
    }
    // profiling marks (HIP events on the context's stream)
    void mark(int stage) {
        if (stage >= 0) c->progress_stage.store(stage, std::memory_order_relaxed);
        if (!c->profile) return;
        hipEvent_t e;
        hip(hipEventCreate(&e), "hipEventCreate");
        hip(hipEventRecord(e, st), "hipEventRecord");
        evs.push_back(e);
        ev_stage.push_back(stage);
    }
    void stage(pcx_mat& m, int s) {
        mark(s);
        check_err(mat_stage(m, s, st, err), stage_name(s));
        mark(-1);
    }
    void sync() {
        c->progress_wait.store(1, std::memory_order_relaxed);
        hip(hipStreamSynchronize(st), "hipStreamSynchronize");
        c->progress_wait.store(0, std::memory_order_relaxed);
    }
    template <class T>
    T read(const T* dev) {
        T v;
        hip(hipMemcpyAsync(&v, dev, sizeof(T), hipMemcpyDeviceToHost, st), "D2H");
        sync();
        return v;
    }

    // ---- exchanges
    void allreduce(void* buf, int64_t count, int dtype, int op) {
        if (!comm || count <= 0) return;
        mark(M_EXCHANGE);
        comm_bytes += 8.0 * (double)count;
        comm_rc(comm->allreduce(buf, count, dtype, op, st, err));
        mark(-1);
    }
    // dd slots [s0, s1) of every column of a [world][rows][pitch/2] dd buffer
    void gather_slots(double* buf, int64_t rows, int64_t pitch, int s0, int s1, pcx_workspace* w) {
        if (!comm) return;
        mark(M_EXCHANGE);
        const int64_t width = (int64_t)(s1 - s0) * 2, blk = rows * pitch;
        if (width * rows > w->xcap) {
            err = "exchange buffer too small";
            throw Fail{PCX_EINVAL};
        }
        hip(copy2d(w->xsend, width, buf + (int64_t)rank * blk + 2 * s0, pitch, width, rows, st), "pack");
        comm_bytes += 8.0 * (double)(width * rows);
        comm_rc(comm->allgather(w->xsend, w->xrecv, width * rows * 8, st, err));
        for (int r = 0; r < world; r++)
            if (r != rank)
                hip(copy2d(buf + (int64_t)r * blk + 2 * s0, pitch, w->xrecv + (int64_t)r * width * rows, width, width,
                           rows, st),
                    "unpack");
        mark(-1);
    }
    // whole per-rank blocks of a [world][bytes] buffer (in place)
    void gather_block(void* buf, int64_t bytes) {
        if (!comm) return;
        mark(M_EXCHANGE);
        comm_bytes += (double)bytes;
        comm_rc(comm->allgather(static_cast<char*>(buf) + (int64_t)rank * bytes, buf, bytes, st, err));
        mark(-1);
    }
};

// ------------------------------------------------------------------ workspace
pcx_workspace* workspace(pcx_ctx* c, int64_t n_rows, int64_t E, int64_t n_total, int n_scaled, int world,
                         std::string& err, int& rc) {
    pcx_workspace* w = c->ws;
    // capacity semantics in the scaled-event count: a context that runs many shapes of
    // bounds (the batched-rounds scheduler sets scaled_floor = E) reuses one workspace
    if (w && w->n_rows == n_rows && w->E == E && w->n_scaled >= n_scaled && w->world == world &&
        w->n_total == n_total)
        return w;
    n_scaled = std::max(n_scaled, (int)std::min<int64_t>(c->scaled_floor, E));
    delete c->ws;  // one cached workspace per context (a C5 shard's is ~50 GB)
    c->ws = nullptr;
    w = new (std::nothrow) pcx_workspace;
    if (!w) {
        rc = PCX_ENOMEM;
        err = "workspace: out of host memory";
        return nullptr;
    }
    w->n_rows = n_rows;
    w->E = E;
    w->n_total = n_total;
    w->n_scaled = n_scaled;
    w->world = world;
    const int64_t S = std::max(1, n_scaled);
    const int64_t ceb = (E + BT - 1) / BT;
    // enough row chunks to give ~2048 column-pass blocks, at least 32 rows each
#ifndef PCX_COL_TARGET  // (a build parameter for A/B runs: column-pass blocks aimed at)
#define PCX_COL_TARGET 2048
#endif
    w->col_blocks = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(std::max<int64_t>(1, PCX_COL_TARGET / ceb),
                                                                             (n_rows + 31) / 32),
                                                           4096));
    const int64_t nb = (E + COV_TILE - 1) / COV_TILE;
    w->cov_tiles = nb * (nb + 1) / 2;
    w->wcd_rows = (n_rows + COV_STAGE - 1) / COV_STAGE * COV_STAGE;
    w->wcd_ld = nb * COV_TILE;
    const int64_t stages = w->wcd_rows / COV_STAGE;
    const int64_t ks = (16 * 3 * 256 + w->cov_tiles - 1) / w->cov_tiles;
    w->cov_kslices = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(32, ks), stages >= 8 ? stages / 8 : 1));
    w->xcap = E * CS * 2;
    // selection compaction: up to 256k (key, weight) pairs per scaled event and rank (4 GB at C5)
    w->ccap = n_scaled > 0 ? std::min<int64_t>(262144, n_rows) : 0;

    // small buffers (zeroed per call) in one block, the big ones in their own
    struct Item {
        void** dst;
        size_t bytes;
        bool zero;
    };
    std::vector<Item> items = {
        {(void**)&w->rep, (size_t)n_rows * 8, true},
        {(void**)&w->tok, (size_t)n_rows * 8, true},
        {(void**)&w->part, (size_t)(w->col_blocks * E * 16) * 8, true},
        {(void**)&w->mpart, (size_t)(w->col_blocks * E * CM) * 8, true},
        {(void**)&w->cstat, (size_t)(world * E * CS * 2) * 8, true},
        {(void**)&w->cmax, (size_t)(world * E * CM) * 8, true},
        {(void**)&w->cov_perm, (size_t)w->wcd_ld * 4, true},
        {(void**)&w->cov_pos, (size_t)E * 4, true},
        {(void**)&w->zsum, (size_t)E * 8, true},
        {(void**)&w->scal, (size_t)(world * SS * 2) * 8, true},
        {(void**)&w->spart, (size_t)(4096 * 8) * 8, true},
        {(void**)&w->ev, (size_t)(EV_SLOTS * E) * 8, true},
        {(void**)&w->pvec, (size_t)(4 * (E + 64)) * 8, true},
        {(void**)&w->rowv, (size_t)(6 * n_rows) * 8, true},
        {(void**)&w->rowstat, (size_t)(2 * n_rows) * 4, true},
        {(void**)&w->skey, (size_t)(world * 4) * 8, true},
        {(void**)&w->info, (size_t)16 * 8, true},
        {(void**)&w->sel_state, (size_t)(S * SELS) * 8, true},
        {(void**)&w->sel_isum, (size_t)(S * 4) * 8, true},

        {(void**)&w->sel_arg, (size_t)(S * 2) * 8, true},
        {(void**)&w->sel_act, (size_t)S * 4, true},
        {(void**)&w->hard, (size_t)E * 4, true},
        {(void**)&w->ccount, (size_t)S * 8, true},
        {(void**)&w->cbuf, (size_t)(S * w->ccap * 2) * 8, false},
        {(void**)&w->vsave, (size_t)(S * (SEL_NB * 3 + 4)) * 8, true},
        {(void**)&w->hard_cols, (size_t)E * 4, true},
        {(void**)&w->hard_modes, (size_t)E * 4, true},
        {(void**)&w->scols, (size_t)S * 4, false},
        {(void**)&w->sidx, (size_t)E * 4, false},
        {(void**)&w->scalars, (size_t)4 * 8, true},
        // hist_w | hist_n (one SUM per pass), hist_min | hist_max | sel_imin | sel_imax (one MAX):
        // the runner places hist_n / hist_max right after the pass's active rows (select())
        {(void**)&w->hist_w, (size_t)(S * SEL_NB * 4) * 8, false},
        {(void**)&w->hist_min, (size_t)(S * SEL_NB * 2 + S * 4) * 8, false},
        {(void**)&w->xsend, (size_t)w->xcap * 8, false},
        {(void**)&w->xrecv, (size_t)(w->xcap * world) * 8, false},
        {(void**)&w->T, (size_t)(S * n_rows) * 8, false},
        {(void**)&w->cslab, (size_t)std::max<int64_t>(w->cov_kslices * E * E * 8, 24 * E), false},  // + rank counts
        {(void**)&w->C, (size_t)(E * E) * 8, false},
        {(void**)&w->Mw, (size_t)(2 * E * E + 8 * E + 64) * 8, false},
        {(void**)&w->wcd, (size_t)(w->wcd_rows * w->wcd_ld) * 8, false},
        {(void**)&w->tokp, (size_t)(w->wcd_rows + 64) * 8, false},
        {(void**)&w->rowpart, (size_t)(((w->wcd_ld + 511) / 512) * w->wcd_rows * 2) * 4, false},
        {(void**)&w->zA, (size_t)(w->wcd_rows * (w->wcd_ld + 256)), false},
        {(void**)&w->zB, (size_t)(w->wcd_rows * (w->wcd_ld + 256)), false},
        {(void**)&w->dscale, (size_t)(2 * w->wcd_ld) * 8, false},  // dscale, then escale
    };
    auto align = [](size_t b) { return (b + 255) / 256 * 256; };
    size_t zb = 0;
    for (auto& it : items)
        if (it.zero) zb += align(it.bytes);
    void* zbase = nullptr;
    hipError_t e = hipMalloc(&zbase, zb);
    if (e != hipSuccess) {
        delete w;
        rc = PCX_ENOMEM;
        err = "workspace: hipMalloc of " + std::to_string(zb) + " bytes failed";
        return nullptr;
    }
    w->blocks.push_back(zbase);
    w->zero_base = zbase;
    w->zero_bytes = zb;
    size_t off = 0;
    w->bytes = zb;
    for (auto& it : items) {
        if (it.zero) {
            *it.dst = at<void>(zbase, off);
            off += align(it.bytes);
        } else {
            void* p = nullptr;
            e = hipMalloc(&p, std::max<size_t>(it.bytes, 256));
            if (e != hipSuccess) {
                const size_t want = it.bytes;
                delete w;
                rc = PCX_ENOMEM;
                err = "workspace: hipMalloc of " + std::to_string(want) + " bytes failed";
                return nullptr;
            }
            w->blocks.push_back(p);
            w->bytes += it.bytes;
            *it.dst = p;
        }
    }
    c->ws = w;
    return w;
}

// ------------------------------------------------------------------ host <-> device staging
// Buffers of at least IO_CACHE_MIN bytes (the reports, `original`, `filled`) come from the context's
// io_bufs, grown on demand and kept between calls, in call order; smaller ones are allocated per call.
constexpr size_t IO_CACHE_MIN = (size_t)64 << 20;
constexpr size_t ARENA_MAX = (size_t)16 << 20;  // outputs up to this size share the vectors' arena

// the context's pinned buffer for the arena's copy back, grown on demand
bool pin_small(pcx_ctx* c, size_t bytes) {
    if (c->pin_small_bytes >= bytes) return true;
    if (c->pin_small) (void)hipHostFree(c->pin_small);
    c->pin_small = nullptr;
    c->pin_small_bytes = 0;
    if (hipHostMalloc(&c->pin_small, bytes, hipHostMallocDefault) != hipSuccess) {
        c->pin_small = nullptr;
        return false;
    }
    c->pin_small_bytes = bytes;
    return true;
}
struct Io {
    pcx_ctx* c;
    std::vector<void*> owned;
    size_t next = 0;  // the next io_bufs slot
    explicit Io(pcx_ctx* ctx) : c(ctx) {}
    ~Io() {
        for (void* p : owned) (void)hipFree(p);
    }
    void* get(Run& R, size_t bytes, const char* what) {
        void* p = nullptr;
        if (bytes >= IO_CACHE_MIN) {
            if (next == c->io_bufs.size()) c->io_bufs.push_back({nullptr, 0});
            auto& b = c->io_bufs[next++];
            if (b.second < bytes) {
                if (b.first) (void)hipFree(b.first);
                b = {nullptr, 0};
                R.hip(hipMalloc(&b.first, bytes), what);
                b.second = bytes;
            }
            return b.first;
        }
        R.hip(hipMalloc(&p, bytes), what);
        owned.push_back(p);
        return p;
    }
    template <class T>
    T* dev(Run& R, const T* host, int64_t n) {  // device copy of a host input (NULL stays NULL)
        if (!host || n <= 0) return nullptr;
        void* p = get(R, n * sizeof(T), "hipMalloc(input)");
        R.hip(hipMemcpyAsync(p, host, n * sizeof(T), hipMemcpyHostToDevice, R.st), "H2D");
        return (T*)p;
    }
    double* out(Run& R, double* host, int64_t n) {  // device buffer for a host output
        if (!host || n <= 0) return nullptr;
        return (double*)get(R, n * 8, "hipMalloc(output)");
    }
    // the small host outputs (the per-reporter and per-event vectors) share one device arena, so
    // they come back in one copy through a pinned buffer: ~17 separate pageable copies of a
    // consensus took 0.25 ms of a 1k x 100 call
    char* arena = nullptr;
    size_t arena_cap = 0, arena_used = 0;
    double* out_small(Run& R, int64_t n, size_t cap) {
        const size_t b = ((size_t)n * 8 + 255) / 256 * 256;
        if (!arena) {
            arena = (char*)get(R, cap, "hipMalloc(small outputs)");
            arena_cap = cap;
        }
        if (arena_used + b > arena_cap) return nullptr;
        double* p = (double*)(arena + arena_used);
        arena_used += b;
        return p;
    }
};

// Device -> pageable host copy of a large output (the host-memory path's `filled` / `original`,
// 33 GB each at C5).  A plain hipMemcpy stages it through the runtime's pinned buffer on one
// thread, where the destination's first-touch page faults also land: 17-26 GB/s measured for C5's
// outputs (tools/c5_host_latency.py).  Here the DMA of chunk k+1 runs into a pinned slot while
// host threads move chunk k into place (chunked_copy, pcx_sync.h), so PCIe and the page faults
// overlap and the faults spread over the threads.
constexpr size_t STAGE_CHUNK = (size_t)64 << 20;
constexpr int STAGE_SLOTS = 3;
constexpr size_t STAGE_MIN = (size_t)256 << 20;  // smaller copies: one hipMemcpyAsync

int host_threads() {
    int t = 0;
    if (const char* e = getenv("OMP_NUM_THREADS")) t = atoi(e);  // the job's host-core share (16 per GPU on the pool)
    if (t < 1) t = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 16));
}

// pinned staging slots for d2h_staged (grown once, kept in the context)
bool stage_slots(pcx_ctx* c) {
    const size_t need = STAGE_CHUNK * STAGE_SLOTS;
    if (c->pinned_bytes >= need) return true;
    if (c->pinned) (void)hipHostFree(c->pinned);
    c->pinned = nullptr;
    c->pinned_bytes = 0;
    if (hipHostMalloc(&c->pinned, need, hipHostMallocDefault) != hipSuccess) {
        c->pinned = nullptr;
        return false;
    }
    c->pinned_bytes = need;
    return true;
}

// the staged copy on stream `st` through the context's slots (stage_slots first); 0 or PCX_EHIP
int d2h_staged_on(pcx_ctx* c, hipStream_t st, void* dst, const void* src, size_t bytes) {
    hipEvent_t ev[STAGE_SLOTS] = {};
    struct Evs {  // (the guard before the first creation: a failed one leaks none made before it)
        hipEvent_t* e;
        ~Evs() {
            for (int k = 0; k < STAGE_SLOTS; k++)
                if (e[k]) (void)hipEventDestroy(e[k]);
        }
    } evs{ev};
    for (int k = 0; k < STAGE_SLOTS; k++)
        if (hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) return PCX_EHIP;
    char* pin = static_cast<char*>(c->pinned);
    const char* s = static_cast<const char*>(src);
    char* d = static_cast<char*>(dst);
    const int64_t nchunks = (int64_t)((bytes + STAGE_CHUNK - 1) / STAGE_CHUNK);
    auto len_of = [&](int64_t k) { return std::min(STAGE_CHUNK, bytes - (size_t)k * STAGE_CHUNK); };
    return chunked_copy(
        nchunks, STAGE_SLOTS, host_threads(),
        [&](int64_t k, int slot) -> int {
            hipError_t e = hipMemcpyAsync(pin + slot * STAGE_CHUNK, s + k * STAGE_CHUNK, len_of(k),
                                          hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipEventRecord(ev[slot], st);
            return e == hipSuccess ? 0 : PCX_EHIP;
        },
        [&](int slot) { return hipEventSynchronize(ev[slot]) == hipSuccess ? 0 : PCX_EHIP; },
        [&](int64_t k, int slot, int t, int T) {
            const size_t len = len_of(k), a = len * t / T, b = len * (t + 1) / T;
            if (b > a) memcpy(d + k * STAGE_CHUNK + a, pin + slot * STAGE_CHUNK + a, b - a);
        });
}

void d2h_staged(Run& R, void* dst, const void* src, size_t bytes) {
    if (!stage_slots(R.c)) R.hip(hipErrorOutOfMemory, "hipHostMalloc(staging)");
    if (d2h_staged_on(R.c, R.st, dst, src, bytes)) R.hip(hipErrorUnknown, "staged D2H of an output");
}

// The host path's `filled` is complete once k_wcd has run (M_WCD); its copy back (33 GB at C5)
// then runs on the context's side stream, behind an event on the main one, while the device
// computes the covariance and the rest -- instead of after all of it.  Joined before the call
// returns (the destructor too, on a failure path: the main stream has drained by then).
struct EarlyD2H {
    std::thread th;
    hipEvent_t ready = nullptr;
    int rc = 0;
    void start(Run& R, void* dst, const void* src, size_t bytes) {
        pcx_ctx* c = R.c;
        if (!c->side_stream) R.hip(hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking), "side stream");
        if (!stage_slots(c)) R.hip(hipErrorOutOfMemory, "hipHostMalloc(staging)");
        R.hip(hipEventCreateWithFlags(&ready, hipEventDisableTiming), "hipEventCreate");
        R.hip(hipEventRecord(ready, R.st), "hipEventRecord");
        R.hip(hipStreamWaitEvent(c->side_stream, ready, 0), "hipStreamWaitEvent");
        th = std::thread([this, c, dst, src, bytes] { rc = d2h_staged_on(c, c->side_stream, dst, src, bytes); });
    }
    int join() {
        if (th.joinable()) th.join();
        if (ready) (void)hipEventDestroy(ready);
        ready = nullptr;
        return rc;
    }
    ~EarlyD2H() { join(); }
};

// the reports' H2D in row chunks, each followed by an event, so that host threads can rewrite the
// chunks already copied (the in-place `original`) while the later ones are in flight.  A thread
// waits until chunk k's event has been recorded (an unrecorded event reads as complete), then on
// the event; abort() (a failure while issuing) releases the waiters.
struct ChunkGate {
    std::vector<hipEvent_t> ev;
    std::vector<int64_t> row0;  // chunk k: rows [row0[k], row0[k + 1])
    std::mutex mu;
    std::condition_variable cv;
    int recorded = 0;
    bool aborted = false;
    int nchunks() const { return (int)ev.size(); }
    void mark(int k) {
        std::lock_guard<std::mutex> lk(mu);
        recorded = k + 1;
        cv.notify_all();
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
    bool wait(int k) {  // false: aborted
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return recorded > k || aborted; });
            if (recorded <= k) return false;
        }
        return hipEventSynchronize(ev[k]) == hipSuccess;
    }
    ~ChunkGate() {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

// result["original"] for host memory, built by host threads from the caller's reports while the
// device works (started once the reports' H2D has drained), instead of copied back (33 GB of D2H at
// C5): x = (r - lo) / (hi - lo) for a scaled event as IEEE division -- the device's div_rn is that
// division bit for bit, tests/test_fastdiv.py -- truncated for an integer dtype (Q3), r itself
// otherwise; a NaN report keeps its bits (as the device's `original` does).  In place (Q2: original
// IS the caller's reports) only the scaled columns are written.  `filled` still comes from the
// device (its fills are known only at the end): its D2H runs beside this pass, which overlaps it.
// (Building `filled` here too, after the device, measured slower: 1.58-1.66 s against 1.47-1.51 s
// in place at C5 -- the host's memory bandwidth, not PCIe, bound it.)  Rows split over
// host_threads() threads; a small matrix runs on the calling thread.
struct HostOriginal {
    std::vector<std::thread> th;
    ChunkGate* gate_ = nullptr;  // (released on destruction: a failure before every chunk was issued)
    // gate: the reports' H2D chunks (in place: a chunk is rewritten only once it has been copied)
    void start(const double* rep_in, double* original, int64_t n_rows, int64_t E, const std::vector<uint8_t>& scaled,
               const double* lo, const double* hi, bool int_dtype, ChunkGate* gate = nullptr) {
        std::vector<int32_t> sc;
        std::vector<double> lr;
        for (int64_t j = 0; j < (int64_t)scaled.size(); j++)
            if (scaled[j]) {
                sc.push_back((int32_t)j);
                lr.push_back(lo[j]);
                lr.push_back(hi[j] - lo[j]);
            }
        auto scp = std::make_shared<std::vector<int32_t>>(std::move(sc));
        auto lrp = std::make_shared<std::vector<double>>(std::move(lr));
        const bool inplace = original == rep_in;
        auto body = [=](int64_t r0, int64_t r1) {
            const int32_t* cl = scp->data();
            const double* l = lrp->data();
            const size_t nc = scp->size();
            for (int64_t i = r0; i < r1; i++) {
                const double* in = rep_in + i * E;
                double* o = original + i * E;
                if (!inplace) memcpy(o, in, (size_t)E * 8);
                for (size_t k = 0; k < nc; k++) {
                    const double r = in[cl[k]];
                    double x = (r - l[2 * k]) / l[2 * k + 1];
                    if (int_dtype) x = std::trunc(x);
                    o[cl[k]] = std::isnan(x) ? r : x;
                }
            }
        };
        const int T = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, n_rows / 1024));
        if (gate) {  // every thread takes its share of each chunk as the chunk lands
            gate_ = gate;
            for (int t = 0; t < T; t++)
                th.emplace_back([=] {
                    for (int k = 0; k < gate->nchunks(); k++) {
                        if (!gate->wait(k)) return;  // (the call fails: the array is unspecified)
                        const int64_t a = gate->row0[k], n = gate->row0[k + 1] - a;
                        body(a + n * t / T, a + n * (t + 1) / T);
                    }
                });
            return;
        }
        if (T <= 1 || n_rows * E < ((int64_t)1 << 20)) {
            body(0, n_rows);
            return;
        }
        for (int t = 0; t < T; t++) th.emplace_back(body, n_rows * t / T, n_rows * (t + 1) / T);
    }
    void join() {
        for (auto& t : th) t.join();
        th.clear();
    }
    ~HostOriginal() {
        // a call that failed before marking every chunk (a hipMalloc of the device copy, an H2D)
        // leaves threads waiting on the gate: release them (after a normal join this does nothing)
        if (gate_) gate_->abort();
        join();
    }
};

int64_t pow2_at_least(int64_t n) {
    int64_t p = 2;
    while (p < n) p <<= 1;
    return p;
}

// events whose decision is rounding-decided: replay the reference's own float order
// known_H >= 0: the selection's last read already returned the count (k_sel_compact lists the
// marked events every pass), so no list launch and no host read here
void hard_replay(Run& R, pcx_mat& m, pcx_workspace* w, pcx_result* res, int64_t known_H = -1) {
    int64_t H = known_H;
    if (H < 0) {
        R.mark(M_HARD_LIST);
        R.hip(hard_list(m, w->hard_cols, w->hard_modes, R.st), "k_hard_list");
        R.mark(-1);
        H = R.read(m.info + INFO_HARD);
    }
    if (H <= 0) return;
    res->n_hard += (int32_t)H;
    const int64_t N = m.n_total, cap = std::max<int64_t>(1, m.n_rows);
    const int64_t P_max = pow2_at_least(N);
    // batch size: keep the batch's scratch near 2 GB
    const int64_t per = cap * 16 * (1 + R.world) + P_max * 16 + N * 16 + 64;
    const int64_t Hb = std::max<int64_t>(1, std::min<int64_t>(H, (int64_t)(2ll << 30) / per));
    void* scratch = nullptr;
    const size_t bytes = (size_t)(Hb * per + 4096);
    R.hip(hipMalloc(&scratch, bytes), "hipMalloc(hard replay scratch)");
    struct Free {
        void* p;
        ~Free() { (void)hipFree(p); }
    } fr{scratch};
    size_t off = 0;
    auto carve = [&](size_t b) {
        void* p = at<void>(scratch, off);
        off += (b + 255) / 256 * 256;
        return p;
    };
    HardArgs h{};
    h.cap = cap;
    h.send = (double*)carve(Hb * cap * 16);
    h.recv = !R.comm ? h.send : (double*)carve(R.world * Hb * cap * 16);
    h.keys = (uint64_t*)carve(Hb * P_max * 16);
    h.X = (double*)carve(Hb * N * 8);
    h.W = (double*)carve(Hb * N * 8);
    h.hs = (double*)carve(Hb * 4 * 8);
    h.send_cnt = (int64_t*)carve(Hb * 8);
    h.recv_cnt = !R.comm ? h.send_cnt : (int64_t*)carve(R.world * Hb * 8);
    for (int64_t b0 = 0; b0 < H; b0 += Hb) {
        h.n_hard = (int32_t)std::min<int64_t>(Hb, H - b0);
        h.cols = w->hard_cols + b0;
        h.modes = w->hard_modes + b0;
        R.mark(M_HARD_GATHER);
        R.check_err(hard_stage(m, h, M_HARD_GATHER, R.st, R.err), "hard gather");
        R.mark(-1);
        if (R.comm) {
            // compact the send rows of the batch: [n_hard][cap] pairs, counts
            R.mark(M_EXCHANGE);
            R.comm_bytes += (double)h.n_hard * (double)(cap * 16 + 8);
            R.comm_rc(R.comm->allgather(h.send, h.recv, (int64_t)h.n_hard * cap * 16, R.st, R.err));
            R.comm_rc(R.comm->allgather(h.send_cnt, h.recv_cnt, (int64_t)h.n_hard * 8, R.st, R.err));
            R.mark(-1);
        }
        // segment length: the largest gathered count, rounded up to a power of two
        std::vector<int64_t> cnt((size_t)R.world * h.n_hard);
        R.hip(hipMemcpyAsync(cnt.data(), h.recv_cnt, cnt.size() * 8, hipMemcpyDeviceToHost, R.st), "D2H counts");
        R.sync();
        int64_t nmax = 1;
        for (int j = 0; j < h.n_hard; j++) {
            int64_t t = 0;
            for (int r = 0; r < R.world; r++) t += cnt[(size_t)r * h.n_hard + j];
            nmax = std::max(nmax, t);
        }
        h.P = pow2_at_least(nmax);
        R.mark(M_HARD_PREP);
        R.check_err(hard_stage(m, h, M_HARD_PREP, R.st, R.err), "hard prep");
        R.mark(-1);
        R.mark(M_HARD_SORT);
        R.check_err(hard_stage(m, h, M_HARD_SORT, R.st, R.err), "hard sort");
        R.mark(-1);
        R.mark(M_HARD_WALK);
        R.check_err(hard_stage(m, h, M_HARD_WALK, R.st, R.err), "hard walk");
        R.mark(-1);
        R.sync();  // the scratch is reused by the next batch / freed
    }
}

// the selection histograms of a pass over `active` events: hist_n right after hist_w's active
// rows, hist_max right after hist_min's, so each pass reduces over ranks in one SUM and one MAX
void sel_layout(pcx_mat& m, int64_t active) {
    m.hist_n = m.hist_w + active * SEL_NB * 3;
    m.hist_max = m.hist_min + active * SEL_NB;
}

// weighted medians of the scaled events (phase 1: interpolation fills, phase 2: outcomes),
// plus the replay of rounding-decided binary fills (phase 1)
void select(Run& R, pcx_mat& m, pcx_workspace* w, int phase, pcx_result* res) {
    m.sel_phase = phase;
    const int S = m.n_scaled;
    int64_t known_H = -1;
    if (!R.comm && m.n_rows <= SEL_EXACT_MAX) {
        // small matrices: replay the reference's float walk directly
        if (S) R.stage(m, M_SEL_EXACT);
    } else if (S) {
        // first pass, with no host read before it: the key range of every needed event is
        // known (M_COLSTATS, the fill), so one histogram pass over the whole range also collects
        // the totals the walk starts from; launched for all S events (those not needed exit),
        // its collectives sized for S.  Counting only for reputation=None interpolation medians.
        R.stage(m, M_SEL_INIT);  // (also the sampled windows, k_sel_sample: every rank's samples summed)
        R.allreduce(w->hist_w, (int64_t)S * SEL_NB * 3, PCX_F64, PCX_SUM);
        sel_layout(m, S);
        m.sel_imin = m.hist_min + (int64_t)S * SEL_NB * 2;  // right after hist_max's S rows
        m.sel_imax = m.sel_imin + (int64_t)S * 2;
        R.hip(hipMemsetAsync(m.sel_imin, 0, (size_t)S * 4 * 8, R.st), "sel_imin");  // (MAX identity)
        m.sel_first = 1;
        R.mark(M_SEL_HIST);
        R.check_err(sel_hist(m, S, R.st), "k_sel_hist");
        R.mark(-1);
        m.sel_first = 0;
        // two collectives: the counts (and limbs unless every weight is equal), and the (complemented)
        // minima with the maxima -- bucket keys, then the weights' bit patterns
        if (!(phase == 1 && !m.rep_raw))
            R.allreduce(w->hist_w, (int64_t)S * SEL_NB * 4, PCX_U64, PCX_SUM);
        else
            R.allreduce(m.hist_n, (int64_t)S * SEL_NB, PCX_U64, PCX_SUM);
        R.allreduce(w->hist_min, (int64_t)S * SEL_NB * 2 + (int64_t)S * 4, PCX_U64, PCX_MAX);
        R.stage(m, M_SEL_START);
        R.mark(M_SEL_STEP);
        R.check_err(sel_step(m, S, R.st), "k_sel_step");
        R.mark(-1);
        R.stage(m, M_SEL_COMPACT);
        int64_t inf5[5];  // active, argmax, (pick1), (hard), weight-mode active
        R.hip(hipMemcpyAsync(inf5, m.info + INFO_SEL_ACTIVE, sizeof(inf5), hipMemcpyDeviceToHost, R.st), "D2H");
        R.sync();
        int64_t active = inf5[0], wactive = inf5[4];
        known_H = inf5[3];
        if (inf5[1] > 0) {  // dominant weights: the first row holding the max weight (all ranks)
            R.stage(m, M_SEL_ARGMAX);
            R.allreduce(w->sel_arg, S, PCX_U64, PCX_MIN);
            R.stage(m, M_SEL_VALUE);
            R.allreduce(w->sel_arg + S, S, PCX_U64, PCX_MAX);
            R.stage(m, M_SEL_VALUE_FINISH);
        }
        // Later passes, with no host round trip between them: pass p + 1 is launched before the
        // host has read pass p's active count, sized by the last count it knows (an upper bound:
        // events only leave; the extra workgroups see info[IN_SEL_ACTIVE] and exit, the extra
        // collective rows are reduced and ignored, and all ranks size them alike), while pass p's
        // five info words travel to pinned memory behind it.  When a count comes back 0 the pass
        // already launched after it finds nothing to do (one empty pass per phase: three short
        // launches against one host round trip per pass).
        int passes = 1;
        if (active > 0) {
            pcx_ctx* c = R.c;
            if (!c->sel_pin) {  // the events first: sel_pin is published only with both of them made
                for (hipEvent_t& ev : c->sel_ev)
                    if (!ev) R.hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
                int64_t* pin = nullptr;
                R.hip(hipHostMalloc((void**)&pin, 16 * sizeof(int64_t), hipHostMallocDefault), "hipHostMalloc(sel)");
                c->sel_pin = pin;
            }
            auto launch_pass = [&](int64_t a_ub, int64_t w_ub, int slot) {
                if (passes == MAX_SEL_PASSES + 1) {  // (+1: the speculative pass after the last)
                    R.err = "weighted selection did not converge";
                    throw Fail{PCX_EINVAL};
                }
                sel_layout(m, a_ub);
                R.mark(M_SEL_HIST);
                R.check_err(sel_hist(m, (int)a_ub, R.st), "k_sel_hist");
                R.mark(-1);
                // exact integers: order-independent reductions (limbs only when some event walks weights)
                if (w_ub > 0)
                    R.allreduce(w->hist_w, a_ub * SEL_NB * 4, PCX_U64, PCX_SUM);
                else
                    R.allreduce(m.hist_n, a_ub * SEL_NB, PCX_U64, PCX_SUM);
                R.allreduce(w->hist_min, a_ub * SEL_NB * 2, PCX_U64, PCX_MAX);
                R.mark(M_SEL_STEP);
                R.check_err(sel_step(m, (int)a_ub, R.st), "k_sel_step");
                R.mark(-1);
                R.stage(m, M_SEL_COMPACT);
                R.hip(hipMemcpyAsync(c->sel_pin + 8 * slot, m.info + INFO_SEL_ACTIVE, 5 * sizeof(int64_t),
                                     hipMemcpyDeviceToHost, R.st),
                      "D2H");
                R.hip(hipEventRecord(c->sel_ev[slot], R.st), "event record");
                passes++;
            };
            int slot = 0;
            launch_pass(active, wactive, slot);
            while (true) {
                launch_pass(active, wactive, slot ^ 1);  // (speculative: pass `slot`'s count unknown yet)
                c->progress_wait.store(1, std::memory_order_relaxed);
                R.hip(hipEventSynchronize(c->sel_ev[slot]), "hipEventSynchronize");
                c->progress_wait.store(0, std::memory_order_relaxed);
                const int64_t* r = c->sel_pin + 8 * slot;
                known_H = r[3];
                if (r[0] == 0) {
                    passes--;  // (the pass launched after it had nothing to do)
                    break;
                }
                active = r[0];
                wactive = r[4];
                slot ^= 1;
            }
        }
        res->sel_passes += passes;
    }
    hard_replay(R, m, w, res, known_H);
    if (S) R.stage(m, M_SEL_FINISH);
}

// ------------------------------------------------------------------ clustering algorithms
// nc of "k-means" (:392-405), "hierarchical" (:407-419) or "clusterfeck" (:148-242,
// :421-424) into rowv[RV_N1] (pcx_matrix.hip cluster_stage; one rank)
void cluster_nc(Run& R, pcx_mat& m, pcx_workspace* w, const pcx_problem* p) {
    const int64_t N = m.n_rows, E = m.n_events;
    const int alg = m.algorithm;
    const int64_t K = alg == PCX_ALG_KMEANS ? p->kmeans_k : 0, RS = alg == PCX_ALG_KMEANS ? p->kmeans_restarts : 0;
    const int64_t nS = alg == PCX_ALG_CLUSTERFECK ? N * E : K * E;
    auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
    const int64_t dbytes = al(8 * 3 * E) + al(8 * N * E) + al(8 * nS) + 2 * al(8 * K * E) + al(8 * K) + 6 * al(8 * N) +
                           al(8 * 8);
    const int64_t ibytes = 3 * al(4 * N) + al(4 * (RS * K + 1));
    if (!w->grow(w->clw, (size_t)(dbytes + ibytes))) {
        R.err = "workspace: hipMalloc of the clustering scratch failed";
        throw Fail{PCX_ENOMEM};
    }
    char* b = (char*)w->clw.p;
    auto take = [&](int64_t bytes) {
        char* q = b;
        b += al(bytes);
        return q;
    };
    ClusterArgs a{};
    a.alg = alg;
    a.k = (int32_t)K;
    double* e3 = (double*)take(8 * 3 * E);
    a.mu = e3;
    a.sd = e3 + E;
    a.outc = e3 + 2 * E;
    a.X = (double*)take(8 * N * E);
    a.S = (double*)take(8 * nS);
    a.book = (double*)take(8 * K * E);
    a.best = (double*)take(8 * K * E);
    a.cs = (double*)take(8 * K);
    a.dist = (double*)take(8 * N);
    a.dm = (double*)take(8 * N);
    a.dm1 = (double*)take(8 * N);
    a.crep = (double*)take(8 * N);
    a.wtok = (double*)take(8 * N);
    (void)take(8 * N);
    a.kst = (double*)take(8 * 8);
    a.lab = (int32_t*)take(4 * N);
    a.cnt = (int32_t*)take(4 * N);
    a.par = (int32_t*)take(4 * N);
    a.kinit = (int32_t*)take(4 * (RS * K + 1));
    auto step = [&](int s) {
        std::string e;
        if (cluster_stage(m, a, s, R.st, e) != hipSuccess) {
            R.err = e.empty() ? "cluster_stage launch failed" : e;
            throw Fail{PCX_EHIP};
        }
    };
    R.mark(M_CLUSTER);
    if (alg == PCX_ALG_CLUSTERFECK) {
        double thr = p->cluster_threshold;  // the reference's default rule (:187-190, :210-213)
        if (!(thr > 0.0)) {
            thr = std::log10((double)E) / 1.77;
            if (thr == 0.0) thr = 0.3;
        }
        a.thr = thr;
        step(CL_WTOK);
        a.weights = a.wtok;  // outcomes = np.ma.average(features, axis=0, weights=rep) (:167)
        step(CL_MU);
        step(CL_X_F);  // features = reports_filled (:423)
        R.hip(hipMemsetAsync(a.cnt, 0, 4 * N, R.st), "hipMemset(cluster)");
        step(CL_FECK);
    } else {
        a.weights = m.rep;  // wpca's weighted mean (:317)
        step(CL_MU);
        step(CL_X_WCD);
        if (alg == PCX_ALG_HIERARCHICAL) {
            a.thr = p->hierarchy_threshold;
            step(CL_HIER);
        } else {
            step(CL_WHITEN);
            R.hip(hipMemcpyAsync(a.kinit, p->kmeans_init, 4 * RS * K, hipMemcpyHostToDevice, R.st), "H2D kinit");
            for (int r = 0; r < RS; r++) {
                a.restart = r;
                step(KM_INIT);
                for (;;) {  // Lloyd steps until |avg_prev - avg| <= 1e-5 (scipy _kmeans)
                    step(KM_ITER);
                    if (R.read(a.kst + 3) == 0.0) break;  // KS_CONT
                }
                step(KM_KEEP);
            }
            step(KM_FINAL);
        }
    }
    R.mark(-1);
}

}  // namespace

void workspace_free(pcx_ctx* c) {
    delete c->ws;
    c->ws = nullptr;
}

// The checks that do not depend on the rank: run once per call, before any worker of a
// multi-device context starts (so invalid input never reaches the abort path).
int check_problem(const pcx_problem* p, int world, int entry, std::string& err) {
    if (p->scaled && (!p->lo || !p->hi)) {
        err = "scaled given without lo / hi";
        return PCX_EINVAL;
    }
    const int alg = p->algorithm;
    if (alg < PCX_ALG_PCA || alg > PCX_ALG_CLUSTERFECK) {
        err = "algorithm must be an enum pcx_algorithm value (0..7)";
        return PCX_EINVAL;
    }
    const bool clustering = alg >= PCX_ALG_KMEANS;
    if (clustering && (world != 1 || (entry != 0 && entry != 3))) {
        err = "the clustering algorithms run on one rank, through the consensus / lie_detector entries";
        return PCX_EINVAL;
    }
    if (alg == PCX_ALG_KMEANS && (!p->kmeans_init || p->kmeans_k < 1 || p->kmeans_k > p->n_total ||
                                  p->kmeans_k > 1024 || p->kmeans_restarts < 1)) {
        err = "k-means needs kmeans_init and 1 <= kmeans_k <= min(N, 1024), kmeans_restarts >= 1";
        return PCX_EINVAL;
    }
    if (alg == PCX_ALG_KMEANS)
        for (int64_t q = 0; q < (int64_t)p->kmeans_k * p->kmeans_restarts; q++)
            if (p->kmeans_init[q] < 0 || p->kmeans_init[q] >= p->n_total) {
                err = "kmeans_init rows must lie in [0, N)";
                return PCX_EINVAL;
            }
    if (alg == PCX_ALG_HIERARCHICAL && std::isnan(p->hierarchy_threshold)) {
        err = "hierarchy_threshold is NaN";
        return PCX_EINVAL;
    }
    if (alg == PCX_ALG_COKURTOSIS && !p->aux_scores && entry != 4) {
        err = "cokurtosis needs aux_scores";
        return PCX_EINVAL;
    }
    if (!std::isfinite(p->catch_tolerance) || !std::isfinite(p->alpha)) {
        err = "catch_tolerance / alpha must be finite";
        return PCX_EINVAL;
    }
    if (p->mem_kind != PCX_MEM_DEVICE && p->mem_kind != PCX_MEM_HOST) {
        err = "mem_kind must be PCX_MEM_DEVICE or PCX_MEM_HOST";
        return PCX_EINVAL;
    }
    return 0;
}

int run_matrix(pcx_ctx* c, const pcx_problem* p, pcx_result* r, int entry, const double* scores_in, int rank_rule,
               double* nc_out, std::string& err) {
    if (!p || !r) {
        err = "null problem / result";
        return PCX_EINVAL;
    }
    const int world = c->comm ? c->comm->world : 1, rank = c->comm ? c->comm->rank : 0;
    const int64_t n_rows = p->n_rows, E = p->n_events, N = p->n_total;
    if (n_rows < 1 || E < 1 || N < n_rows || !p->reports) {
        err = "bad shape or missing reports";
        return PCX_EINVAL;
    }
    if (E > 65536 || n_rows > 0x7fffffffll) {
        err = "n_events > 65536 or n_rows >= 2^31 per rank";
        return PCX_EINVAL;
    }
    if (p->row_offset < 0 || p->row_offset + n_rows > N || (world == 1 && (N != n_rows || p->row_offset != 0))) {
        err = "row_offset / n_total inconsistent with n_rows and the context's world";
        return PCX_EINVAL;
    }
    if (const int rc = check_problem(p, world, entry, err)) return rc;
    const int alg = p->algorithm;
    const bool clustering = alg >= PCX_ALG_KMEANS;
    hipError_t he = hipSetDevice(c->device);
    if (he != hipSuccess) {
        err = std::string("hipSetDevice: ") + hipGetErrorString(he);
        return PCX_EHIP;
    }
    Run R{c, c->stream, err, c->comm, world, rank, {}, {}};
    c->progress_stage.store(-1, std::memory_order_relaxed);
    c->progress_wait.store(0, std::memory_order_relaxed);
    const bool host = p->mem_kind == PCX_MEM_HOST;
    const bool filled_input = entry >= 2;  // wpca / lie_detector / nonconformity: reports already filled
    ChunkGate gate;          // (outlives host_orig: its threads wait on it)
    HostOriginal host_orig;  // (joined on every exit path, before the caller's arrays are returned)
    EarlyD2H early_filled;
    try {
        Io io(c);
        // ---- scaled events (host view)
        std::vector<uint8_t> sc_h;
        const uint8_t* sc_in = filled_input ? nullptr : p->scaled;
        if (sc_in) {
            sc_h.resize(E);
            if (host)
                memcpy(sc_h.data(), sc_in, E);
            else {
                R.hip(hipMemcpyAsync(sc_h.data(), sc_in, E, hipMemcpyDeviceToHost, R.st), "D2H scaled");
                R.sync();
            }
        }
        std::vector<int32_t> scols, sidx(E, -1);
        for (int64_t j = 0; j < (int64_t)sc_h.size(); j++)
            if (sc_h[j]) {
                sidx[j] = (int32_t)scols.size();
                scols.push_back((int32_t)j);
            }
        const int n_scaled = (int)scols.size();
        int rc = 0;
        pcx_workspace* w = workspace(c, n_rows, E, N, n_scaled, world, err, rc);
        if (!w) return rc;
        R.hip(hipMemsetAsync(w->zero_base, 0, w->zero_bytes, R.st), "hipMemset(workspace)");
        if (n_scaled) R.hip(hipMemcpyAsync(w->scols, scols.data(), n_scaled * 4, hipMemcpyHostToDevice, R.st), "H2D");
        R.hip(hipMemcpyAsync(w->sidx, sidx.data(), E * 4, hipMemcpyHostToDevice, R.st), "H2D");

        // ---- result["original"] on the host (HostOriginal): a new array is built from the caller's
        // reports (only read) beside their H2D; in place, once the H2D has drained (below)
        const bool cons = entry == 0, lie = entry == 3;
        const bool inplace = (cons || entry == 1) && r->original &&
                             (const void*)r->original == (const void*)p->reports;
        const bool host_orig_on = host && (cons || entry == 1) && r->original;
#ifndef PCX_ORIG_EARLY
#define PCX_ORIG_EARLY 1
#endif
        if (host_orig_on && !inplace && PCX_ORIG_EARLY)
            host_orig.start(p->reports, r->original, n_rows, E, sc_h, p->lo, p->hi, p->int_dtype != 0);
        // in place: the reports copied in row chunks, each rewritten by the host threads once it
        // has landed (the whole H2D drained first measured 1.44 s against 1.33 s for a new array)
        const bool gated = host_orig_on && inplace && PCX_ORIG_EARLY && (size_t)(n_rows * E) * 8 >= STAGE_MIN;
        if (gated) {
            const int K = 16;
            gate.ev.assign(K, nullptr);
            for (int k = 0; k <= K; k++) gate.row0.push_back(n_rows * k / K);
            for (auto& e : gate.ev) R.hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
            host_orig.start(p->reports, r->original, n_rows, E, sc_h, p->lo, p->hi, p->int_dtype != 0, &gate);
        }

        // ---- inputs / outputs on the device
        pcx_mat m{};
        R.mark(M_H2D);
        const double* reports = p->reports;
        if (host && gated) {
            double* d = (double*)io.get(R, (size_t)(n_rows * E) * 8, "hipMalloc(input)");
            struct Abort {  // a failure while issuing releases the waiting threads
                ChunkGate& g;
                bool done = false;
                ~Abort() {
                    if (!done) g.abort();
                }
            } ab{gate};
            for (int k = 0; k < gate.nchunks(); k++) {
                const int64_t a = gate.row0[k] * E, n = gate.row0[k + 1] * E - a;
                R.hip(hipMemcpyAsync(d + a, p->reports + a, n * 8, hipMemcpyHostToDevice, R.st), "H2D");
                R.hip(hipEventRecord(gate.ev[k], R.st), "hipEventRecord");
                gate.mark(k);
            }
            ab.done = true;
            reports = d;
        } else if (host) {
            reports = io.dev(R, p->reports, n_rows * E);
        }
        const double* rep_raw = host ? io.dev(R, p->reputation, N) : p->reputation;
        const uint8_t* scaled = host ? io.dev(R, sc_in, E) : sc_in;
        const double* lo = sc_in ? (host ? io.dev(R, p->lo, E) : p->lo) : nullptr;
        const double* hi = sc_in ? (host ? io.dev(R, p->hi, E) : p->hi) : nullptr;
        const double* aux_src = entry == 4 ? scores_in : p->aux_scores;
        const double* aux = aux_src ? (host ? io.dev(R, aux_src, n_rows) : aux_src) : nullptr;
        R.mark(-1);
        struct OutMap {
            double* user;
            double* dev;
            int64_t n;
        };
        std::vector<OutMap> outs;
        // (the vectors' arena: every per-reporter and per-event output at most)
        const size_t small_cap = (size_t)(16 * (n_rows + 32) + 24 * (E + 32)) * 8;
        auto out = [&](double* user, int64_t n) -> double* {
            if (!user) return nullptr;
            if (!host) return user;
            double* d = (size_t)n * 8 <= ARENA_MAX ? io.out_small(R, n, small_cap) : nullptr;
            if (!d) d = io.out(R, user, n);
            outs.push_back({user, d, n});
            return d;
        };
        m.old_rep = (cons || lie) ? out(r->old_rep, n_rows) : nullptr;
        m.this_rep = (cons || lie) ? out(r->this_rep, n_rows) : nullptr;
        m.smooth_rep = (cons || lie) ? out(r->smooth_rep, n_rows) : nullptr;
        m.scores = (cons || lie) ? out(r->scores, n_rows) : nullptr;
        m.na_row = cons ? out(r->na_row, n_rows) : nullptr;
        m.participation_rows = cons ? out(r->participation_rows, n_rows) : nullptr;
        m.relative_part = cons ? out(r->relative_part, n_rows) : nullptr;
        m.reporter_bonus = cons ? out(r->reporter_bonus, n_rows) : nullptr;
        m.adj_first_loadings = cons ? out(r->adj_first_loadings, E) : nullptr;
        m.outcomes_raw = cons ? out(r->outcomes_raw, E) : nullptr;
        m.outcomes_adjusted = cons ? out(r->outcomes_adjusted, E) : nullptr;
        m.outcomes_final = cons ? out(r->outcomes_final, E) : nullptr;
        m.certainty = cons ? out(r->certainty, E) : nullptr;
        m.consensus_reward = cons ? out(r->consensus_reward, E) : nullptr;
        m.nas_filled = cons ? out(r->nas_filled, E) : nullptr;
        m.participation_columns = cons ? out(r->participation_columns, E) : nullptr;
        m.author_bonus = cons ? out(r->author_bonus, E) : nullptr;
        // result.original aliasing the reports (the same pointer): the reference's own `original` is
        // the caller's array rescaled in place (__init__.py:121, 266-269, 584, Q2) -- rescale the
        // scaled columns in place instead of writing a copy of every column (host memory: the
        // device copy of the reports is rescaled and copied back into the caller's array)
        // host memory: `original` is built on the host from the caller's reports while the device
        // works (HostOriginal), not written by the device and copied back
        m.original = (cons || entry == 1) && !inplace && !host_orig_on ? out(r->original, n_rows * E) : nullptr;
        m.orig_inplace = inplace ? 1 : 0;  // (host: the device copy of the reports, for later stages)
        m.rescaled = 0;
        m.filled = (cons || entry == 1) ? out(r->filled, n_rows * E) : nullptr;
        if (host_orig_on && !gated && (inplace || !PCX_ORIG_EARLY)) {  // once the reports' H2D has drained (the caller's array is rewritten in place)
            hipEvent_t ev = nullptr;
            R.hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
            struct EvGuard {
                hipEvent_t e;
                ~EvGuard() { (void)hipEventDestroy(e); }
            } evg{ev};
            R.hip(hipEventRecord(ev, R.st), "hipEventRecord");
            R.hip(hipEventSynchronize(ev), "hipEventSynchronize(H2D)");
            host_orig.start(p->reports, r->original, n_rows, E, sc_h, p->lo, p->hi, p->int_dtype != 0);
        }
        m.weighted_mean = entry == 2 ? out(r->weighted_mean, E) : nullptr;
        m.nc_out = entry == 4 ? out(nc_out, n_rows) : nullptr;
        double* cov_out = entry == 2 ? out(r->covariance, E * E) : nullptr;
        double* ld_out = (entry == 2 || lie) ? out(r->adj_first_loadings, E) : nullptr;
        double* sc_out = entry == 2 ? out(r->scores, n_rows) : nullptr;

        // ---- the kernel view
        m.n_rows = n_rows;
        m.n_events = E;
        m.n_total = N;
        m.row_offset = p->row_offset;
        m.world = world;
        m.rank = rank;
        m.int_dtype = filled_input ? 0 : (p->int_dtype ? 1 : 0);
        m.algorithm = alg;
        m.catch_tolerance = p->catch_tolerance;
        m.alpha = p->alpha;
        m.n_scaled = n_scaled;
        m.sel_phase = 1;
        m.col_blocks = (int32_t)w->col_blocks;
        m.cov_tiles = (int32_t)w->cov_tiles;
        m.cov_kslices = (int32_t)w->cov_kslices;
        m.no_fill = filled_input ? 1 : 0;
        m.rank_rule = entry == 4 ? (rank_rule ? 1 : 0) : (alg == PCX_ALG_PCA ? 1 : 0);
        // numpy/OpenBLAS run np.dot single-threaded below m*n = 9216 (interface/gemv.c: 2304 x
        // GEMM_MULTITHREAD_THRESHOLD): there the reference's summation order is known and replayed
        m.ob_order = (world == 1 && N * E < 9216) ? 1 : 0;
        m.scores_given = (entry == 4 || alg == PCX_ALG_COKURTOSIS) ? 1 : 0;
        m.reports = reports;
        m.scaled = scaled;
        m.lo = lo;
        m.hi = hi;
        m.rep_raw = rep_raw;
        m.scaled_cols = w->scols;
        m.scaled_index = w->sidx;
        m.rep = w->rep;
        m.tok = w->tok;
        m.T = w->T;
        m.part = w->part;
        m.mpart = w->mpart;
        m.cstat = w->cstat;
        m.cmax = w->cmax;
        m.scal = w->scal;
        m.spart = w->spart;
        m.ev = w->ev;
        m.cslab = w->cslab;
        m.C = w->C;
        m.Mw = w->Mw;
        m.pvec = w->pvec;
        m.rowv = w->rowv;
        m.rowstat = w->rowstat;
        m.skey = w->skey;
        m.info = w->info;
        m.sel_state = w->sel_state;
        m.sel_isum = w->sel_isum;
        m.hist_w = w->hist_w;
        m.hist_min = w->hist_min;  // (hist_n, hist_max, sel_imin, sel_imax: select())
        m.sel_arg = w->sel_arg;
        m.sel_act = w->sel_act;
        m.hard = w->hard;
        m.hard_cols = w->hard_cols;
        m.hard_modes = w->hard_modes;
        m.cbuf = w->ccap > 0 ? w->cbuf : nullptr;
        m.vsave = w->vsave;
        m.ccount = w->ccount;
        m.ccap = w->ccap;
        m.scalars = w->scalars;
        m.wcd = w->wcd;
        m.tokp = w->tokp;
        m.wcd_rows = w->wcd_rows;
        m.wcd_ld = w->wcd_ld;
        m.rowpart = w->rowpart;
        m.max_components = p->max_components < 1 ? 1 : (p->max_components > E ? (int32_t)E : p->max_components);
        m.components = -1;
        m.variance_threshold = p->variance_threshold;
        m.aux_scores = aux;
        r->n_hard = 0;
        r->sel_passes = 0;
        r->grid_events = 0;
        r->mixed_int8 = 0;
        r->cov_guard = 0;
        r->cov_guard_cols = 0;
        r->cov_err_bound = 0.0;

        const double* cstat = w->cstat;
        (void)cstat;
        const int64_t cpitch = CS * 2;
        // a1: reputation, tokens (:138-146)
        R.stage(m, M_REPUTATION);
        R.gather_slots(w->scal, 1, SS * 2, 0, SC_BIGTOK_SLOT + 2, w);  // .. SC_MAXTOK
        // a2/a3: rescale + NA + present sums (:266-299)
        R.stage(m, M_COLSTATS);
        R.gather_slots(w->cstat, E, cpitch, 0, 4, w);
        R.gather_block(w->cmax, E * CM * 8);
        R.stage(m, M_GUESS);  // binary fills (:304-309)
        if (!filled_input) select(R, m, w, 1, r);  // scaled fills: weighted median (:300-303)
        if (entry == 1) {      // interpolate: rescaled + filled matrices (:266-313)
            R.stage(m, M_MATRICES);
        } else {
            R.stage(m, M_MEAN);
            const bool wpca = alg == PCX_ALG_PCA || alg == PCX_ALG_BIG_FIVE || alg == PCX_ALG_FIXED_VARIANCE ||
                              clustering;  // the clusterings call wpca too (:393, :408, :422): the loading
            const bool run_wpca = entry == 2 || (entry != 4 && wpca);
            int64_t flags = 0;
            bool mats_written = false;  // k_wcd writes "original" / "filled" on the way
            if (run_wpca) {
                // a5: wcd materialised (:322) in the M_COV_PLAN column order; a6: covariance (:326),
                // general tiles on fp64 MFMA, pure-grid tiles on int8 MFMA; a7: power iteration (:330-336)
                m.cov_perm = w->cov_perm;
                m.cov_pos = w->cov_pos;
                m.zA = w->zA;
                m.zB = w->zB;
                m.zsum = w->zsum;
                m.dscale = w->dscale;
                m.escale = w->dscale + w->wcd_ld;
                R.stage(m, M_COV_PLAN);
                int64_t plan[3];  // general events, mixed pairs on int8, every token the same power of two
                R.hip(hipMemcpyAsync(plan, m.info + INFO_COV_GENERAL, sizeof(plan), hipMemcpyDeviceToHost, R.st),
                      "D2H plan");
                R.sync();
                const int64_t n_general = plan[0];
                const int64_t nb = w->wcd_ld / COV_TILE;
                const int64_t jb = (n_general + COV_TILE - 1) / COV_TILE, gb = jb * COV_TILE;
                m.cov_jb = (int32_t)jb;
                const int64_t np = gb < E ? E - gb : 0;  // grid positions
                m.zq = (np + 255) / 256 * 256;
                r->grid_events = (int32_t)np;  // grid events past the general tiles
                // k-slices of the int8 products: int32-exact row ranges (|tok z z| <= 252,
                // |z d| <= 254 per row) and at least two WGs per CU
                const int64_t nst = w->wcd_rows / 64, tp = (np + 255) / 256, tq = (PCX_NDIG * gb + 255) / 256;
                // one workgroup per CU runs every (tile, k-slice) item for the same time, so the
                // launch takes ceil(items / CUs) rounds of items of 1/k of the rows; each k-slice
                // also writes an int32 slab that k_cov_reduce reads back.  Pick the k in
                // [int32-exact minimum, 32] with the least modelled time: rounds x item time +
                // slab traffic (a C5 shard: k = 2 instead of 26 for the mixed block, 4.6 GB less)
                int ncu = 256;
                (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device);
                auto ks_for = [&](int64_t tiles, int64_t max_rows, double slab_bytes) {
                    tiles = std::max<int64_t>(1, tiles);
                    const int64_t kmin = std::max<int64_t>(1, (w->wcd_rows + max_rows - 1) / max_rows);
                    const int64_t kmax = std::max<int64_t>(kmin, std::min<int64_t>(32, nst));
                    int64_t best = kmin;
                    double best_cost = 1e300;
                    for (int64_t k = kmin; k <= kmax; k++) {
                        const double rounds = (double)((tiles * k + ncu - 1) / ncu);
                        const double cost = rounds / (double)k * (double)nst * GEMM_I8_STAGE_S +
                                            2.0 * (double)k * slab_bytes / SLAB_BW;
                        if (cost < best_cost * (1.0 - 1e-9)) {
                            best_cost = cost;
                            best = k;
                        }
                    }
                    return (int32_t)std::max<int64_t>(1, std::min<int64_t>(best, nst));
                };
                // lower tiles only do work; their slabs hold the lower triangle
                m.ks_gg = ks_for(tp * (tp + 1) / 2, 8000000, 2.0 * (double)np * (double)np);
                m.ks_mx = ks_for(tp * tq, 8000000, 4.0 * (double)np * (double)(PCX_NDIG * gb));  // |z d| <= 254 per row
                if (np > 0 && !w->grow(w->pgg, (size_t)(m.ks_gg * m.zq * m.zq * 4))) {
                    err = "workspace: hipMalloc of the int8 covariance products failed";
                    throw Fail{PCX_ENOMEM};
                }
                m.Pgg = (int32_t*)w->pgg.p;
                // mixed pairs on int8 digits when the bounds are finite and the memory is there
                m.cov_mixed = plan[1] && np > 0 && gb > 0 && w->grow(w->zd, (size_t)(w->wcd_rows * zd_ld(gb))) &&
                                      w->grow(w->pmx, (size_t)(m.ks_mx * m.zq * PCX_NDIG * gb * 4)) &&
                                      w->grow(w->dtok, (size_t)(((PCX_NDIG + G_NSTAT) * gb + 1) * 8))
                                  ? 1
                                  : 0;
                r->mixed_int8 = m.cov_mixed;
                m.zD = (int8_t*)w->zd.p;
                m.dtok = (int64_t*)w->dtok.p;
                // the guard's sums follow the digit sums (zeroed with them); as doubles past the
                // covariance's packed triangle in cslab, so that one SUM exchanges both
                m.gacc = m.cov_mixed ? m.dtok + PCX_NDIG * gb : nullptr;
                m.gsum = m.cov_mixed ? w->cslab + E * (E + 1) / 2 : nullptr;
                m.gg_smax = PCX_NDIG - 1;
                // mixed: the later full passes (M_GEMV2, M_OUTCOMES) read F compactly -- the general
                // positions' filled values (Fg, written by k_wcd), the grid ones from the 2-bit codes
                // and the missing bits (nam) -- instead of the reports (a quarter of the bytes at C5)
                m.compact = m.cov_mixed && w->grow(w->fg, (size_t)(w->wcd_rows * gb * 8)) &&
                                    w->grow(w->nam, (size_t)(w->wcd_rows / 16 * w->wcd_ld * 2))
                                ? 1
                                : 0;
                m.Fg = m.compact ? (double*)w->fg.p : nullptr;
                m.nam = m.compact ? (uint16_t*)w->nam.p : nullptr;
                // the row weights' balanced base-256 digits for the int8-MFMA outcome sums (M_OUTCOMES)
                // (a 256-byte header, then two vectors' digits: pcx_matrix.hip wdig_vec)
                // (and the codes of the grid events the general tiles end with, positions [n_general, gb))
                m.zbg = m.compact && gb >= 128 && w->grow(w->zbg, (size_t)(w->wcd_rows / 16) * 128 * 4)
                            ? (uint32_t*)w->zbg.p
                            : nullptr;
                m.wdig = m.compact && (gb == 0 || m.zbg) && w->grow(w->wdig, 256 + (size_t)w->wcd_rows * 32)
                             ? (int8_t*)w->wdig.p
                             : nullptr;
                // (its header: the weight vectors' largest |w|, noted by k_nweights / k_smooth)
                if (m.wdig) R.hip(hipMemsetAsync(m.wdig, 0, 256, R.st), "hipMemset(wdig)");
                // general x general pairs on int8 digits too (k_gemm_i8x) when the memory is there:
                // 21 digit-pair products on int8 MFMA instead of k_syrk's fp64 tiles
                // (it reads the general positions' F - mu from the compact Fg, so k_wcd writes no wcd)
                if (m.cov_mixed && m.compact) {
                    const int64_t nt = (gb + 255) / 256, npair = gemm_i8x_pairs(PCX_NDIG - 1);
                    // |d e| <= 127^2 per row: int32-exact k-slices of <= 133,143 rows
                    m.ks_gx = ks_for(npair * nt * (nt + 1) / 2, 133120,
                                     4.0 * (double)(npair * nt * (nt + 1) / 2) * 256.0 * 256.0);
                    // every token 2^k (reputation=None: 1 up to 1e6 rows): the digits of w are those of tok w (zD)
                    const bool same = plan[2] != 0;
                    m.cov_gg8 = (same || w->grow(w->ze, (size_t)(w->wcd_rows * zd_ld(gb)))) &&
                                        w->grow(w->pgx, (size_t)(gemm_i8x_slab(m.ks_gx, 0, 0, 0, (int)nt) * 256 * 256 * 4))
                                    ? 1
                                    : 0;
                    m.zE = same ? m.zD : (int8_t*)w->ze.p;
                    m.Pgx = (int32_t*)w->pgx.p;
                }
                m.Pmx = (int32_t*)w->pmx.p;
                r->mixed_int8 = m.cov_mixed ? (m.cov_gg8 ? 3 : 1) : 0;
                m.cov_fp_tiles = (int32_t)(m.cov_gg8     ? 0
                                           : m.cov_mixed ? jb * (jb + 1) / 2
                                                         : jb * nb - jb * (jb - 1) / 2);
                // fp64 slabs: [E][E] for the trapezoid; the mixed triangle's [gb][gb] slabs are
                // small, so it takes more k-slices (~16 WGs per CU) within the same cslab
                m.fp_ld = m.cov_mixed ? gb : E;
                m.fp_ks = (int32_t)w->cov_kslices;
                if (m.cov_mixed && m.cov_fp_tiles > 0) {
                    // k_syrk holds 3 WGs per CU: the k up to `cap` with the least modelled time
                    // (rounds of items of 1/k of the rows + the [gb][gb] slabs' lower halves)
                    const int64_t cap = std::min<int64_t>(w->cov_kslices * E * E / (gb * gb),
                                                          std::max<int64_t>(1, w->wcd_rows / (8 * 8)));
                    const int64_t slots = 3 * (int64_t)ncu, T = m.cov_fp_tiles;
                    const double nst8 = (double)(w->wcd_rows / 8), slab = 4.0 * (double)gb * (double)gb;
                    int64_t best = 1;
                    double best_cost = 1e300;
                    for (int64_t k = 1; k <= cap; k++) {
                        const double cost = (double)((T * k + slots - 1) / slots) / (double)k * nst8 * SYRK_STAGE_S +
                                            2.0 * (double)k * slab / SLAB_BW;
                        if (cost < best_cost * (1.0 - 1e-9)) {
                            best_cost = cost;
                            best = k;
                        }
                    }
                    m.fp_ks = (int32_t)best;
                }
                R.stage(m, M_WCD);
                mats_written = true;
                if (host && cons && m.filled && (size_t)(n_rows * E) * 8 >= STAGE_MIN)
                    early_filled.start(R, r->filled, m.filled, (size_t)(n_rows * E) * 8);
                m.rescaled = m.orig_inplace;  // later stages read the scaled columns rescaled already
                R.stage(m, M_COV);
                R.stage(m, M_COV_I8);
                auto cov_reduce = [&] {
                    R.stage(m, M_COV_REDUCE);
                    if (R.comm) {  // the partial covariance: one SUM of its lower triangle (cslab is free now)
                        R.hip(tri_pack(w->C, w->cslab, E, 0, R.st), "tri pack");
                        // (and the guard's sums, k_guard_stats wrote them past the triangle)
                        R.allreduce(w->cslab, E * (E + 1) / 2 + (m.cov_mixed ? G_NSTAT * gb + 1 : 0), PCX_F64, PCX_SUM);
                        R.hip(tri_pack(w->C, w->cslab, E, 1, R.st), "tri unpack");
                    }
                    R.stage(m, M_COV_FINISH);
                };
                cov_reduce();
                r->cov_guard = 0;
                r->cov_guard_cols = 0;
                r->cov_err_bound = 0.0;
                if (m.cov_mixed) {
                    // the int8 emulation's error bound against the entries (k_cov_guard); above 2^-40
                    // the covariance is recomputed: the remaining digit pairs, or fp64 (k_syrk)
                    R.stage(m, M_COV_GUARD);
                    int64_t gi[3];
                    R.hip(hipMemcpyAsync(gi, m.info + INFO_COV_GUARD, sizeof(gi), hipMemcpyDeviceToHost, R.st),
                          "D2H guard");
                    R.sync();
                    r->cov_guard = (int32_t)gi[0];
                    r->cov_guard_cols = (int32_t)gi[1];
                    std::memcpy(&r->cov_err_bound, &gi[2], 8);
                    if (gi[0] == COV_GUARD_PAIRS) {
                        m.gg_smax = 2 * PCX_NDIG - 2;
                        R.stage(m, M_COV_REST);
                        cov_reduce();
                    } else if (gi[0] == COV_GUARD_FP64) {
                        R.stage(m, M_WCD_REBUILD);  // (reads cov_gg8 as it ran)
                        m.cov_mixed = 0;
                        m.cov_gg8 = 0;
                        m.cov_fp_tiles = (int32_t)(jb * nb - jb * (jb - 1) / 2);
                        m.fp_ld = E;
                        m.fp_ks = (int32_t)w->cov_kslices;
                        R.stage(m, M_COV);
                        cov_reduce();
                        r->mixed_int8 = 0;
                    }
                }
                R.stage(m, M_POWER);
                // big-five / fixed-variance components (:373-390, :429-451); a non-finite
                // covariance makes the reference's second svd raise (Oracle: LinAlgError).  (PCA
                // needs no flags on the host here: no read, no sync)
                if (entry != 2 && alg != PCX_ALG_PCA && !clustering) {
                    flags = R.read(m.info + INFO_FLAGS);
                    if (!(flags & PCX_FLAG_SVD_FAIL)) R.stage(m, M_EIG);
                }
            } else {
                R.stage(m, M_ZERO_LOADING);
            }
            if (entry == 2 && alg != PCX_ALG_PCA) m.algorithm = PCX_ALG_PCA;  // wpca: the first loading's scores
            R.stage(m, M_SCORES);  // also sums the rows' NaN / zero counts (na_row, :549-567)
            R.gather_block(w->skey, 4 * 8);
            if (clustering) {  // the clusterings' scores stay zeros (:357); nc from the clusters
                R.hip(hipMemsetAsync(w->rowv, 0, n_rows * 8, R.st), "hipMemset(scores)");
                cluster_nc(R, m, w, p);
            }
            if (entry == 2) {
                R.stage(m, M_WMEAN_OUT);
                if (cov_out) R.hip(hipMemcpyAsync(cov_out, w->C, E * E * 8, hipMemcpyDeviceToDevice, R.st), "cov");
                if (ld_out) R.hip(hipMemcpyAsync(ld_out, w->ev + 3 * E, E * 8, hipMemcpyDeviceToDevice, R.st), "ld");
                if (sc_out) R.hip(hipMemcpyAsync(sc_out, w->rowv, n_rows * 8, hipMemcpyDeviceToDevice, R.st), "scores");
            } else {
                if ((alg != PCX_ALG_ABSOLUTE && !clustering) || entry == 4) {
                    // a8/a9: sign-choice rule (:487-500; the other algorithms: nonconformity, :475-485)
                    R.stage(m, M_NCSUMS);
                    R.gather_slots(w->scal, 1, SS * 2, 2, 6, w);
                    R.stage(m, M_GEMV2);
                    R.gather_slots(w->cstat, E, cpitch, 4, 6, w);
                    R.stage(m, M_DECIDE);
                }
                if (entry == 4) {
                    R.stage(m, M_NC_OUT);
                } else {
                    // a10: reputation update (:460-472)
                    R.stage(m, M_REPU);
                    R.gather_slots(w->scal, 1, SS * 2, 6, 8, w);
                    R.stage(m, M_SMOOTH);
                    if (lie) {
                        R.stage(m, M_AGENTS);
                        if (ld_out)
                            R.hip(hipMemcpyAsync(ld_out, w->ev + 3 * E, E * 8, hipMemcpyDeviceToDevice, R.st), "ld");
                    } else {
                        // a12-a14: outcomes, participation, certainty (:510-546)
                        R.stage(m, M_OUTCOMES);
                        R.gather_slots(w->cstat, E, cpitch, 6, 14, w);
                        R.hip(hipMemsetAsync(w->hard, 0, E * 4, R.st), "hipMemset(hard)");
                        R.stage(m, M_EVENTS);
                        select(R, m, w, 2, r);  // scaled outcomes: weighted median (:519-523)
                        R.stage(m, M_SCALED_CERT);
                        R.gather_slots(w->cstat, E, cpitch, 14, 16, w);
                        R.stage(m, M_FINAL);
                        R.stage(m, M_ROWSUMS);
                        R.gather_slots(w->scal, 1, SS * 2, 8, 10, w);
                        R.stage(m, M_AGENTS);
                        if (!mats_written) R.stage(m, M_MATRICES);
                    }
                }
            }
        }
        // ---- scalars and host outputs
        int64_t info[4];
        double sc2[2];
        R.hip(hipMemcpyAsync(info, w->info, sizeof(info), hipMemcpyDeviceToHost, R.st), "D2H info");
        R.hip(hipMemcpyAsync(sc2, w->scalars, sizeof(sc2), hipMemcpyDeviceToHost, R.st), "D2H scalars");
        R.mark(M_D2H);
        // the arena's outputs in one copy through the context's pinned buffer, then into place
        const bool arena_pin = io.arena_used > 0 && pin_small(c, io.arena_used);
        if (arena_pin)
            R.hip(hipMemcpyAsync(c->pin_small, io.arena, io.arena_used, hipMemcpyDeviceToHost, R.st), "D2H vectors");
        for (auto& o : outs) {
            const bool in_arena = (char*)o.dev >= io.arena && (char*)o.dev < io.arena + io.arena_cap;
            if (in_arena && arena_pin) continue;
            if ((size_t)o.n * 8 < STAGE_MIN)
                R.hip(hipMemcpyAsync(o.user, o.dev, o.n * 8, hipMemcpyDeviceToHost, R.st), "D2H output");
        }
        const bool early = early_filled.th.joinable();
        if (early && early_filled.join()) R.hip(hipErrorUnknown, "staged D2H of filled");
        for (auto& o : outs)
            if ((size_t)o.n * 8 >= STAGE_MIN && !(early && o.user == r->filled))
                d2h_staged(R, o.user, o.dev, (size_t)o.n * 8);
        R.mark(-1);
        R.sync();
        host_orig.join();
        if (arena_pin)
            for (auto& o : outs)
                if ((char*)o.dev >= io.arena && (char*)o.dev < io.arena + io.arena_cap)
                    memcpy(o.user, (char*)c->pin_small + ((char*)o.dev - io.arena), (size_t)o.n * 8);

        r->participation = sc2[0];
        r->avg_certainty = sc2[1];
        const bool branchless = (alg == PCX_ALG_ABSOLUTE && entry != 4) || clustering || entry == 1 || entry == 2;
        r->branch = branchless ? PCX_BRANCH_NONE : (int32_t)info[INFO_BRANCH];
        r->pi_iters = (int32_t)info[INFO_PI_ITERS];
        r->flags = (int32_t)info[INFO_FLAGS];
        r->components = m.components;
        r->comm_bytes = R.comm_bytes;
        // per-stage device time
        if (c->profile && !R.evs.empty()) {
            for (int k = 0; k < PCX_NSTAGES; k++) c->stage_ms[k] = 0.0;
            for (size_t i = 0; i + 1 < R.evs.size(); i++) {
                if (R.ev_stage[i] < 0) continue;
                float ms = 0.f;
                if (hipEventElapsedTime(&ms, R.evs[i], R.evs[i + 1]) == hipSuccess)
                    c->stage_ms[R.ev_stage[i]] += ms;
            }
        }
        for (hipEvent_t e : R.evs) (void)hipEventDestroy(e);
        return PCX_OK;
    } catch (const Fail& f) {
        (void)hipStreamSynchronize(R.st);
        for (hipEvent_t e : R.evs) (void)hipEventDestroy(e);
        if (err.empty()) err = "single-matrix run failed";
        return f.code;
    } catch (const std::bad_alloc&) {
        err = "out of host memory";
        return PCX_ENOMEM;
    }
}

}  // namespace pcx
