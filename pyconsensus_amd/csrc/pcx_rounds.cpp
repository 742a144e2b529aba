// pcx_rounds.cpp -- batched rounds above the one-wave round kernel's limits (N > 64
// reporters or E > 32 events).
//
// The Monte Carlo regime (README.rst:52-56) loops Oracle(...).consensus()
// (__init__.py:102-611) over many independent rounds.  Rounds up to 64 x 32 are one
// wavefront each (pcx_batched.hip).  Larger rounds run here: each is one single-matrix
// consensus (pcx_runner.cpp, the same kernels and arithmetic as pcx_consensus_f64 on
// that round alone), and a pool of worker threads -- each with its own context, cached
// workspace and non-blocking HIP stream -- keeps many rounds' stage chains in flight on
// the GPU at once, so the per-stage launch and host-sync latency of one round overlaps
// the others.  Rounds are handed out by an atomic counter; the per-round scalars are
// gathered on the host and copied to the caller's [B] arrays once at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "pcx_internal.h"
#include "pcx_sync.h"

namespace pcx {

namespace {
// worker contexts (streams) kept in flight: each round is a chain of ~30 dependent stage
// launches and a few host polls, so throughput grows with the rounds in flight
int pool_size() {
    const char* e = getenv("PCX_ROUND_WORKERS");
    const int n = e ? atoi(e) : 16;
    return std::max(1, std::min(n, 64));
}

double* at(double* base, int64_t off) { return base ? base + off : nullptr; }
}  // namespace

void rounds_free(pcx_ctx* c) {
    for (pcx_ctx* w : c->pool) {
        (void)hipSetDevice(w->device);
        workspace_free(w);
        ctx_host_free(w);  // (a round above SEL_EXACT_MAX rows took the pipelined selection's pinned words)
        if (w->stream) (void)hipStreamDestroy(w->stream);
        delete w;
    }
    c->pool.clear();
}

int run_rounds(pcx_ctx* c, const pcx_batch* in, pcx_batch_result* out, std::string& err) {
    const int64_t B = in->n_rounds, N = in->n_reporters, E = in->n_events;
    if (B == 0) return 0;
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // inputs produced on the caller's stream
    if (e != hipSuccess) {
        err = std::string("rounds: ") + hipGetErrorString(e);
        return PCX_EHIP;
    }
    // workspaces are sized for the most scaled events any round of this batch has (the
    // selection buffers scale with it), not for E
    int max_scaled = 0;
    if (in->scaled) {
        const int64_t rows = in->bounds_shared ? 1 : B;
        std::vector<uint8_t> sc(rows * E);
        e = hipMemcpy(sc.data(), in->scaled, rows * E, hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
            err = std::string("rounds: D2H scaled: ") + hipGetErrorString(e);
            return PCX_EHIP;
        }
        for (int64_t b = 0; b < rows; b++) {
            int n = 0;
            for (int64_t j = 0; j < E; j++) n += sc[b * E + j] != 0;
            max_scaled = std::max(max_scaled, n);
        }
    }
    const int K = (int)std::min<int64_t>(pool_size(), B);
    while ((int)c->pool.size() < K) {
        pcx_ctx* w = new (std::nothrow) pcx_ctx;
        if (!w) {
            err = "rounds: out of host memory";
            return PCX_ENOMEM;
        }
        w->device = c->device;
        e = hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete w;
            err = std::string("rounds: hipStreamCreate: ") + hipGetErrorString(e);
            return PCX_EHIP;
        }
        c->pool.push_back(w);
    }
    std::vector<int32_t> kinit;  // k-means restart rows: device [B][restarts][k] -> host (pcx_problem)
    const int64_t kper = (int64_t)in->kmeans_restarts * in->kmeans_k;
    if (in->algorithm == PCX_ALG_KMEANS) {
        kinit.resize(B * kper);
        e = hipMemcpy(kinit.data(), in->kmeans_init, B * kper * 4, hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
            err = std::string("rounds: D2H kmeans_init: ") + hipGetErrorString(e);
            return PCX_EHIP;
        }
    }
    for (pcx_ctx* w : c->pool) w->scaled_floor = max_scaled;  // one workspace serves every round's bounds
    std::vector<double> part(B), avg(B);
    std::vector<int32_t> branch(B), flags(B), iters(B), comps(B);
    // test hook (pcx_test_inject_enomem): worker k's first round reports PCX_ENOMEM without
    // running, exercising the hand-back below (tests/test_rounds_gpu.py); one call only
    const int fault_k = c->test_enomem_worker;
    c->test_enomem_worker = -1;
    auto one = [&](pcx_ctx* w, int64_t b, std::string& werr) -> int {
            pcx_problem p{};
            p.n_rows = N;
            p.n_events = E;
            p.n_total = N;
            p.row_offset = 0;
            p.reports = in->reports + b * N * E;
            p.reputation = in->reputation ? in->reputation + b * N : nullptr;
            const int64_t bo = in->bounds_shared ? 0 : b * E;
            p.scaled = in->scaled ? in->scaled + bo : nullptr;
            p.lo = in->scaled ? in->lo + bo : nullptr;
            p.hi = in->scaled ? in->hi + bo : nullptr;
            p.catch_tolerance = in->catch_tolerance;
            p.alpha = in->alpha;
            p.int_dtype = in->int_dtype;
            p.algorithm = in->algorithm;
            p.max_components = in->max_components;
            p.mem_kind = PCX_MEM_DEVICE;
            p.variance_threshold = in->variance_threshold;
            p.aux_scores = in->aux_scores ? in->aux_scores + b * N : nullptr;
            p.hierarchy_threshold = in->hierarchy_threshold;
            p.cluster_threshold = in->cluster_threshold;
            p.kmeans_k = in->kmeans_k;
            p.kmeans_restarts = in->kmeans_restarts;
            p.kmeans_init = kinit.empty() ? nullptr : kinit.data() + b * kper;
            pcx_result r{};
            r.old_rep = at(out->old_rep, b * N);
            r.this_rep = at(out->this_rep, b * N);
            r.smooth_rep = at(out->smooth_rep, b * N);
            r.scores = at(out->scores, b * N);
            r.na_row = at(out->na_row, b * N);
            r.participation_rows = at(out->participation_rows, b * N);
            r.relative_part = at(out->relative_part, b * N);
            r.reporter_bonus = at(out->reporter_bonus, b * N);
            r.adj_first_loadings = at(out->adj_first_loadings, b * E);
            r.outcomes_raw = at(out->outcomes_raw, b * E);
            r.outcomes_adjusted = at(out->outcomes_adjusted, b * E);
            r.outcomes_final = at(out->outcomes_final, b * E);
            r.certainty = at(out->certainty, b * E);
            r.consensus_reward = at(out->consensus_reward, b * E);
            r.nas_filled = at(out->nas_filled, b * E);
            r.participation_columns = at(out->participation_columns, b * E);
            r.author_bonus = at(out->author_bonus, b * E);
            r.original = at(out->original, b * N * E);
            r.filled = at(out->filled, b * N * E);
            const int rc = run_matrix(w, &p, &r, 0, nullptr, 0, nullptr, werr);
            if (rc) return rc;
            part[b] = r.participation;
            avg[b] = r.avg_certainty;
            branch[b] = r.branch;
            flags[b] = r.flags;
            iters[b] = r.pi_iters;
            comps[b] = r.components;
            return 0;
    };
    // a worker whose workspace does not fit (PCX_ENOMEM) leaves the pool and hands its round
    // back: fewer rounds run in flight instead of the batch failing (pcx_sync.h)
    std::vector<char> faulted(K, 0);
    std::vector<int64_t> retry;
    const int rc = schedule_rounds(
        K, B, PCX_ENOMEM,
        [&](int k, int64_t b, std::string& werr) -> int {
            if (k == fault_k && !faulted[k]) {
                faulted[k] = 1;
                werr = "injected PCX_ENOMEM (pcx_test_inject_enomem)";
                return PCX_ENOMEM;
            }
            return one(c->pool[k], b, werr);
        },
        [&](int k) { workspace_free(c->pool[k]); }, retry, err);
    if (rc) return rc;
    // the handed-back rounds, one at a time on a context whose workspace is resident
    for (int64_t b : retry) {
        pcx_ctx* w = c->pool[0];
        for (pcx_ctx* q : c->pool)
            if (q->ws) {
                w = q;
                break;
            }
        std::string werr;
        if (const int rb = one(w, b, werr)) {
            err = "round " + std::to_string(b) + ": " + werr;
            return rb;
        }
    }
    (void)hipSetDevice(c->device);
    auto put = [&](void* dst, const void* src, size_t bytes) {
        if (dst && e == hipSuccess) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream);
    };
    put(out->participation, part.data(), B * 8);
    put(out->avg_certainty, avg.data(), B * 8);
    put(out->branch, branch.data(), B * 4);
    put(out->flags, flags.data(), B * 4);
    put(out->pi_iters, iters.data(), B * 4);
    put(out->components, comps.data(), B * 4);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // the host arrays die with this call
    if (e != hipSuccess) {
        err = std::string("rounds: scalar copy: ") + hipGetErrorString(e);
        return PCX_EHIP;
    }
    return 0;
}

}  // namespace pcx
