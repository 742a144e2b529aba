// pcx_api.cpp -- the extern "C" boundary of libpcx (declared in include/pcx.h).
// Host-side validation, context/stream management and kernel launches; no
// compute happens here.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>
#include <cstdlib>

#include "../../include/pcx.h"
#include "pcx_internal.h"
#include "pcx_seqsum.h"

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(PCX_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

extern "C" {

int pcx_abi_version(void) { return PCX_ABI_VERSION; }

const char* pcx_last_error(void) { return g_err.c_str(); }

namespace {
pcx_ctx* new_ctx(int device_id, const char* who) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || device_id < 0 || device_id >= n) {
        g_err = std::string(who) + ": no HIP device " + std::to_string(device_id);
        return nullptr;
    }
    pcx_ctx* c = new (std::nothrow) pcx_ctx;
    if (!c) {
        g_err = std::string(who) + ": out of host memory";
        return nullptr;
    }
    c->device = device_id;
    return c;
}

pcx_ctx* with_comm(pcx_ctx* c, pcx::Comm* comm, const std::string& err) {
    if (!c) return nullptr;
    if (!comm) {
        g_err = err.empty() ? "communicator setup failed" : err;
        delete c;
        return nullptr;
    }
    c->comm = comm;
    return c;
}
}  // namespace

pcx_ctx* pcx_create(int device_id) { return new_ctx(device_id, "pcx_create"); }

int pcx_comm_unique_id(pcx_comm_id* out) {
    if (!out) return fail(PCX_EINVAL, "pcx_comm_unique_id: null argument");
    std::string err;
    const int rc = pcx::comm_rccl_unique_id(out, err);
    return rc ? fail(rc, err) : PCX_OK;
}

pcx_ctx* pcx_create_rank(int device_id, int world, int rank, const pcx_comm_id* id) {
    if (!id || world < 1 || rank < 0 || rank >= world) {
        g_err = "pcx_create_rank: bad id / world / rank";
        return nullptr;
    }
    pcx_ctx* c = new_ctx(device_id, "pcx_create_rank");
    if (!c) return nullptr;
    std::string err;  // world == 1 too: a one-rank RCCL communicator (every exchange still runs)
    return with_comm(c, pcx::comm_rccl(device_id, world, rank, id, err), err);
}

pcx_group* pcx_group_create(int world) {
    pcx_group* g = pcx::group_create(world);
    if (!g) g_err = "pcx_group_create: world must be >= 1";
    return g;
}

void pcx_group_destroy(pcx_group* g) { pcx::group_destroy(g); }

pcx_ctx* pcx_create_grouped(int device_id, pcx_group* g, int rank) {
    pcx_ctx* c = new_ctx(device_id, "pcx_create_grouped");
    if (!c) return nullptr;
    std::string err;
    return with_comm(c, pcx::comm_group(g, rank, err), err);
}

pcx_ctx* pcx_create_custom(int device_id, int world, int rank, const pcx_comm_ops* ops) {
    pcx_ctx* c = new_ctx(device_id, "pcx_create_custom");
    if (!c) return nullptr;
    std::string err;
    return with_comm(c, pcx::comm_custom(world, rank, ops, err), err);
}

int pcx_ctx_world(const pcx_ctx* ctx) { return ctx && ctx->comm ? ctx->comm->world : 1; }
int pcx_ctx_rank(const pcx_ctx* ctx) { return ctx && ctx->comm ? ctx->comm->rank : 0; }

int pcx_release_workspace(pcx_ctx* ctx) {
    if (!ctx) return fail(PCX_EINVAL, "pcx_release_workspace: null context");
    (void)hipSetDevice(ctx->device);
    pcx::workspace_free(ctx);
    return PCX_OK;
}

void pcx_destroy(pcx_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    pcx::workspace_free(ctx);
    delete ctx->comm;
    delete ctx;
}

int pcx_set_stream(pcx_ctx* ctx, void* s) {
    if (!ctx) return fail(PCX_EINVAL, "pcx_set_stream: null context");
    ctx->stream = reinterpret_cast<hipStream_t>(s);
    return PCX_OK;
}

int pcx_synchronize(pcx_ctx* ctx) {
    if (!ctx) return fail(PCX_EINVAL, "pcx_synchronize: null context");
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e == hipSuccess ? PCX_OK : hip_fail(e, "pcx_synchronize");
}

int pcx_consensus_batched_f64(pcx_ctx* ctx, const pcx_batch* in, pcx_batch_result* out) {
    if (!ctx || !in || !out) return fail(PCX_EINVAL, "pcx_consensus_batched_f64: null argument");
    if (in->n_rounds < 0 || in->n_rounds > 0x7fffffff)
        return fail(PCX_EINVAL, "batched: n_rounds must be in [0, 2^31)");
    if (in->n_reporters < 1 || in->n_reporters > 64)
        return fail(PCX_EINVAL, "batched: n_reporters must be in [1, 64]");
    if (in->n_events < 1 || in->n_events > 32) return fail(PCX_EINVAL, "batched: n_events must be in [1, 32]");
    if (!in->reports) return fail(PCX_EINVAL, "batched: reports is NULL");
    if (in->scaled && (!in->lo || !in->hi)) return fail(PCX_EINVAL, "batched: scaled given without lo/hi");
    if (in->algorithm < PCX_ALG_PCA || in->algorithm > PCX_ALG_CLUSTERFECK)
        return fail(PCX_EINVAL, "batched: algorithm must be an enum pcx_algorithm value (0..7)");
    if (in->algorithm == PCX_ALG_KMEANS &&
        (!in->kmeans_init || in->kmeans_k < 1 || in->kmeans_k > 8 || in->kmeans_k > in->n_reporters ||
         in->kmeans_restarts < 1))
        return fail(PCX_EINVAL, "batched: k-means needs kmeans_init and 1 <= kmeans_k <= min(N, 8), restarts >= 1");
    if (in->algorithm == PCX_ALG_HIERARCHICAL && std::isnan(in->hierarchy_threshold))
        return fail(PCX_EINVAL, "batched: hierarchy_threshold is NaN");
    if (in->algorithm == PCX_ALG_BIG_FIVE && (in->max_components < 1 || in->max_components > in->n_events))
        return fail(PCX_EINVAL, "batched: big-five needs 1 <= max_components <= n_events");
    if (in->algorithm == PCX_ALG_FIXED_VARIANCE && !std::isfinite(in->variance_threshold))
        return fail(PCX_EINVAL, "batched: variance_threshold must be finite");
    if (in->algorithm == PCX_ALG_COKURTOSIS && !in->aux_scores)
        return fail(PCX_EINVAL, "batched: cokurtosis needs aux_scores (aux[\"cokurt\"])");
    if (!std::isfinite(in->catch_tolerance) || !std::isfinite(in->alpha))
        return fail(PCX_EINVAL, "batched: catch_tolerance/alpha must be finite");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    pcx::BatchArgs a{};
    a.B = in->n_rounds;
    a.N = (int)in->n_reporters;
    a.E = (int)in->n_events;
    a.ES = a.E | 1;
    a.reports = in->reports;
    a.reputation = in->reputation;
    a.scaled = in->scaled;
    a.lo = in->lo;
    a.hi = in->hi;
    a.bounds_shared = in->bounds_shared;
    a.int_dtype = in->int_dtype;
    a.algorithm = in->algorithm;
    a.max_components = in->max_components;
    a.variance_threshold = in->variance_threshold;
    a.aux_scores = in->aux_scores;
    a.hierarchy_threshold = in->hierarchy_threshold;
    a.cluster_threshold = in->cluster_threshold;
    a.kmeans_k = in->kmeans_k;
    a.kmeans_restarts = in->kmeans_restarts;
    a.kmeans_init = in->kmeans_init;
    a.catch_tol = in->catch_tolerance;
    a.alpha = in->alpha;
    a.old_rep = out->old_rep;
    a.this_rep = out->this_rep;
    a.smooth_rep = out->smooth_rep;
    a.scores = out->scores;
    a.na_row = out->na_row;
    a.participation_rows = out->participation_rows;
    a.relative_part = out->relative_part;
    a.reporter_bonus = out->reporter_bonus;
    a.adj_first_loadings = out->adj_first_loadings;
    a.outcomes_raw = out->outcomes_raw;
    a.outcomes_adjusted = out->outcomes_adjusted;
    a.outcomes_final = out->outcomes_final;
    a.certainty = out->certainty;
    a.consensus_reward = out->consensus_reward;
    a.nas_filled = out->nas_filled;
    a.participation_columns = out->participation_columns;
    a.author_bonus = out->author_bonus;
    a.participation = out->participation;
    a.avg_certainty = out->avg_certainty;
    a.branch = out->branch;
    a.flags = out->flags;
    a.pi_iters = out->pi_iters;
    a.components = out->components;
    a.original = out->original;
    a.filled = out->filled;
    const char* st_env = getenv("PCX_STAMPS");
    if (st_env && st_env[0] == '1' && a.B > 0) {  // diagnostic: per-phase clock breakdown
        long long* d = nullptr;
        if (hipMalloc(&d, a.B * 32 * sizeof(long long)) == hipSuccess) {
            (void)hipMemsetAsync(d, 0, a.B * 32 * sizeof(long long), ctx->stream);
            a.stamps = d;
        }
    }
    e = pcx::launch_batched(a, ctx->stream);
    if (a.stamps) {
        // stamp ids in program order (pcx_batched.hip STAMP(k)); a phase is named by its closing stamp
        static const int order[] = {0, 1, 2, 13, 14, 3, 4, 5, 6, 7, 8, 15, 16, 9, 10, 11, 12};
        const int no = (int)(sizeof(order) / sizeof(order[0]));
        std::vector<long long> h(a.B * 32);
        (void)hipMemcpyAsync(h.data(), a.stamps, h.size() * sizeof(long long), hipMemcpyDeviceToHost, ctx->stream);
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(a.stamps);
        double acc[32] = {0};
        for (int64_t b = 0; b < a.B; b++)
            for (int k = 1; k < no; k++) {
                const long long t1 = h[b * 32 + order[k]], t0 = h[b * 32 + order[k - 1]];
                if (t1 && t0) acc[order[k]] += (double)(t1 - t0);
            }
        fprintf(stderr, "PCX_STAMPS mean cycles per phase:");
        for (int k = 1; k < no; k++) fprintf(stderr, " %d:%.0f", order[k], acc[order[k]] / (double)a.B);
        double sort = 0, walk = 0;
        for (int64_t b = 0; b < a.B; b++) {
            sort += (double)h[b * 32 + 20];
            walk += (double)h[b * 32 + 21];
        }
        fprintf(stderr, " median_sort:%.0f median_walk:%.0f\n", sort / (double)a.B, walk / (double)a.B);
    }
    return e == hipSuccess ? PCX_OK : hip_fail(e, "batched_round_kernel launch");
}

namespace {
int run(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r, int entry, const double* scores, int rank_rule, double* nc,
        const char* who) {
    if (!ctx || !p || !r) return fail(PCX_EINVAL, std::string(who) + ": null argument");
    std::string err;
    const int rc = pcx::run_matrix(ctx, p, r, entry, scores, rank_rule, nc, err);
    return rc ? fail(rc, std::string(who) + ": " + err) : PCX_OK;
}
}  // namespace

int pcx_consensus_f64(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r) {
    return run(ctx, p, r, 0, nullptr, 0, nullptr, "pcx_consensus_f64");
}

int pcx_interpolate_f64(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r) {
    return run(ctx, p, r, 1, nullptr, 0, nullptr, "pcx_interpolate_f64");
}

int pcx_wpca_f64(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r) {
    return run(ctx, p, r, 2, nullptr, 0, nullptr, "pcx_wpca_f64");
}

int pcx_lie_detector_f64(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r) {
    return run(ctx, p, r, 3, nullptr, 0, nullptr, "pcx_lie_detector_f64");
}

int pcx_nonconformity_f64(pcx_ctx* ctx, const pcx_problem* p, const double* scores, int rank_rule, double* nc,
                          pcx_result* r) {
    if (!scores || !nc) return fail(PCX_EINVAL, "pcx_nonconformity_f64: scores and nc are required");
    return run(ctx, p, r, 4, scores, rank_rule, nc, "pcx_nonconformity_f64");
}

int pcx_profile_enable(pcx_ctx* ctx, int on) {
    if (!ctx) return fail(PCX_EINVAL, "pcx_profile_enable: null context");
    ctx->profile = on ? 1 : 0;
    return PCX_OK;
}

int pcx_profile_read(pcx_ctx* ctx, double* ms) {
    if (!ctx || !ms) return fail(PCX_EINVAL, "pcx_profile_read: null argument");
    for (int k = 0; k < PCX_NSTAGES; k++) ms[k] = ctx->stage_ms[k];
    return PCX_OK;
}

const char* pcx_stage_name(int k) { return pcx::stage_name(k); }

double pcx_seqsum_const(double c, int64_t k) { return pcx::seqsum_const(c, k); }

int64_t pcx_seqsum_first_above(double c, double t, int64_t kmax) { return pcx::seqsum_first_above(c, t, kmax); }

}  // extern "C"
