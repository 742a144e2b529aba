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
#include <atomic>
#include <thread>
#include <algorithm>

#include "../../include/pcx.h"
#include "pcx_internal.h"
#include "pcx_sync.h"
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

pcx_ctx* pcx_create_devices(int n_devices, const int* device_ids) {
    if (n_devices < 1 || !device_ids) {
        g_err = "pcx_create_devices: need n_devices >= 1 and device_ids";
        return nullptr;
    }
    pcx_ctx* c = new_ctx(device_ids[0], "pcx_create_devices");
    if (!c) return nullptr;
    for (int k = 1; k < n_devices; k++) {
        pcx_ctx* probe = new_ctx(device_ids[k], "pcx_create_devices");
        if (!probe) {
            delete c;
            return nullptr;
        }
        delete probe;
    }
    bool distinct = true;
    for (int a = 0; a < n_devices; a++)
        for (int b = a + 1; b < n_devices; b++) distinct = distinct && device_ids[a] != device_ids[b];
    std::string err;
    std::vector<pcx::Comm*> comms;
    if (distinct) {
        const int rc = pcx::comm_rccl_all(n_devices, device_ids, comms, err);
        if (rc) {
            g_err = "pcx_create_devices: " + err;
            delete c;
            return nullptr;
        }
    } else {
        c->group = pcx::group_create(n_devices);
        for (int k = 0; k < n_devices && c->group; k++) comms.push_back(pcx::comm_group(c->group, k, err));
    }
    for (int k = 0; k < n_devices; k++) {
        pcx_ctx* s = (k < (int)comms.size() && comms[k]) ? new (std::nothrow) pcx_ctx : nullptr;
        if (s) {
            s->device = device_ids[k];
            s->comm = comms[k];
        } else if (k < (int)comms.size()) {
            delete comms[k];
        }
        c->sub.push_back(s);
    }
    for (pcx_ctx* s : c->sub)
        if (!s) {
            g_err = "pcx_create_devices: communicator setup failed" + (err.empty() ? std::string() : ": " + err);
            pcx_destroy(c);
            return nullptr;
        }
    return c;
}

int pcx_ctx_world(const pcx_ctx* ctx) {
    if (ctx && !ctx->sub.empty()) return (int)ctx->sub.size();
    return ctx && ctx->comm ? ctx->comm->world : 1;
}
int pcx_ctx_rank(const pcx_ctx* ctx) { return ctx && ctx->comm ? ctx->comm->rank : 0; }

int pcx_ctx_usable(const pcx_ctx* ctx) {
    if (!ctx) return 0;
    if (ctx->comm && ctx->comm->aborted) return 0;
    for (const pcx_ctx* s : ctx->sub)
        if (s->comm && s->comm->aborted) return 0;
    return 1;
}

int pcx_release_workspace(pcx_ctx* ctx) {
    if (!ctx) return fail(PCX_EINVAL, "pcx_release_workspace: null context");
    for (pcx_ctx* s : ctx->sub) pcx_release_workspace(s);
    pcx::rounds_free(ctx);
    (void)hipSetDevice(ctx->device);
    pcx::workspace_free(ctx);
    pcx::io_bufs_free(ctx);
    return PCX_OK;
}

}  // extern "C"
namespace pcx {
void ctx_host_free(pcx_ctx* c) {
    if (c->mscr) (void)hipFree(c->mscr);
    c->mscr = nullptr;
    c->mscr_bytes = 0;
    if (c->pinned) (void)hipHostFree(c->pinned);
    c->pinned = nullptr;
    c->pinned_bytes = 0;
    if (c->sel_pin) (void)hipHostFree(c->sel_pin);
    c->sel_pin = nullptr;
    if (c->pin_small) (void)hipHostFree(c->pin_small);
    c->pin_small = nullptr;
    c->pin_small_bytes = 0;
    for (hipEvent_t& ev : c->sel_ev) {
        if (ev) (void)hipEventDestroy(ev);
        ev = nullptr;
    }
    if (c->side_stream) (void)hipStreamDestroy(c->side_stream);
    c->side_stream = nullptr;
    io_bufs_free(c);
}
void io_bufs_free(pcx_ctx* c) {
    for (auto& b : c->io_bufs)
        if (b.first) (void)hipFree(b.first);
    c->io_bufs.clear();
}
}  // namespace pcx
extern "C" {

void pcx_destroy(pcx_ctx* ctx) {
    if (!ctx) return;
    for (pcx_ctx* s : ctx->sub) pcx_destroy(s);
    if (ctx->group) pcx::group_destroy(ctx->group);
    pcx::rounds_free(ctx);
    (void)hipSetDevice(ctx->device);
    pcx::ctx_host_free(ctx);
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
    if (in->n_reporters < 1 || in->n_reporters > 0x7fffffff)
        return fail(PCX_EINVAL, "batched: n_reporters must be in [1, 2^31)");
    if (in->n_events < 1 || in->n_events > 65536) return fail(PCX_EINVAL, "batched: n_events must be in [1, 65536]");
    const bool large = in->n_reporters > 64 || in->n_events > 32;  // beyond one wavefront per round
    if (!in->reports) return fail(PCX_EINVAL, "batched: reports is NULL");
    if (in->scaled && (!in->lo || !in->hi)) return fail(PCX_EINVAL, "batched: scaled given without lo/hi");
    if (in->algorithm < PCX_ALG_PCA || in->algorithm > PCX_ALG_CLUSTERFECK)
        return fail(PCX_EINVAL, "batched: algorithm must be an enum pcx_algorithm value (0..7)");
    if (in->algorithm == PCX_ALG_KMEANS &&
        (!in->kmeans_init || in->kmeans_k < 1 || in->kmeans_k > (large ? 1024 : 8) || in->kmeans_k > in->n_reporters ||
         in->kmeans_restarts < 1))
        return fail(PCX_EINVAL, "batched: k-means needs kmeans_init and 1 <= kmeans_k <= min(N, 8; 1024 above 64 x 32), "
                                "restarts >= 1");
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
    if (large) {
        if (pcx::medium_fits(a) && !getenv("PCX_NO_MEDIUM")) {
            // one workgroup per round (pcx_medium.hip), in chunks of bounded scratch
            const size_t cap = (size_t)2 << 30;
            const int64_t chunk = pcx::medium_chunk(a, cap);
            const size_t per = ((a.filled ? 0 : (size_t)a.N * a.E) + (size_t)a.E * a.E) * sizeof(double);
            const size_t need = per * (size_t)chunk;
            if (ctx->mscr_bytes < need) {
                if (ctx->mscr) (void)hipFree(ctx->mscr);
                ctx->mscr = nullptr;
                ctx->mscr_bytes = 0;
                e = hipMalloc(&ctx->mscr, need);
                if (e != hipSuccess) return hip_fail(e, "hipMalloc(medium scratch)");
                ctx->mscr_bytes = need;
            }
            double* Fscr = (double*)ctx->mscr;
            double* Cscr = Fscr + (a.filled ? 0 : (size_t)chunk * a.N * a.E);
            const char* mst = getenv("PCX_STAMPS");
            if (mst && mst[0] == '1') {  // diagnostic: per-phase clock breakdown
                long long* d = nullptr;
                if (hipMalloc(&d, a.B * 32 * sizeof(long long)) == hipSuccess) {
                    (void)hipMemsetAsync(d, 0, a.B * 32 * sizeof(long long), ctx->stream);
                    a.stamps = d;
                }
            }
            for (int64_t b0 = 0; b0 < a.B && e == hipSuccess; b0 += chunk)
                e = pcx::launch_medium(a, b0, std::min<int64_t>(chunk, a.B - b0), Fscr, Cscr, ctx->stream);
            if (a.stamps) {  // stamps 0..15 in program order (pcx_medium.hip MSTAMP(k))
                std::vector<long long> h(a.B * 32);
                (void)hipMemcpyAsync(h.data(), a.stamps, h.size() * sizeof(long long), hipMemcpyDeviceToHost,
                                     ctx->stream);
                (void)hipStreamSynchronize(ctx->stream);
                (void)hipFree(a.stamps);
                double acc[16] = {0};
                for (int64_t b = 0; b < a.B; b++)
                    for (int k = 1, prev = 0; k < 16; k++) {
                        const long long t1 = h[b * 32 + k], t0 = h[b * 32 + prev];
                        if (t1 && t0) {
                            acc[k] += (double)(t1 - t0);
                            prev = k;
                        }
                    }
                fprintf(stderr, "PCX_STAMPS medium mean cycles per phase:");
                for (int k = 1; k < 16; k++) fprintf(stderr, " %d:%.0f", k, acc[k] / (double)a.B);
                double mp[3] = {0, 0, 0};  // wave 0's outcome medians: total+dom, rank, walk
                for (int64_t b = 0; b < a.B; b++)
                    for (int k = 0; k < 3; k++) mp[k] += (double)h[b * 32 + 20 + k];
                fprintf(stderr, " wave0 medians total:%.0f rank:%.0f walk:%.0f", mp[0] / (double)a.B,
                        mp[1] / (double)a.B, mp[2] / (double)a.B);
                double sub[4] = {0, 0, 0, 0};  // the nonconformity phase's steps (stamps 24-27 after 8)
                for (int64_t b = 0; b < a.B; b++)
                    for (int k = 0; k < 4; k++) {
                        const long long t1 = h[b * 32 + 24 + k], t0 = h[b * 32 + (k ? 23 + k : 8)];
                        if (t1 && t0) sub[k] += (double)(t1 - t0);
                    }
                fprintf(stderr, " nc: minmax+norm:%.0f n12:%.0f dots:%.0f ranks:%.0f", sub[0] / (double)a.B,
                        sub[1] / (double)a.B, sub[2] / (double)a.B, sub[3] / (double)a.B);
                double pw[2] = {0, 0};  // power iteration: presquares (6 -> 28), steps (28 -> 29)
                for (int64_t b = 0; b < a.B; b++) {
                    const long long* hb = &h[b * 32];
                    if (hb[28] && hb[6]) pw[0] += (double)(hb[28] - hb[6]);
                    if (hb[29] && hb[28]) pw[1] += (double)(hb[29] - hb[28]);
                }
                fprintf(stderr, " pi: presq:%.0f steps:%.0f\n", pw[0] / (double)a.B, pw[1] / (double)a.B);
            }
            return e == hipSuccess ? PCX_OK : hip_fail(e, "medium_round_kernel launch");
        }
        // one single-matrix consensus per round, many rounds in flight (pcx_rounds.cpp)
        std::string err;
        const int rc = pcx::run_rounds(ctx, in, out, err);
        return rc ? fail(rc, "pcx_consensus_batched_f64: " + err) : PCX_OK;
    }
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
// pcx_create_devices context: shard the host matrix's rows over the devices, one
// worker thread per device running the rank's consensus (collective over the ranks)
int run_devices(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r, int entry, const double* scores, int rank_rule,
                double* nc, std::string& err) {
    const int n = (int)ctx->sub.size();
    const int64_t N = p->n_rows, E = p->n_events;
    if (p->mem_kind != PCX_MEM_HOST) {
        err = "a multi-device context takes the matrix in host memory (PCX_MEM_HOST)";
        return PCX_EINVAL;
    }
    if (p->n_total != N || p->row_offset != 0) {
        err = "a multi-device context takes the whole matrix (n_total == n_rows, row_offset 0)";
        return PCX_EINVAL;
    }
    if (N < n || E < 1 || !p->reports) {
        err = "bad shape (fewer rows than devices) or missing reports";
        return PCX_EINVAL;
    }
    // the rank-independent checks once, here: a bad argument fails before any worker starts,
    // so it never takes the abort path below (which leaves an RCCL context unusable)
    if (const int rc = pcx::check_problem(p, n, entry, err)) return rc;
    std::vector<pcx_problem> ps(n, *p);
    std::vector<pcx_result> rs(n);
    std::vector<std::string> errs(n);
    std::vector<int> rcs;
    const int64_t base = N / n, rem = N % n;
    auto at = [](double* a, int64_t off) { return a ? a + off : nullptr; };
    for (int k = 0; k < n; k++) {
        const int64_t off = k * base + (k < rem ? k : rem), cnt = base + (k < rem ? 1 : 0);
        pcx_problem& q = ps[k];
        q.n_rows = cnt;
        q.n_total = N;
        q.row_offset = off;
        q.reports = p->reports + off * E;
        q.aux_scores = p->aux_scores ? p->aux_scores + off : nullptr;
        pcx_result& o = rs[k];
        o = pcx_result{};
        o.old_rep = at(r->old_rep, off);
        o.this_rep = at(r->this_rep, off);
        o.smooth_rep = at(r->smooth_rep, off);
        o.scores = at(r->scores, off);
        o.na_row = at(r->na_row, off);
        o.participation_rows = at(r->participation_rows, off);
        o.relative_part = at(r->relative_part, off);
        o.reporter_bonus = at(r->reporter_bonus, off);
        o.original = at(r->original, off * E);
        o.filled = at(r->filled, off * E);
        if (k == 0) {  // event vectors are identical on every rank: device 0 writes them
            o.adj_first_loadings = r->adj_first_loadings;
            o.outcomes_raw = r->outcomes_raw;
            o.outcomes_adjusted = r->outcomes_adjusted;
            o.outcomes_final = r->outcomes_final;
            o.certainty = r->certainty;
            o.consensus_reward = r->consensus_reward;
            o.nas_filled = r->nas_filled;
            o.participation_columns = r->participation_columns;
            o.author_bonus = r->author_bonus;
            o.weighted_mean = r->weighted_mean;
            o.covariance = r->covariance;
        }
    }
    // the first failing worker releases the ranks waiting on it in an exchange: it aborts every
    // other rank's communicator (RCCL: ncclCommAbort; group: pcx_group::abort)
    pcx::run_workers(
        n,
        [&](int k) {
            const int64_t off = ps[k].row_offset;
            return pcx::run_matrix(ctx->sub[k], &ps[k], &rs[k], entry, scores ? scores + off : nullptr, rank_rule,
                                   nc ? nc + off : nullptr, errs[k]);
        },
        [&](int k) {
            if (ctx->group) pcx::group_abort(ctx->group);
            for (pcx_ctx* o : ctx->sub)
                if (o->comm && o != ctx->sub[k]) o->comm->abort();
        },
        rcs);
    if (ctx->group) pcx::group_reset(ctx->group);  // every worker has left the exchange
    int first = -1;
    for (int k = 0; k < n && first < 0; k++)
        if (rcs[k] && errs[k].find("exchange aborted") == std::string::npos) first = k;
    for (int k = first < 0 ? 0 : first; k < n; k++)
        if (rcs[k]) {
            err = "device " + std::to_string(ctx->sub[k]->device) + " (rank " + std::to_string(k) + "): " + errs[k];
            return rcs[k];
        }
    double bytes = 0;
    for (int k = 0; k < n; k++) bytes += rs[k].comm_bytes;
    const pcx_result& z = rs[0];
    r->participation = z.participation;
    r->avg_certainty = z.avg_certainty;
    r->branch = z.branch;
    r->flags = z.flags;
    r->pi_iters = z.pi_iters;
    r->components = z.components;
    r->n_hard = z.n_hard;
    r->sel_passes = z.sel_passes;
    r->comm_bytes = bytes;
    r->grid_events = z.grid_events;
    r->mixed_int8 = z.mixed_int8;
    return 0;
}

int run(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r, int entry, const double* scores, int rank_rule, double* nc,
        const char* who) {
    if (!ctx || !p || !r) return fail(PCX_EINVAL, std::string(who) + ": null argument");
    std::string err;
    if (!ctx->sub.empty()) {
        const int rc = run_devices(ctx, p, r, entry, scores, rank_rule, nc, err);
        return rc ? fail(rc, std::string(who) + ": " + err) : PCX_OK;
    }
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
    for (pcx_ctx* s : ctx->sub) s->profile = on ? 1 : 0;
    ctx->profile = on ? 1 : 0;
    return PCX_OK;
}

int pcx_profile_read(pcx_ctx* ctx, double* ms) {
    if (!ctx || !ms) return fail(PCX_EINVAL, "pcx_profile_read: null argument");
    const pcx_ctx* src = ctx->sub.empty() ? ctx : ctx->sub[0];  // multi-device: device 0's stages
    for (int k = 0; k < PCX_NSTAGES; k++) ms[k] = src->stage_ms[k];
    return PCX_OK;
}

const char* pcx_stage_name(int k) { return pcx::stage_name(k); }

int pcx_ctx_progress(const pcx_ctx* ctx, int* stage, int* host_waiting) {
    if (!ctx || !stage || !host_waiting) return fail(PCX_EINVAL, "pcx_ctx_progress: null argument");
    const pcx_ctx* src = ctx->sub.empty() ? ctx : ctx->sub[0];
    *stage = src->progress_stage.load(std::memory_order_relaxed);
    *host_waiting = src->progress_wait.load(std::memory_order_relaxed);
    return PCX_OK;
}

double pcx_seqsum_const(double c, int64_t k) { return pcx::seqsum_const(c, k); }

int64_t pcx_seqsum_first_above(double c, double t, int64_t kmax) { return pcx::seqsum_first_above(c, t, kmax); }
int pcx_mixed_digits(void) { return PCX_NDIG; }
int pcx_rccl_version(int* runtime, int* compiled) { return pcx::rccl_version(runtime, compiled); }
int pcx_selftest_abort_once(int users, int aborters, int iters) {
    return pcx::selftest_abort_once(users, aborters, iters, 0);
}
int pcx_selftest_abort_slow_holder(int users, int aborters) {
    return pcx::selftest_abort_once(users, aborters, 1, 1);
}
int pcx_selftest_group_abort(int world, int steps, int fail_rank, int fail_step) {
    return pcx::selftest_group_abort(world, steps, fail_rank, fail_step);
}
int pcx_selftest_rounds_sched(int workers, int64_t rounds, int enomem_worker, int64_t fail_round) {
    return pcx::selftest_rounds_sched(workers, rounds, enomem_worker, fail_round);
}
int pcx_selftest_chunked_copy(int64_t bytes, int64_t chunk, int slots, int threads, int64_t fail_chunk) {
    return pcx::selftest_chunked_copy(bytes, chunk, slots, threads, fail_chunk);
}
int pcx_test_inject_enomem(pcx_ctx* ctx, int worker) {
    if (!ctx) return fail(PCX_EINVAL, "pcx_test_inject_enomem: null context");
    ctx->test_enomem_worker = worker;
    return PCX_OK;
}

}  // extern "C"
