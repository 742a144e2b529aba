/*
 * pcx.h -- C ABI of libpcx, the MI355X (gfx950) implementation of
 * pyconsensus's Oracle.consensus() hot path (algorithm "PCA", plus "absolute",
 * "big-five", "fixed-variance" and "cokurtosis" on the same kernels, and the
 * clustering algorithms "k-means", "hierarchical" and "clusterfeck" in the
 * batched regime).
 *
 * The reference (IanMadlenya/pyconsensus) is pure Python with no FFI: its whole
 * public surface is `Oracle(reports, event_bounds, reputation, ...).consensus()`
 * (pyconsensus/__init__.py:102-146, 502-611).  The entry points below are what a
 * binding of that path needs; each cites the reference code it replaces.  The
 * Python host layer (pyconsensus_amd/oracle.py) keeps the reference's class, its
 * constructor arguments and its result dict, and calls this ABI through ctypes.
 *
 * Conventions
 *   - Every pointer in a problem/result struct is DEVICE memory (hipMalloc or a
 *     torch tensor's data_ptr()) on the device the context was created for.
 *   - Matrices are row-major: reports[i*E + j] = reporter i, event j.
 *     NaN marks a missing report; 0.0 is ALSO missing (reference NA = 0.0,
 *     __init__.py:68, 278).
 *   - Any output pointer may be NULL: that output is not written.
 *   - Return value 0 = success, negative = error; pcx_last_error() describes the
 *     last error of the calling thread.  No C++ exception crosses the ABI.
 *   - Calls are asynchronous on the context's stream (pcx_set_stream) unless
 *     stated otherwise; a pcx_ctx is not thread-safe (one per thread).
 */
#ifndef PCX_H
#define PCX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCX_ABI_VERSION 8

enum pcx_status {
    PCX_OK = 0,
    PCX_EINVAL = -1,       /* bad argument / unsupported shape            */
    PCX_EHIP = -2,         /* HIP runtime error                           */
    PCX_ENOMEM = -3,       /* scratch allocation failed                   */
    PCX_ECOMM = -4,        /* RCCL error                                  */
};

/* Branch taken by the sign-choice rule (__init__.py:494-498, 482-484). */
enum pcx_branch {
    PCX_BRANCH_SET1 = 1,           /* rank rule ref_ind < 0                   */
    PCX_BRANCH_SET2 = 2,           /* rank rule ref_ind > 0                   */
    PCX_BRANCH_TIE_SET1 = 3,       /* ref_ind == 0 -> nonconformity, ref <= 0 */
    PCX_BRANCH_TIE_SET2 = 4,       /* ref_ind == 0 -> nonconformity, ref > 0  */
    PCX_BRANCH_NONE = 5,           /* algorithm without a branch ("absolute") */
};

/* Flags reported per round (bit set). */
enum pcx_flag {
    PCX_FLAG_ZERO_COV = 1,         /* covariance == 0: loading = e_0 (svd(0) = I, __init__.py:330) */
    PCX_FLAG_SVD_FAIL = 2,         /* non-finite covariance: loading = ones/sqrt(E) (:331-333)       */
    PCX_FLAG_PI_MAXIT = 4,         /* power iteration hit its iteration cap                         */
};

typedef struct pcx_ctx pcx_ctx;

int         pcx_abi_version(void);
const char* pcx_last_error(void);

/* One context per device and host thread.  Replaces nothing in the reference
 * (it has no device state); owns scratch buffers and the stream. */
pcx_ctx* pcx_create(int device_id);
void     pcx_destroy(pcx_ctx* ctx);
int      pcx_set_stream(pcx_ctx* ctx, void* hip_stream);  /* NULL = default stream */
int      pcx_synchronize(pcx_ctx* ctx);

/* ------------------------------------------------------------------------ */
/* Batched regime: B independent rounds of equal shape N x E (Simulator.jl-    */
/* style Monte Carlo, README.rst:52-56).  Each round is the complete            */
/* Oracle(reports, event_bounds, reputation).consensus() of __init__.py:102-611. */
/* N <= 64, E <= 32: one round per wavefront, asynchronous on the stream.      */
/* N <= 256, E <= 64 (all but the clusterings): one 256-thread workgroup per    */
/* round (the same SPEC order), asynchronous.  Any other shape or algorithm     */
/* (E <= 65536): each round is one single-matrix consensus, a pool of worker    */
/* streams keeps many in flight (PCX_ROUND_WORKERS, default 16); synchronous.   */
/* ------------------------------------------------------------------------ */
typedef struct {
    int64_t n_rounds;             /* B                                           */
    int64_t n_reporters;          /* N                                           */
    int64_t n_events;             /* E                                           */
    const double*  reports;       /* [B][N][E]                                   */
    const double*  reputation;    /* [B][N] raw weights, or NULL (= None: 1/N)   */
    const uint8_t* scaled;        /* [B][E] (or [E] if bounds_shared), NULL = event_bounds None */
    const double*  lo;            /* event_bounds[j]["min"], same layout as scaled */
    const double*  hi;            /* event_bounds[j]["max"]                      */
    int32_t bounds_shared;        /* 1: scaled/lo/hi are one [E] row for all rounds */
    int32_t int_dtype;            /* 1: reports had an integer dtype (truncation, Q3) */
    double  catch_tolerance;      /* Oracle(catch_tolerance=0.1)                 */
    double  alpha;                /* Oracle(alpha=0.1)                           */
    int32_t algorithm;            /* enum pcx_algorithm                          */
    int32_t max_components;       /* "big-five": components summed (Oracle caps it at E, :134-137) */
    double  variance_threshold;   /* "fixed-variance": cumulative explained-variance stop (:448) */
    const double* aux_scores;     /* "cokurtosis": [B][N] caller scores, aux["cokurt"] (:455-457) */
    /* clustering algorithms (ABI >= 4; __init__.py:392-428) */
    double  hierarchy_threshold;  /* "hierarchical": fcluster distance cut, Oracle(hierarchy_threshold=0.5) (:406) */
    double  cluster_threshold;    /* "clusterfeck": leader-clustering cut after the reference's default rule
                                     log10(E)/1.77 (0.3 when that is 0) (:210-213); <= 0: computed on the device */
    int32_t kmeans_k;             /* "k-means": code-book size, int(ceil(sqrt(N))) in the reference (:396)     */
    int32_t kmeans_restarts;      /* "k-means": scipy.cluster.vq.kmeans iter= (20)                              */
    const int32_t* kmeans_init;   /* "k-means": [B][restarts][k] rows of the initial code books -- the draws of
                                     scipy's _kpoints, rng.choice(N, k, replace=False) on numpy's global
                                     RandomState, made by the host so the device replays the same restarts */
} pcx_batch;

/* Oracle(algorithm=...) values on the GPU path (__init__.py:368-457). */
enum pcx_algorithm {
    PCX_ALG_PCA = 0,               /* first principal component + rank rule (:368-371)         */
    PCX_ALG_ABSOLUTE = 1,          /* unimplemented branch: nc = 0 (:359-362, Q13)             */
    PCX_ALG_BIG_FIVE = 2,          /* eigenvalue-weighted top max_components scores (:373-390) */
    PCX_ALG_FIXED_VARIANCE = 3,    /* components up to variance_threshold (:429-451)           */
    PCX_ALG_COKURTOSIS = 4,        /* caller-supplied scores aux["cokurt"] (:455-457)          */
    PCX_ALG_KMEANS = 5,            /* cluster sizes of scipy kmeans on whitened wcd (:392-405)          */
    PCX_ALG_HIERARCHICAL = 6,      /* cluster sizes of single-linkage fclusterdata(wcd) (:407-419)     */
    PCX_ALG_CLUSTERFECK = 7,       /* leader clustering of the filled reports (:148-242, :421-424)     */
};

typedef struct {
    /* [B][N] -- result["agents"] */
    double* old_rep;
    double* this_rep;
    double* smooth_rep;
    double* scores;
    double* na_row;
    double* participation_rows;
    double* relative_part;
    double* reporter_bonus;
    /* [B][E] -- result["events"] */
    double* adj_first_loadings;
    double* outcomes_raw;
    double* outcomes_adjusted;
    double* outcomes_final;
    double* certainty;
    double* consensus_reward;
    double* nas_filled;
    double* participation_columns;
    double* author_bonus;
    /* [B] */
    double*  participation;
    double*  avg_certainty;
    int32_t* branch;              /* enum pcx_branch                             */
    int32_t* flags;               /* enum pcx_flag bits                          */
    int32_t* pi_iters;            /* power-iteration steps (incl. squarings)     */
    /* [B][N][E], optional */
    double* original;             /* result["original"]: rescaled reports        */
    double* filled;               /* result["filled"]                            */
    /* [B] */
    int32_t* components;          /* result["components"]: fixed-variance count, else -1 (:449, :610) */
} pcx_batch_result;

int pcx_consensus_batched_f64(pcx_ctx* ctx, const pcx_batch* in, pcx_batch_result* out);

/* ------------------------------------------------------------------------ */
/* Single-matrix regime: one N x E report matrix, optionally sharded by        */
/* contiguous reporter rows over several GPUs (one process -- or one thread --  */
/* per rank).  One call runs the whole Oracle(...).consensus() of              */
/* __init__.py:502-611; stage sequencing, scratch memory and the cross-rank    */
/* exchange (RCCL over xGMI, or the backends below) are owned by the library.   */
/* ------------------------------------------------------------------------ */

/* Multi-rank contexts.  pcx_create() above is a one-rank context.  For RCCL,
 * rank 0 calls pcx_comm_unique_id(), the caller broadcasts the 128 bytes over any
 * channel (e.g. torch.distributed), and every rank calls pcx_create_rank()
 * (ncclCommInitRank, collective over the ranks).  Replaces nothing in the
 * reference (it has no distribution). */
typedef struct { char internal[128]; } pcx_comm_id;
int      pcx_comm_unique_id(pcx_comm_id* out);
pcx_ctx* pcx_create_rank(int device_id, int world, int rank, const pcx_comm_id* id);

/* In-process virtual ranks: `world` threads, each with its own context on any
 * device, exchanging through host memory.  Used to rehearse the sharded path on
 * one GPU (tests, 1-GPU boxes).  The group must outlive its contexts. */
typedef struct pcx_group pcx_group;
pcx_group* pcx_group_create(int world);
void       pcx_group_destroy(pcx_group* g);
pcx_ctx*   pcx_create_grouped(int device_id, pcx_group* g, int rank);

/* Caller-supplied exchange (MPI, gloo, ...).  The library passes HOST buffers
 * (it stages device data through pinned memory); return 0 on success.
 *   allreduce: in place, `count` elements of enum pcx_dtype, enum pcx_redop.
 *   allgather: recv[world][bytes] <- every rank's `bytes` of send, rank order. */
enum pcx_dtype { PCX_F64 = 0, PCX_U64 = 1 };
enum pcx_redop { PCX_SUM = 0, PCX_MIN = 1, PCX_MAX = 2 };
typedef struct {
    void* user;
    int (*allreduce)(void* user, void* buf, int64_t count, int32_t dtype, int32_t op);
    int (*allgather)(void* user, const void* send, void* recv, int64_t bytes);
} pcx_comm_ops;
pcx_ctx* pcx_create_custom(int device_id, int world, int rank, const pcx_comm_ops* ops);

/* One process driving several GPUs (pcx_create(n_devices,
 * device_ids); replaces the reference's single-process Oracle(...).consensus(),
 * __init__.py:502-611, at sizes one GPU cannot hold).  A single-matrix call on this
 * context takes the WHOLE matrix in host memory (PCX_MEM_HOST, n_total == n_rows,
 * row_offset 0) and shards its rows over the devices in contiguous blocks (the
 * first N % n_devices blocks one row longer), one worker thread per device.  The
 * devices exchange through RCCL (ncclCommInitAll, xGMI) when the ids are distinct,
 * through host memory when an id repeats (rehearsal on fewer GPUs).  Results are
 * the one-device call's, bit for bit; the scalars of pcx_result are device 0's
 * (comm_bytes: summed over the devices).  pcx_consensus_batched_f64 on this
 * context runs on device_ids[0]. */
pcx_ctx* pcx_create_devices(int n_devices, const int* device_ids);

int pcx_ctx_world(const pcx_ctx* ctx);
int pcx_ctx_rank(const pcx_ctx* ctx);
/* 1 if the context's communicators can still exchange, 0 once a failed call aborted them (RCCL:
 * ncclCommAbort after a rank of a multi-device call failed mid-exchange): destroy and recreate
 * it then.  An argument error raised before any exchange (PCX_EINVAL from the rank-independent
 * checks) leaves the context usable. */
int pcx_ctx_usable(const pcx_ctx* ctx);
/* Drop the cached scratch of the single-matrix path (it is kept between calls of
 * the same shape: a C5 consensus needs ~50 GB of it). */
int pcx_release_workspace(pcx_ctx* ctx);

enum pcx_mem_kind {
    PCX_MEM_DEVICE = 0,  /* every pointer of pcx_problem / pcx_result is device memory of ctx's device */
    PCX_MEM_HOST = 1,    /* every pointer is host memory; the library copies in and out (timed apart) */
};

typedef struct {
    int64_t n_rows;               /* reporters held by this rank                         */
    int64_t n_events;             /* E                                                   */
    int64_t n_total;              /* N over all ranks (== n_rows on one rank)            */
    int64_t row_offset;           /* global index of this rank's first reporter          */
    const double*  reports;       /* [n_rows][E] row-major, NaN = missing (0.0 too, :278) */
    const double*  reputation;    /* [n_total] raw weights (every rank passes all N), or NULL = None (:138-141) */
    const uint8_t* scaled;        /* [E] event_bounds[j]["scaled"], or NULL = event_bounds None (Q12) */
    const double*  lo;            /* [E] event_bounds[j]["min"]                          */
    const double*  hi;            /* [E] event_bounds[j]["max"]                          */
    double  catch_tolerance;      /* Oracle(catch_tolerance=0.1)                         */
    double  alpha;                /* Oracle(alpha=0.1)                                   */
    int32_t int_dtype;            /* 1: reports had an integer dtype (truncation, Q3)    */
    int32_t algorithm;            /* enum pcx_algorithm (every value; the clustering ones on one rank) */
    int32_t max_components;       /* big-five (Oracle caps it at E, :134-137)            */
    int32_t mem_kind;             /* enum pcx_mem_kind                                   */
    double  variance_threshold;   /* fixed-variance (:448)                               */
    const double* aux_scores;     /* cokurtosis: [n_rows] this rank's aux["cokurt"] (:455-457) */
    /* clustering algorithms (one rank; ABI >= 7; __init__.py:148-242, 392-424) */
    double  hierarchy_threshold;  /* "hierarchical": fcluster distance cut, Oracle(hierarchy_threshold=0.5) */
    double  cluster_threshold;    /* "clusterfeck": leader cut; <= 0: the reference's log10(E)/1.77 rule */
    int32_t kmeans_k;             /* "k-means": code-book size int(ceil(sqrt(N))) (:396)          */
    int32_t kmeans_restarts;      /* "k-means": scipy kmeans iter= (20)                           */
    const int32_t* kmeans_init;   /* "k-means": [restarts][k] HOST rows of the initial code books (the
                                     reference's rng.choice draws, pyconsensus_amd.batched.kmeans_draws) */
} pcx_problem;

typedef struct {
    /* [n_rows] -- result["agents"], this rank's reporters; NULL = not written */
    double *old_rep, *this_rep, *smooth_rep, *scores, *na_row, *participation_rows, *relative_part,
        *reporter_bonus;
    /* [E] -- result["events"] (identical on every rank) */
    double *adj_first_loadings, *outcomes_raw, *outcomes_adjusted, *outcomes_final, *certainty,
        *consensus_reward, *nas_filled, *participation_columns, *author_bonus;
    /* [n_rows][E], optional: result["original"] (rescaled reports), result["filled"].
     * original == (double*)problem.reports (the same pointer) is the reference's own aliasing
     * (__init__.py:121, 266-269, 584: `original` IS the caller's array, rescaled in place): the
     * scaled columns of the reports are then rescaled in place and the other columns are left as
     * they are, which saves writing a copy of the whole matrix (pcx_consensus_f64 and
     * pcx_interpolate_f64; the reports buffer must then be writable).  After a failed call the
     * buffer's scaled columns are unspecified: with several ranks (pcx_create_devices) each rank
     * writes its rescaled rows back as it finishes, so a failure elsewhere can leave some rows
     * rescaled and others not; the reference leaves them rescaled. */
    double *original, *filled;
    /* wpca intermediates (:317-326), optional: [E] weighted_mean, [E][E] covariance_matrix */
    double *weighted_mean, *covariance;
    /* scalars, always written (host memory inside this struct) */
    double  participation;        /* result["participation"]                             */
    double  avg_certainty;        /* result["avg_certainty"]                             */
    int32_t branch;               /* enum pcx_branch                                     */
    int32_t flags;                /* enum pcx_flag bits                                  */
    int32_t pi_iters;             /* power-iteration steps (incl. Gram squarings)        */
    int32_t components;           /* result["components"]: fixed-variance count, else -1 (:449, :610) */
    int32_t n_hard;               /* weighted medians / binary fills replayed in sequential float order */
    int32_t sel_passes;           /* weighted-selection histogram passes                 */
    double  comm_bytes;           /* bytes this rank passed to collectives (all-reduce buffers + all-gather sends) */
    int32_t grid_events;          /* grid events (binary, filled values on {1, 1.5, 2}) past the general 128-event tiles:
                                     their covariance block ran on int8 MFMA */
    int32_t mixed_int8;           /* bit 0: general x grid pairs ran on int8 digit slices too (else fp64 MFMA);
                                     bit 1: and the general x general pairs (digits of tok w x digits of w) */
    /* the int8 covariance's guard (mixed_int8 != 0): an upper bound, rigorous in exact arithmetic, on
     * |C_pq - C~_pq| / sqrt(C_pp C_qq) over the entries with a general position, where C~ is the
     * covariance of the fp64 centred matrix wcd (:322-326) and C the emulation's result.  Above
     * 2^-40 the covariance is recomputed: cov_guard 1 = the remaining digit pairs (i + j >= NDIG, every
     * digit product exact), 2 = the general pairs on fp64 MFMA (k_syrk, as without int8).  0 = passed. */
    int32_t cov_guard;
    int32_t cov_guard_cols;       /* general events whose own bound (the pair (p, p)) exceeded 2^-40   */
    double  cov_err_bound;        /* the bound of the emulation that ran first (before any recompute)  */
} pcx_result;

/* The whole consensus (__init__.py:502-611) on this rank's rows; collective over
 * the context's ranks.  Synchronous: returns after every output is written. */
int pcx_consensus_f64(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r);

/* The reference's stage methods on the same kernels (Oracle.interpolate / wpca /
 * lie_detector / nonconformity(_rank), __init__.py:260-500).
 *   pcx_interpolate_f64: p->reports raw; writes original / filled (:260-313).
 *   pcx_wpca_f64:        p->reports is a FILLED matrix (no NA handling); writes
 *                        weighted_mean, covariance, adj_first_loadings (first
 *                        loading) and scores (first score) (:315-339).
 *   pcx_lie_detector_f64: p->reports FILLED; wpca + nonconformity_rank (PCA) or
 *                        the algorithm's branch, then this_rep / smooth_rep
 *                        (:341-473); writes scores, adj_first_loadings, old_rep,
 *                        this_rep, smooth_rep, branch.
 *   pcx_nonconformity_f64: p->reports FILLED, scores [n_rows] given; rank_rule 1 =
 *                        nonconformity_rank (:487-500), 0 = nonconformity (:475-485);
 *                        writes nc [n_rows] and r->branch. */
int pcx_interpolate_f64(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r);
int pcx_wpca_f64(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r);
int pcx_lie_detector_f64(pcx_ctx* ctx, const pcx_problem* p, pcx_result* r);
int pcx_nonconformity_f64(pcx_ctx* ctx, const pcx_problem* p, const double* scores, int rank_rule, double* nc,
                          pcx_result* r);

/* Per-stage device time of the last single-matrix call (HIP events on the
 * context's stream) when enabled; names by pcx_stage_name(k), k < PCX_NSTAGES. */
#define PCX_NSTAGES 56
int         pcx_profile_enable(pcx_ctx* ctx, int on);
int         pcx_profile_read(pcx_ctx* ctx, double* ms /* [PCX_NSTAGES] */);
const char* pcx_stage_name(int k);
/* Progress of the single-matrix call running on `ctx` (safe to call from another
 * thread while it runs): *stage = the last stage enqueued (pcx_stage_name; -1 before
 * the first), *host_waiting = 1 while the host blocks on the context's stream (a
 * collective waiting for a peer shows as a wait after M_EXCHANGE or a later stage).
 * A multi-device context reports device 0's worker. */
int pcx_ctx_progress(const pcx_ctx* ctx, int* stage, int* host_waiting);

/* Sequential float sums of a constant (weightedstats' builtin-sum walk over equal
 * weights, __init__.py:287-303, :519-523): S(k) = 0 + c + c + ... (k terms, each
 * addition rounded to nearest-even), in O(log k) by binade stepping; and the least
 * k >= 1 with S(k) > t (kmax + 1 if none up to kmax).  Exported for the CPU tests. */
double  pcx_seqsum_const(double c, int64_t k);
int64_t pcx_seqsum_first_above(double c, double t, int64_t kmax);

/* Build parameter: balanced base-254 int8 digits per general event in the covariance's mixed block
 * (pcx_result.mixed_int8 bit 0; the int8 work per row is then grid pairs + digits x general x grid,
 * plus digits (digits + 1) / 2 x the general pairs with bit 1).  For roofline accounting. */
int pcx_mixed_digits(void);

/* The RCCL that serves libpcx's collectives: *runtime = ncclGetVersion() of the librccl the
 * process resolved (with torch loaded first: torch's bundled copy), *compiled = the
 * NCCL_VERSION_CODE of the headers libpcx was built against.  Returns *runtime.  RCCL
 * contexts are refused (PCX_ECOMM, both versions named) unless the major versions agree and
 * the runtime is >= 2.18 (version code 21800). */
int pcx_rccl_version(int* runtime, int* compiled);

/* CPU self-test of the communicator abort path (no RCCL, no GPU): `users` threads run
 * exchanges on a fake handle while `aborters` threads abort it.  Returns the number of
 * violations (the handle freed other than exactly once, used after it was freed, or used
 * successfully after an abort returned); 0 = pass, -1 = bad arguments.  For the tests. */
int pcx_selftest_abort_once(int users, int aborters, int iters);
/* The same abort path when one user is blocked inside its exchange for twice the abort's wait
 * (an RCCL enqueue stuck on a failed peer): every abort must return after the bounded wait, free
 * the handle exactly once (overlapping the blocked use: the documented window, counted once) and
 * fail every later use.  Returns the number of violations; 0 = pass, -1 = bad arguments. */
int pcx_selftest_abort_slow_holder(int users, int aborters);
/* CPU self-test of the virtual-rank exchange (pcx_group, as pcx_create_grouped /
 * pcx_create_devices use it): `world` threads run `steps` slot exchanges; rank `fail_rank`
 * fails at step `fail_step` (-1: none), the first failure aborts the group and must release
 * every waiting rank; after a reset a clean run must pass.  Returns the number of violations. */
int pcx_selftest_group_abort(int world, int steps, int fail_rank, int fail_step);
/* CPU self-test of the round scheduler's hand-out (pcx_consensus_batched_f64 above 256 x 64):
 * `workers` threads take `rounds` fake rounds; worker `enomem_worker` reports PCX_ENOMEM on its
 * first round (-1: none) and must hand it back; round `fail_round` fails (-1: none) and must stop
 * the batch.  Every round must run exactly once.  Returns the number of violations. */
int pcx_selftest_rounds_sched(int workers, int64_t rounds, int enomem_worker, int64_t fail_round);
/* CPU self-test of the host-memory path's staged large copies (pinned slots, host threads):
 * `bytes` through `slots` slots of `chunk` bytes by `threads` threads, memcpy standing in for the
 * DMA; chunk `fail_chunk`'s transfer fails (-1: none) and must stop the copy.  Returns the number
 * of violations (data, a chunk moved twice or after the failure); 0 = pass, -1 = bad arguments. */
int pcx_selftest_chunked_copy(int64_t bytes, int64_t chunk, int slots, int threads, int64_t fail_chunk);
/* Test hook: the NEXT pcx_consensus_batched_f64 call on `ctx` that takes the round scheduler
 * makes its worker `worker` report PCX_ENOMEM for its first round without running it (the
 * hand-back path); -1 clears it.  Consumed by that call.  For the tests only. */
int pcx_test_inject_enomem(pcx_ctx* ctx, int worker);

#ifdef __cplusplus
}
#endif
#endif /* PCX_H */
