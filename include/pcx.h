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

#define PCX_ABI_VERSION 4

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
/* Batched regime: B independent rounds of equal shape N x E, one round per    */
/* wavefront (Simulator.jl-style Monte Carlo, README.rst:52-56).  Each round is */
/* the complete Oracle(reports, event_bounds, reputation).consensus() of       */
/* __init__.py:102-611.                                                          */
/* Limits: 1 <= N <= 64, 1 <= E <= 32.                                          */
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
    PCX_ALG_KMEANS = 5,            /* cluster sizes of scipy kmeans on whitened wcd (:392-405); batched only */
    PCX_ALG_HIERARCHICAL = 6,      /* cluster sizes of single-linkage fclusterdata(wcd) (:407-419); batched only */
    PCX_ALG_CLUSTERFECK = 7,       /* leader clustering of the filled reports (:148-242, :421-424); batched only */
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
/* reporter rows over several GPUs (one process per GPU).  The consensus is a   */
/* fixed sequence of stages (pcx_mat_stage); between some stages the host       */
/* combines per-rank partial buffers across ranks (pyconsensus_amd/pipeline.py, */
/* torch.distributed over RCCL).  Every buffer is caller-allocated device memory */
/* sized as documented in pipeline.py (MatWorkspace).                           */
/* ------------------------------------------------------------------------ */
enum pcx_mat_stage_id {
    PCX_M_REPUTATION = 1,    /* rep, tokens (__init__.py:138-146)                    */
    PCX_M_COLSTATS = 2,      /* rescale + NA + present sums per event (:266-299)     */
    PCX_M_GUESS = 3,         /* binary fills (:304-309), median setup (:300-303)     */
    PCX_M_MEAN = 4,          /* weighted mean mu, old = rep . F (:317-319, 490)     */
    PCX_M_COV = 5,           /* token-weighted covariance partial tiles, fp64 MFMA (:326); needs PCX_M_WCD */
    PCX_M_COV_REDUCE = 6,    /* sum split-K slabs into this rank's partial C         */
    PCX_M_COV_FINISH = 7,    /* C = partial / (sum tokens - 1), symmetric            */
    PCX_M_POWER = 8,         /* leading eigenvector by power iteration (:330-336)    */
    PCX_M_SCORES = 9,        /* scores = wcd . loading (:337), row NA counts         */
    PCX_M_NCSUMS = 10,       /* sums of |set1|, |set2| (:488-489, normalize)         */
    PCX_M_GEMV2 = 11,        /* normalize(set1/2) . F (:492-493)                     */
    PCX_M_DECIDE = 12,       /* rank rule / continuous fallback (:491-498, 475-485)  */
    PCX_M_REPU = 13,         /* nc * rep / mean(rep) and its sum (:460-462)          */
    PCX_M_SMOOTH = 14,       /* this_rep, smooth_rep (:460-472)                      */
    PCX_M_OUTCOMES = 15,     /* smooth . F, participation, certainty bins (:510, 559, 542) */
    PCX_M_EVENTS = 16,       /* catch/unscale binary events (:526-538)               */
    PCX_M_SCALED_CERT = 17,  /* certainty of scaled events (:540-546)                */
    PCX_M_FINAL = 18,        /* reward, author bonus, participation (:545-581)      */
    PCX_M_ROWSUMS = 19,      /* participation_rows normalisation sums (:567-576)     */
    PCX_M_AGENTS = 20,       /* per-reporter outputs (:576-577, 586-595)             */
    PCX_M_MATRICES = 21,     /* result["original"] / result["filled"] (:584-585)     */
    PCX_M_SEL_INIT = 30,     /* weighted median (:303, :520): totals, key range, max weight */
    PCX_M_SEL_START = 31,    /*   dominance test, first histogram range              */
    PCX_M_SEL_ARGMAX = 32,   /*   first row with the dominant weight                 */
    PCX_M_SEL_VALUE = 33,    /*   value at that row                                  */
    PCX_M_SEL_HIST = 34,     /*   exact weight histogram over the current key range  */
    PCX_M_SEL_STEP = 35,     /*   narrow the range; converged columns get their result */
    PCX_M_SEL_FINISH = 36,   /*   results into guess (phase 1) / outcomes_raw (phase 2) */
    PCX_M_SEL_EXACT = 37,    /* weighted median replayed with the reference's float order (n <= 8192, 1 rank) */
    PCX_M_WCD = 39,          /* wcd = F - mu materialised once (:317-322), row NaN/zero counts */
    PCX_M_EIG = 38,          /* big-five / fixed-variance: eigenpairs of C (svd, :375, :431), the
                                eigenvalue-weighted component sum (:377-382, :435-449) -> score vector */
    PCX_M_ZERO_LOADING = 99, /* no wpca ("absolute", "cokurtosis"): first_loading = 0 (:359)          */
};

typedef struct {
    /* shape and parameters */
    int64_t n_rows;               /* rows held by this rank                       */
    int64_t n_events;             /* E                                            */
    int64_t n_total;              /* N over all ranks                             */
    int64_t row_offset;           /* global index of this rank's first row        */
    int32_t world, rank;
    int32_t int_dtype, algorithm;
    double  catch_tolerance, alpha;
    int32_t n_scaled;             /* number of scaled events                      */
    int32_t sel_phase;            /* 1: interpolation medians, 2: outcome medians */
    int32_t col_blocks;           /* row chunks of the column passes (G)          */
    int32_t cov_tiles, cov_kslices;
    /* inputs */
    const double*  reports;       /* [n_rows][E]                                  */
    const uint8_t* scaled;        /* [E] or NULL (event_bounds None)              */
    const double*  lo;            /* [E]                                          */
    const double*  hi;            /* [E]                                          */
    const double*  rep_raw;       /* [n_total] raw reputation, or NULL = uniform   */
    const int32_t* scaled_cols;   /* [n_scaled] event index of each scaled event   */
    const int32_t* scaled_index;  /* [E] position of event j among scaled events, -1 if binary */
    /* workspace */
    double*   rep;                /* [n_rows]                                     */
    double*   tok;                /* [n_rows]                                     */
    double*   T;                  /* [n_scaled][n_rows] rescaled scaled events, NaN = missing */
    double*   part;               /* [col_blocks][E][8][2] column-pass block partials */
    double*   mpart;              /* [col_blocks][E][4] block max/min partials     */
    double*   cstat;              /* [world][E][16][2] per-rank column sums (dd)   */
    double*   cmax;               /* [world][E][4] per-rank max rep / argmax / min / max */
    double*   scal;               /* [world][16][2] per-rank scalar sums (dd)      */
    double*   spart;              /* [4096][4][2] row-pass block partials          */
    double*   ev;                 /* [16][E] event vectors (guess, mu, old, ...)   */
    double*   cslab;              /* [cov_kslices][E][E] covariance partial tiles  */
    double*   C;                  /* [E][E] covariance                             */
    double*   Mw;                 /* [2][E][E] power-iteration working matrices    */
    double*   pvec;               /* [4][E + 64] power-iteration scratch           */
    double*   rowv;               /* [6][n_rows] scores, this, smooth, u, ...       */
    uint32_t* rowstat;            /* [n_rows][2] NaN / zero counts per row         */
    uint64_t* skey;               /* [world][4] score min/max keys, flags          */
    int64_t*  info;               /* [16] host-visible status (branch, iterations, active columns) */
    /* weighted-median selection state (per scaled event) */
    uint64_t* sel_sum;            /* [world][n_scaled][256][4] limb sums + counts  */
    uint64_t* sel_min;            /* [world][n_scaled][256][2] min key, min weight bits */
    uint64_t* sel_max;            /* [world][n_scaled][256] max key                */
    uint64_t* sel_state;          /* [n_scaled][16] range, sums, flags             */
    double*   sel_val;            /* [world][n_scaled][4] max weight, value, result */
    /* outputs ([E] events, [n_rows] agents of this rank) */
    double *old_rep, *this_rep, *smooth_rep, *scores, *na_row, *participation_rows, *relative_part,
        *reporter_bonus;
    double *adj_first_loadings, *outcomes_raw, *outcomes_adjusted, *outcomes_final, *certainty,
        *consensus_reward, *nas_filled, *participation_columns, *author_bonus;
    double* scalars;              /* [4]: participation, avg_certainty, branch, flags */
    double* original;             /* [n_rows][E] rescaled reports (PCX_M_MATRICES), optional */
    double* filled;               /* [n_rows][E] filled reports (PCX_M_MATRICES), optional   */
    /* covariance operands (PCX_M_COV): the centred, filled matrix materialised once */
    double* wcd;                  /* [wcd_rows][wcd_ld] wcd = F - mu (:322), zero padded          */
    double* tokp;                 /* [wcd_rows + 64] tokens, zero past n_rows                       */
    int64_t wcd_rows;             /* n_rows rounded up to the 16-row stage                          */
    int64_t wcd_ld;               /* E rounded up to the 128-column tile                            */
    uint32_t* rowpart;            /* [ceil(wcd_ld/512)][wcd_rows][2] per-column-block NaN / zero row counts */
    /* algorithms other than PCA (enum pcx_algorithm) */
    int32_t max_components;       /* "big-five" component count                                     */
    int32_t components;           /* out ("fixed-variance"): components used, else -1               */
    double  variance_threshold;   /* "fixed-variance" stop                                          */
    const double* aux_scores;     /* "cokurtosis": [n_rows] scores of this rank's rows              */
} pcx_mat;

/* Run one stage on the context's stream (PCX_M_POWER and the selection steps may
 * synchronise the stream to read convergence state). */
int pcx_mat_stage(pcx_ctx* ctx, pcx_mat* m, int stage);

#ifdef __cplusplus
}
#endif
#endif /* PCX_H */
