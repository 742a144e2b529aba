/*
 * pcx.h -- C ABI of libpcx, the MI355X (gfx950) implementation of
 * pyconsensus's Oracle.consensus() hot path (algorithm="PCA").
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

#define PCX_ABI_VERSION 1

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
    int32_t algorithm;            /* 0 = "PCA", 1 = "absolute" (nc = 0, Q13)     */
} pcx_batch;

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
} pcx_batch_result;

int pcx_consensus_batched_f64(pcx_ctx* ctx, const pcx_batch* in, pcx_batch_result* out);

#ifdef __cplusplus
}
#endif
#endif /* PCX_H */
