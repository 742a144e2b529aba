// pcx_internal.h -- declarations shared by the libpcx translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <string>
#include <vector>

#include "../../include/pcx.h"

// Kernel-side view of one single-matrix consensus on one rank: problem, scratch and
// outputs as device pointers (built by pcx_runner.cpp, passed by value to every
// kernel of pcx_matrix.hip).  Internal: the public boundary is pcx_problem /
// pcx_result (include/pcx.h).
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
    int32_t sel_first;            /* the selection's first histogram pass: over the column's whole key
                                     range (known from M_COLSTATS / the fill), also collecting the
                                     totals, weight extremes and fill-row sums (no separate init pass) */
    int32_t col_blocks;           /* row chunks of the column passes (G)          */
    int32_t cov_tiles, cov_kslices;
    int32_t no_fill;              /* reports are already filled (stage entries): no NA fill */
    int32_t rank_rule;            /* sign choice by nonconformity_rank (:487-500), else nonconformity */
    int32_t scores_given;         /* scores come from aux_scores (nonconformity entries, cokurtosis) */
    int32_t ob_order;             /* one rank and N*E < 9216 (OpenBLAS dgemv single-threaded): the np.dot
                                     vectors (:489-492, :510) and np.sum totals (:144, :244-249, :461) in
                                     the reference's own operation order */
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
    int64_t*  info;               /* [16] host-visible status (branch, iterations, counts) */
    /* weighted-median selection: per scaled event (reduced over ranks by SUM / MIN / MAX) */
    uint64_t* sel_state;          /* [n_scaled][SELS] range, sums, mode, result    */
    uint64_t* sel_isum;           /* [n_scaled][4] total weight limbs, count       (SUM) */
    /* a pass over n_active events reduces over ranks in two collectives: one SUM of hist_w | hist_n
       and one MAX of hist_min | hist_max (| sel_imin | sel_imax after the first pass) -- hist_n
       starts right after hist_w's n_active rows, hist_max after hist_min's (the runner moves the
       two pointers per pass), and every minimum is stored complemented (~min) so that MAX reduces it */
    uint64_t* sel_imin;           /* [n_scaled][2] ~(min key, min weight bits)     (MAX) */
    uint64_t* sel_imax;           /* [n_scaled][2] max key, max weight bits        (MAX) */
    uint64_t* hist_w;             /* [n_active][256][3] bucket weight limbs (SUM; weight-mode events) */
    uint64_t* hist_n;             /* [n_active][256] bucket element count          (SUM) */
    uint64_t* hist_min;           /* [n_active][256] ~(bucket min key)             (MAX) */
    uint64_t* hist_max;           /* [n_active][256] bucket max key                (MAX) */
    uint64_t* sel_arg;            /* [2][n_scaled] first dominant row (MIN), its value key (MAX) */
    int32_t*  sel_act;            /* [n_scaled] active scaled events, compacted in event order */
    int32_t*  hard;               /* [E] 0 / hard-replay mode per event (binary fill mean, median) */
    int32_t *hard_cols, *hard_modes; /* [E] the marked events in event order (k_sel_compact / k_hard_list) */
    uint64_t* cbuf;               /* [n_scaled][ccap][2] compacted (key, weight bits) of the range (k_sel_hist) */
    int64_t*  ccount;             /* [n_scaled] compacted elements of this rank                    */
    int64_t   ccap;               /* compaction capacity per event (0: none)                       */
    uint64_t* vsave;              /* [n_scaled][256][3] this rank's first-pass bucket counts, min and max
                                     keys of phase 1, then [n_scaled][4] (lo, hi, shift, 1) of their
                                     range: phase 2's first pass over the same range takes them
                                     instead of recounting (zeroed per call; k_sel_hist) */
    /* outputs ([E] events, [n_rows] agents of this rank) */
    double *old_rep, *this_rep, *smooth_rep, *scores, *na_row, *participation_rows, *relative_part,
        *reporter_bonus;
    double *adj_first_loadings, *outcomes_raw, *outcomes_adjusted, *outcomes_final, *certainty,
        *consensus_reward, *nas_filled, *participation_columns, *author_bonus;
    double* scalars;              /* [4]: participation, avg_certainty            */
    double* original;             /* [n_rows][E] rescaled reports (M_MATRICES), optional */
    double* filled;               /* [n_rows][E] filled reports (M_MATRICES), optional   */
    double* weighted_mean;        /* [E] optional (wpca entry)                     */
    double* nc_out;               /* [n_rows] optional (nonconformity entry)       */
    /* covariance operands (M_COV): the centred, filled matrix materialised once */
    double* wcd;                  /* [wcd_rows][wcd_ld] wcd = F - mu (:322), zero padded          */
    double* tokp;                 /* [wcd_rows + 64] tokens, zero past n_rows                       */
    int64_t wcd_rows;             /* n_rows rounded up to the 16-row stage                          */
    int64_t wcd_ld;               /* E rounded up to the 128-column tile                            */
    uint32_t* rowpart;            /* [ceil(wcd_ld/512)][wcd_rows][2] per-column-block NaN / zero row counts */
    /* wcd column order (M_COV_PLAN): general events first, then the grid events (binary,
       every filled value in {1, 1.5, 2}), each group in event order; the pure-grid tiles
       of the covariance run on int8 MFMA over z = 2 (F - 1) */
    int32_t* cov_perm;            /* [wcd_ld] event at each wcd position, -1 past E                 */
    int32_t* cov_pos;             /* [E] wcd position of each event                                 */
    int8_t*  zA;                  /* [wcd_rows/16][zq][16] tok * z of the positions >= 128 cov_jb, then the token column */
    int8_t*  zB;                  /* [wcd_rows/16][zq][16] z (the token column: 1)                  */
    int64_t* zsum;                /* [E] sum over this rank's rows of tok * z (grid events, exact)   */
    int64_t  zq;                  /* int8 operand width: E - 128 cov_jb + 1 rounded up to 256, or 0  */
    int32_t  cov_jb;              /* first pure-grid 128-column tile (= wcd_ld / 128: none)          */
    int32_t  cov_fp_tiles;        /* fp64 tiles: the Jb x Jb triangle (mixed pairs on int8) or the trapezoid J < cov_jb */
    int32_t  cov_mixed;           /* general x grid pairs on int8 slices of w (M_COV_I8)             */
    double*  Fg;                  /* [wcd_rows][128 cov_jb] the filled F of the general positions (or NULL) */
    uint16_t* nam;                /* [wcd_rows/16][wcd_ld] missing-report bits of 16 rows per position */
    int32_t  compact;             /* M_GEMV2 / M_OUTCOMES read Fg, zB and nam, not the reports      */
    uint32_t* zbg;                /* [wcd_rows/16][128] 2-bit codes of the grid events in the general tiles */
    int8_t*  wdig;                /* row weights' base-256 digits, [wcd_rows/16][16][16] per vector (or NULL) */
    int32_t  orig_inplace;        /* result.original aliases the reports: rescale the scaled columns
                                     in place (k_wcd / k_matrices), nothing else written (Q2)       */
    int32_t  rescaled;            /* set once that ran: later readers take the scaled columns as
                                     already rescaled (col_param: identity)                          */
    /* mixed pairs: w of the general positions (< 128 cov_jb) in 8 balanced int8 digits of 7 bits,
       fixed point at 2^e with e from the column's |F - mu| bound (exact, M_COV_PLAN) */
    int8_t*  zD;                  /* [wcd_rows/16][zd_ld][16] digit s of position q at s * 128 cov_jb + q */
    int64_t* dtok;                /* [PCX_NDIG][128 cov_jb] sum of each digit over this rank's rows (k_digits) */
    double*  dscale;              /* [wcd_ld] 2^-e per general position                               */
    int32_t* Pgg;                 /* [ks_gg][zq][zq] int32 zA^T zB per k-slice (lower part)           */
    int32_t* Pmx;                 /* [ks_mx][zq][PCX_NDIG * 128 cov_jb] int32 zA^T zD per k-slice            */
    int32_t  ks_gg, ks_mx;        /* k-slices of the two int8 products (int32-exact row ranges)       */
    int32_t  fp_ks;               /* k-slices of the fp64 tiles (k_syrk)                              */
    int64_t  fp_ld;               /* row length of one fp64 slab: E, or 128 cov_jb when mixed          */
    /* general x general pairs on int8 as well (cov_gg8, k_gemm_i8x): the digits of tok w (zD) against
       PCX_NDIG digits of w (zE, at 2^f from the column's |F - mu| bound), the digit pairs i + j <=
       PCX_NDIG - 1; k_syrk then runs nothing */
    int32_t  cov_gg8;
    int32_t  ks_gx;               /* k-slices of that product (int32-exact: |d e| <= 127^2 per row)   */
    int8_t*  zE;                  /* [wcd_rows/16][zd_ld][16] digit s of w at s * 128 cov_jb + q (== zD
                                     when every token is 2^k: tok w 2^-e = w 2^-f, the same digits)    */
    double*  escale;              /* [wcd_ld] 2^-f per general position                               */
    int32_t* Pgx;                 /* gemm_i8x_slab(ks, i, j, lower tile) x [256][256] int32            */
    int32_t  gg_smax;             /* the digit pairs i + j <= gg_smax in Pgx (PCX_NDIG - 1; all of them,
                                     2 PCX_NDIG - 2, once the covariance guard asked for the rest)      */
    /* the int8 covariance's error bound against the entries (k_digits -> k_cov_guard): per general
       position, [G_NSTAT][128 cov_jb] int64 sums over this rank's rows and then sum tok^2 (gacc), then
       as doubles over all ranks (gsum, exchanged with the covariance) */
    int64_t* gacc;
    double*  gsum;
    /* algorithms other than PCA (enum pcx_algorithm) */
    int32_t max_components;       /* "big-five" component count                                     */
    int32_t components;           /* out ("fixed-variance"): components used, else -1               */
    double  variance_threshold;   /* "fixed-variance" stop                                          */
    const double* aux_scores;     /* [n_rows] cokurtosis scores / given scores                      */
} pcx_mat;

// int8 covariance GEMM (k_gemm_i8, pcx_gemm_i8.h: PCX_GEMM_KS 64-row MFMA k-steps per LDS ring
// stage); the workspace pads wcd_rows to whole stages (pcx_runner.cpp COV_STAGE)
#include "pcx_gemm_i8.h"
// mixed block (general x grid pairs): balanced base-254 int8 digits per general position.  6
// digits leave a residue <= 2^-48.9 of the column's largest |tok w|; pcx_matrix.hip k_digits
#ifndef PCX_NDIG
#define PCX_NDIG 6
#endif
#define PCX_DBASE 254.0
// positions per 16-row group of the digit operands zD / zE: PCX_NDIG * gb rounded up to the GEMM's
// 256-position tile plus one more tile, so every tile's loads stay inside the row group -- the
// mixed block's last p-tile (NDIG * 128 * odd general tiles need not be a multiple of 256) and
// the general x general tiles (i gb + 256 a .. + 255, a < ceil(gb / 256), reach past digit i into
// digit i + 1 when gb is an odd multiple of 128); the pad positions only feed discarded entries
__host__ __device__ inline int64_t zd_ld(int64_t gb) { return ((int64_t)PCX_NDIG * gb + 255) / 256 * 256 + 256; }


namespace pcx {

// Kernel arguments of the batched round kernel (by value).
struct BatchArgs {
    int64_t B;
    int N, E, ES;
    const double* reports;
    const double* reputation;
    const uint8_t* scaled;
    const double* lo;
    const double* hi;
    int bounds_shared;
    int int_dtype;
    int algorithm;
    int max_components;       // big-five
    double variance_threshold;  // fixed-variance
    const double* aux_scores;   // cokurtosis [B][N]
    double hierarchy_threshold;  // hierarchical
    double cluster_threshold;    // clusterfeck (<= 0: log10(E)/1.77 rule)
    int kmeans_k, kmeans_restarts;
    const int32_t* kmeans_init;  // k-means [B][restarts][k]
    double catch_tol;
    double alpha;
    double *old_rep, *this_rep, *smooth_rep, *scores, *na_row, *participation_rows, *relative_part,
        *reporter_bonus;
    double *adj_first_loadings, *outcomes_raw, *outcomes_adjusted, *outcomes_final, *certainty,
        *consensus_reward, *nas_filled, *participation_columns, *author_bonus;
    double *participation, *avg_certainty;
    int32_t *branch, *flags, *pi_iters, *components;
    double *original, *filled;
    long long* stamps;  // diagnostic phase clocks [B][16] (PCX_STAMPS), normally NULL
};

size_t batched_lds_bytes(int N, int E, int algorithm);
hipError_t launch_batched(const BatchArgs& a, hipStream_t stream);
// rounds above one wavefront (N <= 256, E <= 64; PCA / absolute / cokurtosis): one workgroup each
bool medium_fits(const BatchArgs& a);
int64_t medium_chunk(const BatchArgs& a, size_t scratch_bytes);
hipError_t launch_medium(const BatchArgs& a, int64_t b0, int64_t nb, double* Fscr, double* Cscr, hipStream_t st);

// ---------------------------------------------------------------- single-matrix stages
// Internal stage ids (pcx_stage_name); the runner (pcx_runner.cpp) sequences them.
enum mat_stage_id {
    M_REPUTATION = 1, M_COLSTATS, M_GUESS, M_MEAN, M_COV, M_COV_REDUCE, M_COV_FINISH, M_POWER, M_SCORES,
    M_NCSUMS, M_GEMV2, M_DECIDE, M_REPU, M_SMOOTH, M_OUTCOMES, M_EVENTS, M_SCALED_CERT, M_FINAL, M_ROWSUMS,
    M_AGENTS, M_MATRICES, M_WCD, M_EIG, M_ZERO_LOADING, M_NC_OUT, M_WMEAN_OUT,
    M_SEL_EXACT, M_SEL_INIT, M_SEL_START, M_SEL_ARGMAX, M_SEL_VALUE, M_SEL_VALUE_FINISH, M_SEL_COMPACT,
    M_SEL_HIST, M_SEL_STEP, M_SEL_FINISH, M_HARD_LIST, M_HARD_GATHER, M_HARD_PREP, M_HARD_SORT, M_HARD_WALK,
    M_EXCHANGE, M_H2D, M_D2H, M_COV_PLAN, M_COV_I8, M_CLUSTER, M_COV_GUARD, M_COV_REST, M_WCD_REBUILD, M_NSTAGE
};
static_assert(M_NSTAGE <= PCX_NSTAGES, "stage table");
const char* stage_name(int k);

constexpr int SEL_NB = 256;         // selection buckets per pass
constexpr int SEL_EXACT_MAX = 8192; // one-block exact replay of weightedstats (one rank)

// launch one stage (pcx_matrix.hip)
hipError_t mat_stage(pcx_mat& m, int stage, hipStream_t stream, std::string& err);

// hard replay of weightedstats / the interpolation mean in the reference's sequential float
// order, for events whose exact-arithmetic decision lies within rounding of a threshold
struct HardArgs {
    int32_t n_hard;          // events in this batch
    const int32_t* cols;     // [n_hard] event index
    const int32_t* modes;    // [n_hard] HARD_MEAN (binary fill) / HARD_MEDIAN
    int64_t cap;             // max elements of one event on one rank (= n_rows)
    double* send;            // [n_hard][cap][2] (x, w) of this rank, row order
    int64_t* send_cnt;       // [n_hard]
    double* recv;            // [world][n_hard][cap][2]
    int64_t* recv_cnt;       // [world][n_hard]
    int64_t P;               // sort segment length (power of two >= max total count)
    uint64_t* keys;          // [n_hard][P][2] sort keys (value key, weight key)
    double* W;               // [n_hard][N] weights in row order (scratch)
    double* X;               // [n_hard][N] values in row order (scratch)
    double* hs;              // [n_hard][4] per event: mid, count, status, result
};
enum hard_mode { HARD_NONE = 0, HARD_MEAN = 1, HARD_MEDIAN = 2 };
hipError_t hard_stage(pcx_mat& m, const HardArgs& h, int stage, hipStream_t st, std::string& err);

hipError_t hard_list(pcx_mat& m, int32_t* cols, int32_t* modes, hipStream_t st);

// clustering algorithms on the single-matrix path (one rank): scratch and state
struct ClusterArgs {
    int32_t alg;            // PCX_ALG_KMEANS / HIERARCHICAL / CLUSTERFECK
    double  thr;            // hierarchical distance cut / clusterfeck threshold (default rule applied)
    int32_t k;              // k-means code-book size
    int32_t restart;        // k-means: current restart (row of kinit)
    const double* weights;  // k_cl_mu weights: rep (wpca mean) or wtok (clusterfeck outcomes)
    double* mu;             // [E] np.ma.average of the filled columns
    double* sd;             // [E] whiten's column std
    double* outc;           // [E] clusterfeck outcomes
    double* X;              // [N][E] wcd (hierarchical), whitened wcd (k-means), filled reports (clusterfeck)
    double* S;              // [max(N, k)][E] cluster sums
    double* book;           // [k][E] k-means code book
    double* best;           // [k][E] best restart's code book
    double* cs;             // [k] |code|^2
    double* dist;           // [N] vq distortions / cluster distances
    double* dm;             // [N] clusterfeck row distances
    double* dm1;            // [N]
    double* crep;           // [N] clusterfeck cluster weight sums
    double* wtok;           // [N] reptokens with zeros -> 1e-5 (:202-204)
    double* kst;            // [8] k-means state: prev0, prev1, best_d, continue, ncodes, best_n, it
    int32_t* lab;           // [N] labels / cluster of each row
    int32_t* cnt;           // [N] members per root / code
    int32_t* par;           // [N] union-find parents / clusterfeck first member
    int32_t* kinit;         // [restarts][k] initial code-book rows
};
enum cluster_step { CL_WTOK = 0, CL_MU, CL_X_WCD, CL_X_F, CL_WHITEN, CL_HIER, CL_NC_ROOT, CL_NC_LAB, CL_FECK,
                    KM_INIT, KM_ITER, KM_KEEP, KM_FINAL };
hipError_t cluster_stage(pcx_mat& m, const ClusterArgs& a, int step, hipStream_t st, std::string& err);
hipError_t sel_hist(pcx_mat& m, int n_active, hipStream_t st);
hipError_t sel_step(pcx_mat& m, int n_active, hipStream_t st);
// info[] slots read by the runner
enum info_slot_pub { INFO_BRANCH = 0, INFO_PI_ITERS = 1, INFO_FLAGS = 2, INFO_SEL_ACTIVE = 3, INFO_SEL_ARGMAX = 4,
                     INFO_PICK1 = 5, INFO_HARD = 6, INFO_SEL_WACTIVE = 7, INFO_COV_GENERAL = 8,
                     INFO_COV_MIXED = 9, INFO_COV_TOK1 = 10, INFO_COV_GUARD = 12, INFO_COV_GUARD_COLS = 13,
                     INFO_COV_GUARD_BOUND = 14 };
// the covariance guard's sums per general position (pcx_mat.gacc / gsum rows)
enum cov_guard_stat { G_L1D = 0, G_L1E, G_SD, G_SD2, G_SE, G_SE2, G_NSTAT };
// the covariance guard's outcome (info[INFO_COV_GUARD], pcx_result.cov_guard)
enum cov_guard_mode { COV_GUARD_PASS = 0, COV_GUARD_PAIRS = 1, COV_GUARD_FP64 = 2 };
hipError_t tri_pack(const double* C, double* buf, int64_t E, int unpack, hipStream_t st);

// pack / unpack of strided dd slot ranges for the slot exchange (runner)
hipError_t copy2d(double* dst, int64_t dpitch, const double* src, int64_t spitch, int64_t width, int64_t rows,
                  hipStream_t st);

// ---------------------------------------------------------------- cross-rank exchange
struct Comm {
    int world = 1, rank = 0;
    virtual ~Comm() {}
    // in place over `count` elements on the device, stream-ordered; 0 = ok
    virtual int allreduce(void* buf, int64_t count, int dtype, int op, hipStream_t st, std::string& err) = 0;
    // recv[world][bytes] <- send of every rank; send may alias recv + rank*bytes
    virtual int allgather(const void* send, void* recv, int64_t bytes, hipStream_t st, std::string& err) = 0;
    virtual const char* kind() const = 0;
    // unblock every rank waiting in this communicator after another rank failed (RCCL:
    // ncclCommAbort, exactly once whatever the number of callers); the communicator is
    // unusable afterwards and every later exchange returns PCX_ECOMM
    virtual void abort() {}
    std::atomic<bool> aborted{false};
};
Comm* comm_rccl(int device, int world, int rank, const pcx_comm_id* id, std::string& err);
int comm_rccl_unique_id(pcx_comm_id* out, std::string& err);
int rccl_version(int* runtime, int* compiled);
Comm* comm_group(pcx_group* g, int rank, std::string& err);
Comm* comm_custom(int world, int rank, const pcx_comm_ops* ops, std::string& err);
// one communicator per listed device, all in this process (ncclCommInitAll); 0 = ok
int comm_rccl_all(int n, const int* devices, std::vector<Comm*>& out, std::string& err);
pcx_group* group_create(int world);
void group_destroy(pcx_group* g);
void group_abort(pcx_group* g);  // wake and fail every waiting / later exchange of g
void group_reset(pcx_group* g);  // clear an abort once no rank is inside an exchange

}  // namespace pcx

// the context (pcx_api.cpp / pcx_runner.cpp)
struct pcx_workspace;
struct pcx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    pcx::Comm* comm = nullptr;     // NULL = one rank
    pcx_workspace* ws = nullptr;   // single-matrix scratch, cached between calls
    int profile = 0;
    double stage_ms[PCX_NSTAGES] = {0};
    int scaled_floor = 0;          // allocate the workspace for at least this many scaled events
    void* mscr = nullptr;          // per-round scratch of the workgroup-per-round kernel (pcx_medium.hip)
    size_t mscr_bytes = 0;
    // batched rounds above the one-wave kernel's limits: worker contexts of the round scheduler
    std::vector<pcx_ctx*> pool;
    // pcx_create_devices: one rank context per device, driven by worker threads
    std::vector<pcx_ctx*> sub;
    pcx_group* group = nullptr;    // host exchange of `sub` when a device id repeats
    // progress of the running single-matrix call, readable from another thread
    // (pcx_ctx_progress: a watchdog names the stage a stuck call is in)
    std::atomic<int> progress_stage{-1};
    std::atomic<int> progress_wait{0};   // 1 while the host blocks on the stream
    // test hook (pcx_test_inject_enomem): the round scheduler's worker k reports PCX_ENOMEM for
    // its first round of the NEXT batched call, without running it; -1 = off; consumed by that call
    int test_enomem_worker = -1;
    // pinned staging slots of the host-memory path's large output copies (pcx_runner.cpp)
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
    // the selection passes' info words, read one pass late (pinned, two slots; pcx_runner.cpp select)
    int64_t* sel_pin = nullptr;
    hipEvent_t sel_ev[2] = {nullptr, nullptr};
    // the host-memory path's large device copies (the reports, the matrix outputs), kept between
    // calls (a hipMalloc / hipFree of 33 GB per call is not free); pcx_release_workspace frees them
    std::vector<std::pair<void*, size_t>> io_bufs;
    // pinned buffer of the host path's small outputs (one copy back per call)
    void* pin_small = nullptr;
    size_t pin_small_bytes = 0;
    // the host path's copy of `filled` back, run beside the device work that follows k_wcd
    hipStream_t side_stream = nullptr;
};

namespace pcx {
void workspace_free(pcx_ctx* c);
// entry: 0 consensus, 1 interpolate, 2 wpca, 3 lie_detector, 4 nonconformity
int run_matrix(pcx_ctx* c, const pcx_problem* p, pcx_result* r, int entry, const double* scores_in, int rank_rule,
               double* nc_out, std::string& err);
// the rank-independent argument checks of run_matrix (algorithm, clustering vs world,
// k-means draws, thresholds, aux scores, mem_kind); 0 = ok
int check_problem(const pcx_problem* p, int world, int entry, std::string& err);
// batched rounds of any N x E (pcx_rounds.cpp): each round one single-matrix consensus on a
// pool of worker contexts with their own streams; synchronous
int run_rounds(pcx_ctx* c, const pcx_batch* in, pcx_batch_result* out, std::string& err);
void rounds_free(pcx_ctx* c);
// a context's host-side resources (pinned staging slots, the selection's pinned info words and
// events, the workgroup-per-round scratch): pcx_destroy and rounds_free (the pool's worker contexts)
void ctx_host_free(pcx_ctx* c);
void io_bufs_free(pcx_ctx* c);  // the host path's cached device copies (pcx_ctx.io_bufs)
}  // namespace pcx
