"""ctypes mirror of include/pcx.h (structs and constants).  Keep in sync with the header."""
import ctypes as C

ABI_VERSION = 8

OK, EINVAL, EHIP, ENOMEM, ECOMM = 0, -1, -2, -3, -4
BRANCH_SET1, BRANCH_SET2, BRANCH_TIE_SET1, BRANCH_TIE_SET2, BRANCH_NONE = 1, 2, 3, 4, 5
FLAG_ZERO_COV, FLAG_SVD_FAIL, FLAG_PI_MAXIT = 1, 2, 4
# enum pcx_algorithm (include/pcx.h); the clustering algorithms run in the batched regime only
ALG_PCA, ALG_ABSOLUTE, ALG_BIG_FIVE, ALG_FIXED_VARIANCE, ALG_COKURTOSIS = 0, 1, 2, 3, 4
ALG_KMEANS, ALG_HIERARCHICAL, ALG_CLUSTERFECK = 5, 6, 7
ALGORITHMS = {"PCA": ALG_PCA, "absolute": ALG_ABSOLUTE, "big-five": ALG_BIG_FIVE,
              "fixed-variance": ALG_FIXED_VARIANCE, "cokurtosis": ALG_COKURTOSIS,
              "k-means": ALG_KMEANS, "hierarchical": ALG_HIERARCHICAL, "clusterfeck": ALG_CLUSTERFECK}
CLUSTER_ALGORITHMS = ("k-means", "hierarchical", "clusterfeck")
KMEANS_RESTARTS = 20  # scipy.cluster.vq.kmeans(iter=20)

P_D = C.POINTER(C.c_double)


class Batch(C.Structure):
    _fields_ = [
        ("n_rounds", C.c_int64),
        ("n_reporters", C.c_int64),
        ("n_events", C.c_int64),
        ("reports", C.c_void_p),
        ("reputation", C.c_void_p),
        ("scaled", C.c_void_p),
        ("lo", C.c_void_p),
        ("hi", C.c_void_p),
        ("bounds_shared", C.c_int32),
        ("int_dtype", C.c_int32),
        ("catch_tolerance", C.c_double),
        ("alpha", C.c_double),
        ("algorithm", C.c_int32),
        ("max_components", C.c_int32),
        ("variance_threshold", C.c_double),
        ("aux_scores", C.c_void_p),
        ("hierarchy_threshold", C.c_double),
        ("cluster_threshold", C.c_double),
        ("kmeans_k", C.c_int32),
        ("kmeans_restarts", C.c_int32),
        ("kmeans_init", C.c_void_p),
    ]


# name, per-round shape kind ('N', 'E', '1', 'NE'), dtype
BATCH_OUTPUTS = [
    ("old_rep", "N", "f8"), ("this_rep", "N", "f8"), ("smooth_rep", "N", "f8"),
    ("scores", "N", "f8"), ("na_row", "N", "f8"), ("participation_rows", "N", "f8"),
    ("relative_part", "N", "f8"), ("reporter_bonus", "N", "f8"),
    ("adj_first_loadings", "E", "f8"), ("outcomes_raw", "E", "f8"),
    ("outcomes_adjusted", "E", "f8"), ("outcomes_final", "E", "f8"),
    ("certainty", "E", "f8"), ("consensus_reward", "E", "f8"), ("nas_filled", "E", "f8"),
    ("participation_columns", "E", "f8"), ("author_bonus", "E", "f8"),
    ("participation", "1", "f8"), ("avg_certainty", "1", "f8"),
    ("branch", "1", "i4"), ("flags", "1", "i4"), ("pi_iters", "1", "i4"),
    ("original", "NE", "f8"), ("filled", "NE", "f8"),
    ("components", "1", "i4"),
]


class BatchResult(C.Structure):
    _fields_ = [(name, C.c_void_p) for name, _, _ in BATCH_OUTPUTS]


def out_shape(kind, B, N, E):
    return {"N": (B, N), "E": (B, E), "1": (B,), "NE": (B, N, E)}[kind]


# ---------------------------------------------------------------- single-matrix regime
MEM_DEVICE, MEM_HOST = 0, 1
F64, U64 = 0, 1                  # enum pcx_dtype
RED_SUM, RED_MIN, RED_MAX = 0, 1, 2  # enum pcx_redop
NSTAGES = 56                     # PCX_NSTAGES

MAT_OUTPUT_AGENTS = ["old_rep", "this_rep", "smooth_rep", "scores", "na_row", "participation_rows",
                     "relative_part", "reporter_bonus"]
MAT_OUTPUT_EVENTS = ["adj_first_loadings", "outcomes_raw", "outcomes_adjusted", "outcomes_final",
                     "certainty", "consensus_reward", "nas_filled", "participation_columns", "author_bonus"]

_vp = C.c_void_p


class CommId(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


ALLREDUCE_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32)
ALLGATHER_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)


class CommOps(C.Structure):
    _fields_ = [("user", _vp), ("allreduce", ALLREDUCE_CB), ("allgather", ALLGATHER_CB)]


class Problem(C.Structure):
    _fields_ = [
        ("n_rows", C.c_int64), ("n_events", C.c_int64), ("n_total", C.c_int64), ("row_offset", C.c_int64),
        ("reports", _vp), ("reputation", _vp), ("scaled", _vp), ("lo", _vp), ("hi", _vp),
        ("catch_tolerance", C.c_double), ("alpha", C.c_double),
        ("int_dtype", C.c_int32), ("algorithm", C.c_int32), ("max_components", C.c_int32), ("mem_kind", C.c_int32),
        ("variance_threshold", C.c_double), ("aux_scores", _vp),
        ("hierarchy_threshold", C.c_double), ("cluster_threshold", C.c_double),
        ("kmeans_k", C.c_int32), ("kmeans_restarts", C.c_int32), ("kmeans_init", _vp)]


RESULT_VECTORS = MAT_OUTPUT_AGENTS + MAT_OUTPUT_EVENTS + ["original", "filled", "weighted_mean", "covariance"]


class Result(C.Structure):
    _fields_ = [(n, _vp) for n in RESULT_VECTORS] + [
        ("participation", C.c_double), ("avg_certainty", C.c_double),
        ("branch", C.c_int32), ("flags", C.c_int32), ("pi_iters", C.c_int32), ("components", C.c_int32),
        ("n_hard", C.c_int32), ("sel_passes", C.c_int32), ("comm_bytes", C.c_double),
        ("grid_events", C.c_int32), ("mixed_int8", C.c_int32),
        ("cov_guard", C.c_int32), ("cov_guard_cols", C.c_int32), ("cov_err_bound", C.c_double)]
