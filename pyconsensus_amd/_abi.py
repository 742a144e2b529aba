"""ctypes mirror of include/pcx.h (structs and constants).  Keep in sync with the header."""
import ctypes as C

ABI_VERSION = 1

OK, EINVAL, EHIP, ENOMEM, ECOMM = 0, -1, -2, -3, -4
BRANCH_SET1, BRANCH_SET2, BRANCH_TIE_SET1, BRANCH_TIE_SET2, BRANCH_NONE = 1, 2, 3, 4, 5
FLAG_ZERO_COV, FLAG_SVD_FAIL, FLAG_PI_MAXIT = 1, 2, 4
ALGORITHMS = {"PCA": 0, "absolute": 1}

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
]


class BatchResult(C.Structure):
    _fields_ = [(name, C.c_void_p) for name, _, _ in BATCH_OUTPUTS]


def out_shape(kind, B, N, E):
    return {"N": (B, N), "E": (B, E), "1": (B,), "NE": (B, N, E)}[kind]
