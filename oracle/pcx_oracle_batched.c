/*
 * pcx_oracle_batched.c -- CPU restatement of the batched consensus round.
 *
 * TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.  Built into
 * oracle/lib/libpcx_oracle.so and loaded (ctypes) only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  libpcx never links it.
 *
 * It restates, one round at a time, pyconsensus Oracle(...).consensus() with the
 * default algorithm="PCA" (pyconsensus/__init__.py:102-611), with the arithmetic
 * order written down explicitly (SPEC comments) so that the GPU batched kernel
 * (pyconsensus_amd/csrc/pcx_batched.hip) can be checked against it bit for bit:
 *
 *   - where the reference's order is defined by Python/numpy (sequential Python
 *     loops, builtin sum, numpy pairwise add.reduce, elementwise ops) this file
 *     replays that exact order, so those steps agree bit-for-bit with the
 *     reference too;
 *   - where the reference calls BLAS (np.dot, dgemm) or LAPACK (svd) the order is
 *     OpenBLAS/LAPACK-internal; here it is a fixed sequential-FMA order and the
 *     leading eigenvector comes from power iteration.  Those steps agree with the
 *     reference to rounding (checked against tests/golden/ with tolerances, and
 *     near-tie rounds reported separately).
 *
 * Compiled with -ffp-contract=off: every fma() below is deliberate.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

#include "../include/pcx.h"

#ifndef NMAX
#define NMAX 64 /* reporters per round; libpcx_oracle256.so: 256 (the workgroup-per-round kernel's rounds) */
#endif
#define EMAX 64
#define ES (EMAX + 1)

/* power iteration constants -- must equal pcx_batched.hip */
#define PI_TOL 1e-14
#define PI_MAXIT 256
#define PI_PRESQUARE 3
#define PI_SQUARE_EVERY 32
#define PI_MAX_SQUARINGS 8
#define PI_POLISH 2

/* numpy pairwise summation (umath loops_utils pairwise_sum, PW_BLOCKSIZE 128),
 * as np.add.reduce uses it for a contiguous 1-D array of <= 8192 elements. */
static double pw_sum(const double* a, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; i++) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; k++) r[k] = a[k];
        int i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; k++) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pw_sum(a, n2) + pw_sum(a + n2, n - n2);
}

/* SPEC tree64: over 64 slots (zero padded), a butterfly inside each row of 16 (xor
 * distance 1, 2, 4, 8), then (R0 + R1) + (R2 + R3) of the four row sums. */
static double tree64(const double* a, int n) {
    double t[64], u[64];
    for (int i = 0; i < 64; i++) t[i] = i < n ? a[i] : 0.0;
    for (int s = 1; s <= 8; s <<= 1) {
        for (int i = 0; i < 64; i++) u[i] = t[i] + t[i ^ s];
        memcpy(t, u, sizeof t);
    }
    return (t[0] + t[16]) + (t[32] + t[48]);
}

/* SPEC dot2: compensated dot product (Ogita-Rump-Oishi Dot2: TwoProduct by fma,
 * TwoSum), summed in index order.  Used for the GEMVs whose results feed the
 * discontinuous decisions (ranks, catch): the reference's np.dot is OpenBLAS
 * dgemv, whose summation order is BLAS-internal; a nearly correctly rounded dot
 * reproduces every decision that does not hinge on BLAS rounding. */
static double dot2(const double* a, int sa, const double* b, int sb, int n) {
    double s = 0.0, c = 0.0;
    for (int i = 0; i < n; i++) {
        double x = a[(int64_t)i * sa], y = b[(int64_t)i * sb];
        double p = x * y;
        double pe = fma(x, y, -p);
        double t = s + p;
        double z = t - s;
        double se = (s - (t - z)) + (p - z);
        s = t;
        c = c + (pe + se);
    }
    return s + c;
}

/* np.dot(v, F) for v (N,), F (N, E) row-major with row stride ES, column j, in the exact
 * operation order numpy 2.2 / OpenBLAS 0.3.29 use in the build container (DYNAMIC_ARCH,
 * SkylakeX kernels), the machine the golden vectors come from.  Measured, not documented:
 * tests/golden/probe_openblas_order.py fits this model bit for bit on random inputs with a
 * wide exponent range (every N <= 139, E <= 32).  numpy calls cblas_dgemv(RowMajor, Trans),
 * i.e. column-major dgemv_n on the E x N matrix (single-threaded at these sizes):
 *   - events j < E & ~3 (the 4-row vector kernel): reporters in blocks of 4, each block
 *     t = v1*F1 rounded, then fma with reporters 0, 2, 3; y = y + t; a tail of 2 the same
 *     with reporters (1, 0); a tail of 1: y = y + v*F;
 *   - the last E % 4 events (scalar code): y = fma(F_i, v_i, y) over i, except lda == 2 or 3
 *     (E == 2, 3), unrolled by 4 as y = y + fma(F_i, v_i, F_i+1 v_i+1) per pair;
 *   - E == 1: numpy's ddot (4 x 8-lane fma accumulators per 32, folded to 4 x 4 lanes, 16 per
 *     step, lanes summed (0+2)+(1+3), then a sequential fma tail). */
static double ob_ddot(const double* a, const double* x, int sx, int n) {
    double acc8[4][8] = {{0}}, acc4[4][4];
    const int n32 = n & -32, n16 = n & -16;
    for (int i = 0; i < n32; i += 32)
        for (int k = 0; k < 32; k++) acc8[k / 8][k % 8] = fma(a[i + k], x[(int64_t)(i + k) * sx], acc8[k / 8][k % 8]);
    for (int r = 0; r < 4; r++)
        for (int l = 0; l < 4; l++) acc4[r][l] = acc8[r][l] + acc8[r][l + 4];
    for (int i = n32; i < n16; i += 16)
        for (int k = 0; k < 16; k++) acc4[k / 4][k % 4] = fma(a[i + k], x[(int64_t)(i + k) * sx], acc4[k / 4][k % 4]);
    double A[4];
    for (int l = 0; l < 4; l++) A[l] = ((acc4[0][l] + acc4[1][l]) + acc4[2][l]) + acc4[3][l];
    double d = (A[0] + A[2]) + (A[1] + A[3]);
    for (int i = n16; i < n; i++) d = fma(a[i], x[(int64_t)i * sx], d);
    return d;
}

static double ob_vecmat(const double* v, const double* Fj, int ld, int N, int E, int j) {
    if (E == 1) return ob_ddot(v, Fj, ld, N);
#define FJ(i) Fj[(int64_t)(i) * ld]
    if (j < (E & ~3)) {
        double y = 0.0;
        int n = 0;
        for (; n + 4 <= N; n += 4) {
            double t = FJ(n + 1) * v[n + 1];
            t = fma(FJ(n), v[n], t);
            t = fma(FJ(n + 2), v[n + 2], t);
            t = fma(FJ(n + 3), v[n + 3], t);
            y = y + t;
        }
        if (n + 2 <= N) {
            double t = FJ(n + 1) * v[n + 1];
            t = fma(FJ(n), v[n], t);
            y = y + t;
            n += 2;
        }
        if (n < N) y = y + FJ(n) * v[n];
        return y;
    }
    double t = 0.0;
    int i = 0;
    if (E == 2 || E == 3)
        for (; i + 4 <= N; i += 4) {
            t = t + fma(FJ(i), v[i], FJ(i + 1) * v[i + 1]);
            t = t + fma(FJ(i + 2), v[i + 2], FJ(i + 3) * v[i + 3]);
        }
    for (; i < N; i++) t = fma(FJ(i), v[i], t);
    return t;
#undef FJ
}

static double catch_(double x, double tol) {  /* __init__.py:251-258 */
    if (x < 1.5 - tol) return 1.0;
    if (x > 1.5 + tol) return 2.0;
    return 1.5;
}

static void normalize_(const double* v, int n, double* out) {  /* __init__.py:244-249 */
    double a[NMAX > EMAX ? NMAX : EMAX];
    for (int i = 0; i < n; i++) a[i] = fabs(v[i]);
    double s = pw_sum(a, n);
    if (s == 0) {
        for (int i = 0; i < n; i++) a[i] += 1.0;
        s = pw_sum(a, n);
    }
    for (int i = 0; i < n; i++) out[i] = a[i] / s;
}

/* weightedstats.weighted_median restated (see oracle/pcx_oracle.py). */
static double wmedian(const double* x, const double* w, int n) {
    double W = 0.0;
    for (int i = 0; i < n; i++) W += w[i];
    double mid = 0.5 * W;
    int dom = 0;
    for (int i = 0; i < n; i++) dom |= w[i] > mid;
    if (dom) {
        double m = w[0];
        for (int i = 1; i < n; i++) if (w[i] > m) m = w[i];
        for (int i = 0; i < n; i++) if (w[i] == m) return x[i];
        return NAN;
    }
    int pos = 0;
    for (int i = 0; i < n; i++) pos |= w[i] > 0;
    if (!pos) return NAN;
    double xs[NMAX], ws[NMAX];
    for (int i = 0; i < n; i++) {  /* stable rank by (x, w) */
        int r = 0;
        for (int m = 0; m < n; m++) {
            int lt = (x[m] < x[i]) || (x[m] == x[i] && w[m] < w[i]);
            int eq = (x[m] == x[i]) && (w[m] == w[i]);
            r += lt || (eq && m < i);
        }
        xs[r] = x[i];
        ws[r] = w[i];
    }
    double cum = 0.0;
    int k = 0;
    while (cum <= mid) {
        if (k == n) return NAN; /* the reference raises IndexError here */
        cum += ws[k];
        k++;
    }
    double before = cum - ws[k - 1];
    if (fabs(before - mid) < DBL_EPSILON) {
        if (k >= 2) return (xs[k - 2] + xs[k - 1]) / 2.0;
        if (n == 1) return xs[0] / 1.0;
        return NAN; /* empty slice: ZeroDivisionError in the reference */
    }
    return xs[k - 1];
}

/* scipy.stats.rankdata 'average'; a NaN ranks NaN, so the rule's sums are NaN when any value
 * is (rankdata's nan_policy='propagate' makes every rank NaN: the same sums) */
static void rank_avg(const double* v, int n, double* r) {
    for (int j = 0; j < n; j++) {
        if (isnan(v[j])) {
            r[j] = NAN;
            continue;
        }
        int lt = 0, eq = 0;
        for (int k = 0; k < n; k++) {
            lt += v[k] < v[j];
            eq += v[k] == v[j];
        }
        r[j] = (double)lt + (double)(eq + 1) * 0.5;
    }
}

/* SPEC: M <- (M*M) / max|M*M|, products as sequential fma over the inner index */
static void square_scaled(double (*M)[ES], int E) {
    static __thread double T[EMAX][ES];
    double mx = 0.0;
    for (int j = 0; j < E; j++)
        for (int k = 0; k < E; k++) {
            double acc = 0.0;
            for (int l = 0; l < E; l++) acc = fma(M[j][l], M[l][k], acc);
            T[j][k] = acc;
            double a = fabs(acc);
            if (a > mx) mx = a;
        }
    /* scale by the power of two that brings max|MM| into [1, 2): exact, so only the
     * products round (a zero / subnormal / non-finite maximum divides as before) */
    const int pow2 = mx >= DBL_MIN && isfinite(mx);
    const double sc = pow2 ? ldexp(1.0, -ilogb(mx)) : 1.0;
    for (int j = 0; j < E; j++)
        for (int k = 0; k < E; k++) M[j][k] = pow2 ? T[j][k] * sc : (mx > 0.0 ? T[j][k] / mx : T[j][k]);
}

static void matvec_unit(const double (*M)[ES], int E, const double* x, double* y) {
    double sq[EMAX];
    for (int j = 0; j < E; j++) {
        double acc = 0.0;
        for (int k = 0; k < E; k++) acc = fma(M[j][k], x[k], acc);
        y[j] = acc;
        sq[j] = acc * acc;
    }
    double nrm = sqrt(tree64(sq, E));
    for (int j = 0; j < E; j++) y[j] = y[j] / nrm;
}

/* SPEC power iteration -> unit leading eigenvector of C (replaces svd(C)[0][:,0],
 * __init__.py:330).  Returns steps taken; sets flags. */
static int power_iter(const double (*C)[ES], int E, double* v, int* flags) {
    int finite = 1, nonzero = 0;
    for (int j = 0; j < E; j++)
        for (int k = 0; k < E; k++) {
            finite &= isfinite(C[j][k]) != 0;
            nonzero |= C[j][k] != 0.0;
        }
    if (!finite) {  /* LAPACK raises -> H = ones (:331-333) */
        for (int j = 0; j < E; j++) v[j] = 1.0;
        *flags |= PCX_FLAG_SVD_FAIL;
        return 0;
    }
    if (!nonzero) {  /* svd(0) returns U = I: first column e_0 */
        for (int j = 0; j < E; j++) v[j] = j == 0 ? 1.0 : 0.0;
        *flags |= PCX_FLAG_ZERO_COV;
        return 0;
    }
    static __thread double M[EMAX][ES];
    int kd = 0;
    for (int j = 1; j < E; j++) if (C[j][j] > C[kd][kd]) kd = j;
    double x[EMAX], y[EMAX], sq[EMAX];
    for (int j = 0; j < E; j++) {
        x[j] = C[j][kd];
        sq[j] = x[j] * x[j];
    }
    double nrm = sqrt(tree64(sq, E));
    for (int j = 0; j < E; j++) x[j] = x[j] / nrm;
    for (int j = 0; j < E; j++) memcpy(M[j], C[j], sizeof(double) * E);
    int sqn = 0;
    for (; sqn < PI_PRESQUARE; sqn++) square_scaled(M, E);
    int it = 0, since = 0;
    for (;;) {
        matvec_unit((const double (*)[ES])M, E, x, y);
        double d = 0.0;
        for (int j = 0; j < E; j++) {
            double a = fabs(y[j] - x[j]);
            if (a > d) d = a;
            x[j] = y[j];
        }
        it++;
        since++;
        if (d <= PI_TOL) break;
        if (it >= PI_MAXIT) {
            *flags |= PCX_FLAG_PI_MAXIT;
            break;
        }
        if (since >= PI_SQUARE_EVERY && sqn < PI_MAX_SQUARINGS) {
            square_scaled(M, E);
            sqn++;
            since = 0;
        }
    }
    for (int p = 0; p < PI_POLISH; p++) {
        matvec_unit(C, E, x, y);
        memcpy(x, y, sizeof(double) * E);
    }
    /* SPEC sign (the reference's is whatever LAPACK gesdd returns): measured on
     * the golden set, U[:,0] has its first nonzero component negative, except
     * when it is a unit vector e_k, which LAPACK returns as +e_k. */
    {
        int f = -1, nnz = 0;
        for (int j = 0; j < E; j++)
            if (x[j] != 0.0) {
                nnz++;
                if (f < 0) f = j;
            }
        int neg = nnz == 1 ? x[f] < 0.0 : x[f] > 0.0;
        if (neg)
            for (int j = 0; j < E; j++) x[j] = -x[j];
    }
    memcpy(v, x, sizeof(double) * E);
    return it + PI_POLISH + sqn;
}

/* ------------------------------------------------------------------------
 * "big-five" / "fixed-variance" (__init__.py:373-390, 429-451): the reference
 * takes U, Sigma = svd(C) (LAPACK gesdd).  SPEC: C is symmetric PSD, so the
 * singular pairs are the eigenpairs: Sigma = |lambda| in descending order, U's
 * columns the eigenvectors (each loading is sign-normalised by the reference
 * itself, loading[0] >= 0).  The eigenpairs come from cyclic two-sided Jacobi
 * with the round-robin (circle) pair schedule: every step's pairs are disjoint;
 * all its rotation angles are taken from the matrix at the start of the step,
 * then the rotations are applied rows first, then columns (and V's columns).
 * The GPU kernel applies the same steps lane-parallel in the same two phases.
 * ------------------------------------------------------------------------ */
#define JAC_MAXSWEEP 30
#define JAC_TOL 1e-15

static void jac_pair(int i, int r, int n, int* p, int* q) {
    const int a = i == 0 ? 0 : 1 + (i - 1 + r) % (n - 1);
    const int b = 1 + (n - 2 - i + r) % (n - 1);
    *p = a < b ? a : b;
    *q = a < b ? b : a;
}

/* one rotation's (c, s) from A[p][p], A[q][q], A[p][q]; s == 0 means "skip" */
static void jac_angle(double app, double aqq, double apq, double* c, double* s) {
    *c = 1.0;
    *s = 0.0;
    if (apq == 0.0) return;
    const double tau = (aqq - app) / (2.0 * apq);
    const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
    *c = 1.0 / sqrt(1.0 + t * t);
    *s = t * *c;
}

static void jacobi_eig(double (*A)[ES], double (*V)[ES], int E) {
    for (int j = 0; j < E; j++)
        for (int k = 0; k < E; k++) V[j][k] = j == k ? 1.0 : 0.0;
    if (E < 2) return;
    const int n = E + (E & 1), npair = n / 2;
    for (int sweep = 0; sweep < JAC_MAXSWEEP; sweep++) {
        double off = 0.0, dg = 0.0;  /* max-norms: exact in any order */
        for (int j = 0; j < E; j++)
            for (int k = 0; k < E; k++) {
                const double v = fabs(A[j][k]);
                if (j == k)
                    dg = fmax(dg, v);
                else
                    off = fmax(off, v);
            }
        if (!(off > JAC_TOL * dg)) break;
        for (int r = 0; r < n - 1; r++) {
            int pp[EMAX / 2 + 1], qq[EMAX / 2 + 1];
            double cc[EMAX / 2 + 1], ss[EMAX / 2 + 1];
            for (int i = 0; i < npair; i++) {
                jac_pair(i, r, n, &pp[i], &qq[i]);
                if (qq[i] >= E) {  /* the dummy player of an odd E */
                    cc[i] = 1.0;
                    ss[i] = 0.0;
                } else {
                    jac_angle(A[pp[i]][pp[i]], A[qq[i]][qq[i]], A[pp[i]][qq[i]], &cc[i], &ss[i]);
                }
            }
            for (int i = 0; i < npair; i++) {  /* rows */
                if (ss[i] == 0.0) continue;
                const int p = pp[i], q = qq[i];
                const double c = cc[i], s = ss[i];
                for (int k = 0; k < E; k++) {
                    const double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
            }
            for (int i = 0; i < npair; i++) {  /* columns of A and V */
                if (ss[i] == 0.0) continue;
                const int p = pp[i], q = qq[i];
                const double c = cc[i], s = ss[i];
                for (int j = 0; j < E; j++) {
                    const double ajp = A[j][p], ajq = A[j][q];
                    A[j][p] = c * ajp - s * ajq;
                    A[j][q] = s * ajp + c * ajq;
                    const double vjp = V[j][p], vjq = V[j][q];
                    V[j][p] = c * vjp - s * vjq;
                    V[j][q] = s * vjp + c * vjq;
                }
            }
        }
    }
}

/* net_score = sum_c Sigma_c * (wcd . loading_c) over the selected components, the
 * component loop of :377-382 / :435-448 (score = Sigma * wcd.dot(loading), net +=).
 * Returns the number of components used (fixed-variance) or -1 (big-five). */
static int component_scores(int alg, const double (*C)[ES], int E, int N, const double (*F)[ES], const double* mu,
                            int max_components, double threshold, double* net) {
    static __thread double A[EMAX][ES], V[EMAX][ES];
    double diag[EMAX], sig[EMAX];
    int order[EMAX];
    for (int j = 0; j < E; j++) {
        memcpy(A[j], C[j], sizeof(double) * E);
        diag[j] = C[j][j];
    }
    const double trace = pw_sum(diag, E); /* np.trace: add.reduce of the diagonal */
    jacobi_eig(A, V, E);
    for (int j = 0; j < E; j++) sig[j] = fabs(A[j][j]);
    for (int j = 0; j < E; j++) {  /* descending Sigma, ties by index */
        int rk = 0;
        for (int k = 0; k < E; k++) rk += (sig[k] > sig[j]) || (sig[k] == sig[j] && k < j);
        order[rk] = j;
    }
    const int kmax = alg == PCX_ALG_BIG_FIVE ? max_components : E;
    for (int i = 0; i < N; i++) net[i] = 0.0;
    double ve = 0.0;
    int used = kmax;
    for (int c = 0; c < kmax; c++) {
        const int idx = order[c];
        const double sg = sig[idx];
        const double fl = V[0][idx] < 0.0 ? -1.0 : 1.0; /* loading *= -1 if loading[0] < 0 */
        for (int i = 0; i < N; i++) {
            double d = 0.0;
            for (int j = 0; j < E; j++) d = fma(F[i][j] - mu[j], fl * V[j][idx], d);
            net[i] = net[i] + sg * d;
        }
        if (alg == PCX_ALG_FIXED_VARIANCE) { /* cumsum(Sigma / trace) >= threshold -> stop */
            ve = ve + sg / trace;
            if (ve >= threshold) {
                used = c + 1;
                break;
            }
        }
    }
    return alg == PCX_ALG_FIXED_VARIANCE ? used : -1;
}

/* ------------------------------------------------------------------------
 * Clustering algorithms: k-means (:392-405), hierarchical
 * (:407-419), clusterfeck (:148-242, :421-424).  Each turns the filled reports into
 * a nonconformity vector nc; the rest of the round is the common tail.
 * ------------------------------------------------------------------------ */

/* nc from cluster sizes (:398-405, :412-419): (size - min size) / sum, the sum of
 * integers exact; every cluster the same size gives 0/0 = NaN, as numpy does. */
static void nc_from_sizes(const int* size, int N, double* nc) {
    int mn = size[0];
    for (int i = 1; i < N; i++) mn = size[i] < mn ? size[i] : mn;
    long long tot = 0;
    for (int i = 0; i < N; i++) tot += size[i] - mn;
    for (int i = 0; i < N; i++) nc[i] = (double)(size[i] - mn) / (double)tot;
}

/* hierarchical: scipy fclusterdata(wcd, t, criterion='distance'), single linkage on
 * euclidean pdist.  SPEC: d_ij = sqrt(sum_k (wcd_ik - wcd_jk)^2), sequential, no fma
 * (scipy's pdist order, checked bit for bit); flat clusters = connected components of
 * {d_ij <= t} (single-linkage cophenetic distance <= t). */
static void hier_nc(const double (*F)[ES], const double* mu, int N, int E, double t, double* nc) {
    int parent[NMAX], size[NMAX];
    for (int i = 0; i < N; i++) parent[i] = i;
    for (int i = 0; i < N; i++)
        for (int j = i + 1; j < N; j++) {
            double d2 = 0.0;
            for (int k = 0; k < E; k++) {
                const double df = (F[i][k] - mu[k]) - (F[j][k] - mu[k]);
                d2 = d2 + df * df;
            }
            if (sqrt(d2) <= t) {
                int a = i, b = j;
                while (parent[a] != a) a = parent[a];
                while (parent[b] != b) b = parent[b];
                if (a != b) parent[a > b ? a : b] = a < b ? a : b;
            }
        }
    int root[NMAX], cnt[NMAX] = {0};
    for (int i = 0; i < N; i++) {
        int a = i;
        while (parent[a] != a) a = parent[a];
        root[i] = a;
        cnt[a]++;
    }
    for (int i = 0; i < N; i++) size[i] = cnt[root[i]];
    nc_from_sizes(size, N, nc);
}

/* k-means distance^2 of scipy's _vq.vq as built here: E < 5 the naive loop
 * sum (x-c)^2; otherwise -2 x.c (OpenBLAS dgemm: one fma chain per entry for
 * K < 32, eight interleaved chains summed as a tree for K = 32) + |x|^2 + |c|^2,
 * the squares sequential.  Measured against scipy 1.15 / scipy-openblas in the
 * build container (the goldens' origin). */
static double vq_d2(const double* x, const double* c, int E, double xs, double cs) {
    if (E < 5) {
        double s = 0.0;
        for (int k = 0; k < E; k++) {
            const double d = x[k] - c[k];
            s = s + d * d;
        }
        return s;
    }
    double dot;
    if (E < 32) {
        dot = 0.0;
        for (int k = 0; k < E; k++) dot = fma(x[k], c[k], dot);
    } else {
        double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < E; k++) a[k & 7] = fma(x[k], c[k], a[k & 7]);
        dot = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    }
    return (-2.0 * dot + xs) + cs;
}

static double sqsum(const double* x, int E) {
    double s = 0.0;
    for (int k = 0; k < E; k++) s = s + x[k] * x[k];
    return s;
}

/* vq: labels and distortions of every observation against ncodes codes */
static void vq_(const double (*obs)[ES], int N, int E, const double (*book)[ES], int ncodes, int* lab,
                double* dist) {
    double cs[NMAX];
    for (int c = 0; c < ncodes; c++) cs[c] = sqsum(book[c], E);
    for (int i = 0; i < N; i++) {
        const double xs = sqsum(obs[i], E);
        double low = INFINITY;
        int l = 0;
        for (int c = 0; c < ncodes; c++) {
            const double d = vq_d2(obs[i], book[c], E, xs, cs[c]);
            if (d < low) {
                low = d;
                l = c;
            }
        }
        lab[i] = l;
        dist[i] = low > 0 ? sqrt(low) : 0.0;
    }
}

/* scipy.cluster.vq._kmeans: Lloyd steps until |avg_prev - avg| <= 1e-5; returns the
 * code count, *avg = the last mean distortion (np.mean: pairwise sum / N) */
static int kmeans_run(const double (*obs)[ES], int N, int E, double (*book)[ES], int ncodes, double* avg) {
    double prev0 = INFINITY, prev1 = INFINITY;
    int first = 1;
    for (int it = 0;; it++) {
        int lab[NMAX];
        double dist[NMAX];
        vq_(obs, N, E, (const double (*)[ES])book, ncodes, lab, dist);
        const double a = pw_sum(dist, N) / (double)N;
        if (first) {
            prev1 = a;
            first = 0;
        } else {
            prev0 = prev1;
            prev1 = a;
        }
        /* update_cluster_means: member sums in row order, then / count; empty codes dropped */
        double sum[NMAX][ES];
        int cnt[NMAX] = {0};
        for (int c = 0; c < ncodes; c++)
            for (int k = 0; k < E; k++) sum[c][k] = 0.0;
        for (int i = 0; i < N; i++) {
            cnt[lab[i]]++;
            for (int k = 0; k < E; k++) sum[lab[i]][k] = sum[lab[i]][k] + obs[i][k];
        }
        int m = 0;
        for (int c = 0; c < ncodes; c++)
            if (cnt[c] > 0) {
                for (int k = 0; k < E; k++) book[m][k] = sum[c][k] / (double)cnt[c];
                m++;
            }
        ncodes = m;
        const double diff = fabs(prev0 - prev1);
        if (!(diff > 1e-5) || it + 1 >= 4096) break;  /* 4096: the device's guard (KMEANS_MAXIT) */
    }
    *avg = prev1;
    return ncodes;
}

static void kmeans_nc(const double (*F)[ES], const double* mu, int N, int E, int k, int restarts,
                      const int32_t* init, double* nc) {
    /* whiten(wcd): per-column population std (np.std axis 0: sequential column sums,
     * pairwise when E == 1), zero std -> 1 */
    static __thread double obs[NMAX][ES];
    double sd[EMAX];
    for (int j = 0; j < E; j++) {
        double col[NMAX], sq[NMAX];
        for (int i = 0; i < N; i++) col[i] = F[i][j] - mu[j];
        double s = 0.0;
        if (E == 1) s = pw_sum(col, N);
        else for (int i = 0; i < N; i++) s = s + col[i];
        const double m = s / (double)N;
        for (int i = 0; i < N; i++) sq[i] = (col[i] - m) * (col[i] - m);
        double v = 0.0;
        if (E == 1) v = pw_sum(sq, N);
        else for (int i = 0; i < N; i++) v = v + sq[i];
        sd[j] = sqrt(v / (double)N);
        if (sd[j] == 0.0) sd[j] = 1.0;
    }
    for (int i = 0; i < N; i++)
        for (int j = 0; j < E; j++) obs[i][j] = (F[i][j] - mu[j]) / sd[j];
    static __thread double book[NMAX][ES], best[NMAX][ES];
    double best_d = INFINITY;
    int best_n = 0;
    for (int r = 0; r < restarts; r++) {
        for (int c = 0; c < k; c++) memcpy(book[c], obs[init[r * k + c]], sizeof(double) * E);
        double d;
        const int n = kmeans_run((const double (*)[ES])obs, N, E, book, k, &d);
        if (d < best_d) {
            best_d = d;
            best_n = n;
            for (int c = 0; c < n; c++) memcpy(best[c], book[c], sizeof(double) * E);
        }
    }
    if (best_n == 0) {  /* no restart with a finite distortion: the reference raises */
        for (int i = 0; i < N; i++) nc[i] = NAN;
        return;
    }
    int lab[NMAX], cnt[NMAX] = {0}, size[NMAX];
    double dist[NMAX];
    vq_((const double (*)[ES])obs, N, E, (const double (*)[ES])best, best_n, lab, dist);
    for (int i = 0; i < N; i++) cnt[lab[i]]++;
    for (int i = 0; i < N; i++) size[i] = cnt[lab[i]];
    nc_from_sizes(size, N, nc);
}

/* clusterfeck L2dist (:148-149): sqrt(np.sum((v1 - v2)**2)), numpy pairwise sum */
static double l2dist(const double* a, const double* b, int E) {
    double sq[EMAX];
    for (int k = 0; k < E; k++) sq[k] = (a[k] - b[k]) * (a[k] - b[k]);
    return sqrt(pw_sum(sq, E));
}

typedef struct {
    int n;                 /* clusters */
    int first[NMAX];       /* first member (its row is a singleton's meanVec) */
    int count[NMAX];
    double rep[NMAX];      /* cmax.rep: running sum of member weights */
    double sum[NMAX][ES];  /* sum(vec * repVec, axis=0): running, in member order */
    int of[NMAX];          /* cluster of each row, -1 = none */
} feck_t;

static void feck_mean(const feck_t* c, const double (*F)[ES], int x, int E, double* m) {
    for (int k = 0; k < E; k++) m[k] = c->count[x] == 1 ? F[c->first[x]][k] : c->sum[x][k] / c->rep[x];
}

/* Oracle.cluster (:194-230): rows in order join the nearest cluster (first minimum)
 * when its mean is closer than thr, else found a new cluster (rows with NaN never do);
 * returns the mode (first cluster of largest weight, :162-165) */
static int feck_pass(feck_t* c, const double (*F)[ES], const double* w, int N, int E, double thr) {
    c->n = 0;
    for (int i = 0; i < N; i++) {
        c->of[i] = -1;
        double sd = 0x1p255;  /* 2**255 */
        int bx = -1;
        for (int x = 0; x < c->n; x++) {
            double m[EMAX];
            feck_mean(c, F, x, E, m);
            const double d = l2dist(F[i], m, E);
            if (d < sd) {
                sd = d;
                bx = x;
            }
        }
        if (bx >= 0 && sd < thr) {
            for (int k = 0; k < E; k++) c->sum[bx][k] = c->sum[bx][k] + F[i][k] * w[i];
            c->rep[bx] = c->rep[bx] + w[i];
            c->count[bx]++;
            c->of[i] = bx;
        } else {
            int hasnan = 0;
            for (int k = 0; k < E; k++) hasnan |= isnan(F[i][k]);
            if (!hasnan) {
                const int x = c->n++;
                c->first[x] = i;
                c->count[x] = 1;
                c->rep[x] = w[i];
                for (int k = 0; k < E; k++) c->sum[x][k] = F[i][k] * w[i];
                c->of[i] = x;
            }
        }
    }
    int mode = -1;
    double top = 0.0;
    for (int x = 0; x < c->n; x++)
        if (c->rep[x] > top) {
            top = c->rep[x];
            mode = x;
        }
    return mode;
}

/* per-row distance of its cluster's mean to the best mode's mean (:177-183) */
static void feck_rowdist(const feck_t* c, const double (*F)[ES], int mode, int N, int E, double* dm) {
    double mm[EMAX], dx[NMAX];
    feck_mean(c, F, mode, E, mm);
    for (int x = 0; x < c->n; x++) {
        double m[EMAX];
        feck_mean(c, F, x, E, m);
        dx[x] = l2dist(mm, m, E);
    }
    for (int i = 0; i < N; i++) dm[i] = c->of[i] >= 0 ? dx[c->of[i]] : 0.0;
}

/* clusterfeck: outsideCluster(reports_filled, reptokens) (:185-196, :150-183) */
static void feck_nc(const double (*F)[ES], const double* tok, int N, int E, double thr, double* nc) {
    double w[NMAX];
    for (int i = 0; i < N; i++) w[i] = tok[i] == 0.0 ? 0.00001 : tok[i];  /* :202-204, in the caller's list */
    if (!(thr > 0.0)) {
        thr = log10((double)E) / 1.77;
        if (thr == 0.0) thr = 0.3;
    }
    /* outcomes = np.ma.average(features, axis=0, weights=rep) (:167) */
    double outc[EMAX];
    {
        const double scl = pw_sum(w, N);
        for (int k = 0; k < E; k++) {
            double num;
            if (E == 1) {
                double p[NMAX];
                for (int i = 0; i < N; i++) p[i] = F[i][k] * w[i];
                num = pw_sum(p, N);
            } else {
                num = F[0][k] * w[0];
                for (int i = 1; i < N; i++) num = num + F[i][k] * w[i];
            }
            outc[k] = num / scl;
        }
    }
    static __thread feck_t c1, c2;
    double dm[NMAX], m[EMAX];
    const int mode1 = feck_pass(&c1, F, w, N, E, thr);
    feck_mean(&c1, F, mode1, E, m);
    const double d1 = l2dist(m, outc, E);
    /* best = mode1 (bestDist starts at 2**255); a far mode re-clusters once with 3 x thr */
    feck_rowdist(&c1, F, mode1, N, E, dm);
    if (d1 > 1.07) {
        const int mode2 = feck_pass(&c2, F, w, N, E, thr * 3);
        feck_mean(&c2, F, mode2, E, m);
        const double d2 = l2dist(m, outc, E);
        if (d2 < d1) feck_rowdist(&c2, F, mode2, N, E, dm);
    }
    double mx = dm[0];  /* np.amax: NaN propagates */
    for (int i = 1; i < N; i++)
        if (isnan(dm[i]) || dm[i] > mx) mx = isnan(mx) ? mx : dm[i];
    double rv[NMAX];
    for (int i = 0; i < N; i++) rv[i] = 1.0 - dm[i] / (mx + 0.00000001);
    normalize_(rv, N, nc);
}

#define OUT(p, idx, val) do { if (p) (p)[idx] = (val); } while (0)

static void one_round(const pcx_batch* in, pcx_batch_result* out, int64_t b) {
    const int N = (int)in->n_reporters, E = (int)in->n_events;
    const double* Rin = in->reports + b * N * E;
    const int has_bounds = in->scaled != NULL;
    const int64_t bo = in->bounds_shared ? 0 : b * E;
    double X[NMAX][ES], F[NMAX][ES];
    double rep[NMAX], tok[NMAX];
    unsigned char isnan_[NMAX][EMAX], iszero[NMAX][EMAX];
    int scaled[EMAX];
    double lo[EMAX], hi[EMAX];
    for (int j = 0; j < E; j++) {
        scaled[j] = has_bounds ? in->scaled[bo + j] != 0 : 0;
        lo[j] = has_bounds ? in->lo[bo + j] : 0.0;
        hi[j] = has_bounds ? in->hi[bo + j] : 0.0;
    }
    /* --- a1: reputation (__init__.py:138-146) --- */
    if (in->reputation) {
        const double* rr = in->reputation + b * N;
        double tot = pw_sum(rr, N);
        for (int i = 0; i < N; i++) rep[i] = rr[i] / tot;
    } else {
        for (int i = 0; i < N; i++) rep[i] = 1.0 / (double)N;
    }
    double sumtok = 0.0;
    for (int i = 0; i < N; i++) {
        tok[i] = trunc(rep[i] * 1e6);
        sumtok += tok[i];
    }
    const double denom = sumtok - 1.0;
    /* --- a2: rescale (:266-269), NA detection (:278) --- */
    for (int i = 0; i < N; i++)
        for (int j = 0; j < E; j++) {
            double x = Rin[(int64_t)i * E + j];
            if (scaled[j]) {
                x = (x - lo[j]) / (hi[j] - lo[j]);
                if (in->int_dtype) x = trunc(x);
            }
            X[i][j] = x;
            isnan_[i][j] = isnan(x) != 0;
            iszero[i][j] = x == 0.0;
            OUT(out->original, (b * N + i) * E + j, x);
        }
    /* --- a3: interpolate (:284-313) --- */
    for (int i = 0; i < N; i++) memcpy(F[i], X[i], sizeof(double) * E);
    for (int j = 0; j < E; j++) {
        int nmiss = 0;
        for (int i = 0; i < N; i++) nmiss += isnan_[i][j] | iszero[i][j];
        if (!nmiss) continue;
        double tot = 0.0;
        int np_ = 0;
        double xp[NMAX], wp[NMAX];
        for (int i = 0; i < N; i++)
            if (!(isnan_[i][j] | iszero[i][j])) {
                tot += rep[i];
                xp[np_++] = X[i][j];
            }
        double g;
        if (scaled[j]) {
            int m = 0;
            for (int i = 0; i < N; i++)
                if (!(isnan_[i][j] | iszero[i][j])) wp[m++] = rep[i] / tot;
            g = wmedian(xp, wp, np_);
        } else {
            g = 0.0;
            int m = 0;
            for (int i = 0; i < N; i++)
                if (!(isnan_[i][j] | iszero[i][j])) g += (rep[i] / tot) * xp[m++];
            g = catch_(g, in->catch_tolerance);
        }
        if (in->int_dtype) g = trunc(g);
        for (int i = 0; i < N; i++)
            if (isnan_[i][j] | iszero[i][j]) F[i][j] = g;
    }
    for (int i = 0; i < N; i++)
        for (int j = 0; j < E; j++) OUT(out->filled, (b * N + i) * E + j, F[i][j]);

    double loading[EMAX], s[NMAX], nc[NMAX];
    int flags = 0, iters = 0, branch = PCX_BRANCH_NONE;
    double old[EMAX];
    for (int j = 0; j < E; j++) old[j] = ob_vecmat(rep, &F[0][j], ES, N, E, j);  /* np.dot(rep, F) */
    const int alg = in->algorithm;
    const int pca_like = alg == PCX_ALG_PCA || alg == PCX_ALG_BIG_FIVE || alg == PCX_ALG_FIXED_VARIANCE;
    int comps = -1;
    for (int j = 0; j < E; j++) loading[j] = 0.0; /* no wpca: first_loading = zeros (:359) */
    for (int i = 0; i < N; i++) s[i] = nc[i] = 0.0;
    double mu[EMAX];
    if (pca_like || alg >= PCX_ALG_KMEANS) {  /* the clustering algorithms call wpca too (:393, :408, :422) */
        /* --- a5: weighted mean (np.ma.average, :317-319) --- */
        double den = pw_sum(rep, N);
        for (int j = 0; j < E; j++) {
            double acc;
            if (E == 1) {
                double p[NMAX];
                for (int i = 0; i < N; i++) p[i] = F[i][j] * rep[i];
                acc = pw_sum(p, N);
            } else {
                acc = F[0][j] * rep[0];
                for (int i = 1; i < N; i++) acc = acc + F[i][j] * rep[i];
            }
            mu[j] = acc / den;
        }
        /* --- a6: token-weighted covariance (:326), lower triangle, mirrored --- */
        static __thread double C[EMAX][ES];
        for (int j = 0; j < E; j++)
            for (int k = 0; k <= j; k++) {
                double acc = 0.0;
                for (int i = 0; i < N; i++) acc = fma((F[i][j] - mu[j]) * tok[i], F[i][k] - mu[k], acc);
                C[j][k] = acc / denom;
                C[k][j] = C[j][k];
            }
        /* --- a7: leading eigenvector (:330-336), scores (:337) --- */
        double v[EMAX], sq[EMAX];
        iters = power_iter((const double (*)[ES])C, E, v, &flags);
        for (int j = 0; j < E; j++) sq[j] = v[j] * v[j];
        double nv = sqrt(pw_sum(sq, E));
        for (int j = 0; j < E; j++) loading[j] = v[j] / nv;
        if (alg >= PCX_ALG_KMEANS) {
            /* loading only: scores stay zeros */
        } else if (alg == PCX_ALG_PCA) {
            for (int i = 0; i < N; i++) {
                double acc = 0.0;
                for (int j = 0; j < E; j++) acc = fma(F[i][j] - mu[j], loading[j], acc);
                s[i] = acc;
            }
        } else if (flags & PCX_FLAG_SVD_FAIL) {  /* the reference's second svd raises (:375, :431) */
            for (int i = 0; i < N; i++) s[i] = NAN;
        } else {  /* eigenvalue-weighted component scores (:373-390, :429-451) */
            comps = component_scores(alg, (const double (*)[ES])C, E, N, (const double (*)[ES])F, mu,
                                     in->max_components, in->variance_threshold, s);
        }
    } else if (alg == PCX_ALG_COKURTOSIS) {  /* caller-supplied scores (:455-457) */
        for (int i = 0; i < N; i++) s[i] = in->aux_scores[b * N + i];
    }
    const int clustering = alg >= PCX_ALG_KMEANS;
    if (clustering) {  /* scores stay zeros (:357); nc from the clusters */
        if (alg == PCX_ALG_HIERARCHICAL)
            hier_nc((const double (*)[ES])F, mu, N, E, in->hierarchy_threshold, nc);
        else if (alg == PCX_ALG_KMEANS)
            kmeans_nc((const double (*)[ES])F, mu, N, E, in->kmeans_k, in->kmeans_restarts,
                      in->kmeans_init + b * in->kmeans_restarts * in->kmeans_k, nc);
        else
            feck_nc((const double (*)[ES])F, tok, N, E, in->cluster_threshold, nc);
    } else if (alg != PCX_ALG_ABSOLUTE) {
        /* --- a8/a9: nonconformity_rank (:487-500), tie -> nonconformity (:475-485); the
         * other algorithms call nonconformity directly (:389, :450, :456) --- */
        double mn = s[0], mx = s[0];
        for (int i = 1; i < N; i++) {  /* NaN propagates like np.min / np.max */
            if (isnan(s[i]) || s[i] < mn) mn = isnan(mn) ? mn : s[i];
            if (isnan(s[i]) || s[i] > mx) mx = isnan(mx) ? mx : s[i];
        }
        double set1[NMAX], set2[NMAX], n1[NMAX], n2[NMAX];
        for (int i = 0; i < N; i++) {
            set1[i] = s[i] + fabs(mn);
            set2[i] = s[i] - mx;
        }
        normalize_(set1, N, n1);
        normalize_(set2, N, n2);
        double d1[EMAX], d2[EMAX], new1[EMAX], new2[EMAX], r0[EMAX], r1[EMAX], r2[EMAX];
        for (int j = 0; j < E; j++) {
            double a1 = ob_vecmat(n1, &F[0][j], ES, N, E, j);  /* np.dot(normalize(set), F) */
            double a2 = ob_vecmat(n2, &F[0][j], ES, N, E, j);
            d1[j] = a1;
            d2[j] = a2;
            double t = 0.01 * old[j];
            new1[j] = a1 + t;
            new2[j] = a2 + t;
        }
        double e1[EMAX], e2[EMAX];
        double ref = 0.0;  /* non-PCA algorithms: straight to the continuous rule */
        if (alg == PCX_ALG_PCA) {
            rank_avg(old, E, r0);
            rank_avg(new1, E, r1);
            rank_avg(new2, E, r2);
            for (int j = 0; j < E; j++) {
                e1[j] = fabs(r1[j] - r0[j]);
                e2[j] = fabs(r2[j] - r0[j]);
            }
            ref = pw_sum(e1, E) - pw_sum(e2, E);
        }
        int pick1;
        if (ref == 0) {
            for (int j = 0; j < E; j++) {
                double a = d1[j] - old[j], c = d2[j] - old[j];
                e1[j] = a * a;
                e2[j] = c * c;
            }
            double ref2 = pw_sum(e1, E) - pw_sum(e2, E);
            pick1 = ref2 <= 0;
            branch = pick1 ? PCX_BRANCH_TIE_SET1 : PCX_BRANCH_TIE_SET2;
        } else {
            pick1 = ref < 0;
            branch = pick1 ? PCX_BRANCH_SET1 : PCX_BRANCH_SET2;
        }
        for (int i = 0; i < N; i++) nc[i] = pick1 ? set1[i] : set2[i];
    } /* "absolute": nc = 0 (Q13) */
    /* --- a10: reputation update (:460-472) --- */
    double meanrep = pw_sum(rep, N) / (double)N;
    double u[NMAX], this_[NMAX], smooth[NMAX];
    for (int i = 0; i < N; i++) u[i] = nc[i] * (rep[i] / meanrep);
    /* PCA path: this_rep (then smooth_rep) is a MaskedArray, and a NaN total of |u| leaves it
     * fully MASKED (numpy.ma masks the NaN quotient): participation_columns is then
     * 1 - (a fully masked dot) whose data is the 1, and reporter_bonus / author_bonus are fully
     * masked sums whose data is their first operand's -- normalize(participation_rows) and
     * |participation_columns.data| = 1 (__init__.py:460-472, 559-581; golden
     * q_all_missing_scaled_col); percent_na stays masked (participation NaN) */
    int rep_masked = 0;
    if (alg == PCX_ALG_PCA)
        for (int i = 0; i < N; i++) rep_masked |= isnan(u[i]);
    normalize_(u, N, this_);
    const double a = in->alpha, oma = 1.0 - in->alpha;
    for (int i = 0; i < N; i++) smooth[i] = a * this_[i] + oma * rep[i];
    /* --- a12/a13: outcomes (:510-538) --- */
    double raw[EMAX], adj[EMAX], fin[EMAX], cert[EMAX];
    for (int j = 0; j < E; j++) {
        raw[j] = ob_vecmat(smooth, &F[0][j], ES, N, E, j);  /* np.dot(smooth_rep, F) (:510) */
        if (scaled[j]) {
            double col[NMAX];
            for (int i = 0; i < N; i++) col[i] = F[i][j];
            raw[j] = wmedian(col, smooth, N);
            adj[j] = raw[j];
            fin[j] = adj[j] * (hi[j] - lo[j]);
            fin[j] = fin[j] + lo[j];
        } else {
            adj[j] = catch_(raw[j], in->catch_tolerance);
            fin[j] = adj[j];
        }
    }
    /* --- a14: certainty (:540-546) --- */
    for (int j = 0; j < E; j++) {
        double sel[NMAX];
        int m = 0;
        for (int i = 0; i < N; i++)
            if (F[i][j] == adj[j]) sel[m++] = smooth[i];
        /* an empty match sums to NaN only on the PCA path, where smooth_rep is a
         * MaskedArray (masked sum, Q11); the other algorithms' smooth_rep is a plain
         * ndarray and the builtin sum of nothing is 0 (goldens: algos.npz) */
        cert[j] = m ? pw_sum(sel, m) : (alg == PCX_ALG_PCA ? NAN : 0.0);
    }
    double reward[EMAX];
    normalize_(cert, E, reward);
    double avg_cert = pw_sum(cert, E) / (double)E;
    /* --- a15: participation and bonuses (:549-581) --- */
    double pc[EMAX], pr[NMAX], narow[NMAX], rel[NMAX], relc[EMAX];
    for (int j = 0; j < E; j++) {
        double na[NMAX];
        int nz = 0;
        for (int i = 0; i < N; i++) {
            na[i] = (isnan_[i][j] | iszero[i][j]) ? 1.0 : 0.0;
            nz += iszero[i][j];
        }
        pc[j] = 1.0 - dot2(smooth, 1, na, 1, N);
        OUT(out->nas_filled, b * E + j, (double)nz);
    }
    for (int i = 0; i < N; i++) {
        int nz = 0;
        for (int j = 0; j < E; j++) nz += iszero[i][j];
        narow[i] = (double)nz;
        pr[i] = 1.0 - narow[i] / (double)E;
    }
    double pna = 1.0 - pw_sum(pc, E) / (double)E;
    /* A reporter whose every report is NaN has a fully MASKED row in na_mat, so its
     * participation_rows entry is masked: np.sum skips it, and masked arithmetic
     * keeps the first operand's data -- relative_part = |pr| undivided and
     * reporter_bonus = relative_part (quirk Q15, __init__.py:567,576-577). */
    int rowmasked[NMAX];
    for (int i = 0; i < N; i++) {
        int nn = 0;
        for (int j = 0; j < E; j++) nn += isnan_[i][j];
        rowmasked[i] = nn == E;
    }
    {
        double a2[NMAX];
        for (int i = 0; i < N; i++) a2[i] = rowmasked[i] ? 0.0 : fabs(pr[i]);
        double S = pw_sum(a2, N);
        int bump = S == 0;
        if (bump) {
            for (int i = 0; i < N; i++) a2[i] = rowmasked[i] ? 0.0 : fabs(pr[i]) + 1.0;
            S = pw_sum(a2, N);
        }
        for (int i = 0; i < N; i++) rel[i] = rowmasked[i] ? fabs(pr[i]) : a2[i] / S;
    }
    normalize_(pc, E, relc);
    for (int i = 0; i < N; i++) {
        const int64_t o = b * N + i;
        OUT(out->old_rep, o, rep[i]);
        OUT(out->this_rep, o, this_[i]);
        OUT(out->smooth_rep, o, smooth[i]);
        OUT(out->scores, o, s[i]);
        OUT(out->na_row, o, narow[i]);
        OUT(out->participation_rows, o, pr[i]);
        OUT(out->relative_part, o, rel[i]);
        OUT(out->reporter_bonus, o, (rowmasked[i] || rep_masked) ? rel[i] : rel[i] * pna + smooth[i] * (1.0 - pna));
    }
    for (int j = 0; j < E; j++) {
        const int64_t o = b * E + j;
        OUT(out->adj_first_loadings, o, loading[j]);
        OUT(out->outcomes_raw, o, raw[j]);
        OUT(out->outcomes_adjusted, o, adj[j]);
        OUT(out->outcomes_final, o, fin[j]);
        OUT(out->certainty, o, cert[j]);
        OUT(out->consensus_reward, o, reward[j]);
        OUT(out->participation_columns, o, rep_masked ? 1.0 : pc[j]);
        OUT(out->author_bonus, o, rep_masked ? 1.0 : relc[j] * pna + reward[j] * (1.0 - pna));
    }
    OUT(out->participation, b, 1.0 - pna);
    OUT(out->avg_certainty, b, avg_cert);
    OUT(out->branch, b, branch);
    OUT(out->flags, b, flags);
    OUT(out->pi_iters, b, iters);
    OUT(out->components, b, comps);
}

/* Host-memory restatement of pcx_consensus_batched_f64 (same structs). */
int pcxo_consensus_batched_f64(const pcx_batch* in, pcx_batch_result* out, int n_threads) {
    if (!in || !out || in->n_reporters < 1 || in->n_reporters > NMAX || in->n_events < 1 ||
        in->n_events > EMAX || in->n_rounds < 0 || in->algorithm < 0 || in->algorithm > PCX_ALG_CLUSTERFECK)
        return PCX_EINVAL;
    if (in->algorithm == PCX_ALG_KMEANS &&
        (!in->kmeans_init || in->kmeans_k < 1 || in->kmeans_k > in->n_reporters || in->kmeans_restarts < 1))
        return PCX_EINVAL;
    if (in->algorithm == PCX_ALG_BIG_FIVE && (in->max_components < 1 || in->max_components > in->n_events))
        return PCX_EINVAL;
    if (in->algorithm == PCX_ALG_COKURTOSIS && !in->aux_scores) return PCX_EINVAL;
#pragma omp parallel for schedule(dynamic, 64) num_threads(n_threads > 0 ? n_threads : 1)
    for (int64_t b = 0; b < in->n_rounds; b++) one_round(in, out, b);
    return PCX_OK;
}
