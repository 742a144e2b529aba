// pcx_medium.hip -- batched oracle rounds above one wavefront (64 < N <= 256 reporters or
// 32 < E <= 64 events): one 256-thread workgroup per round.
//
// Each round is Oracle(reports, event_bounds, reputation).consensus() (pyconsensus/
// __init__.py:102-611) in the operation order of the batched SPEC
// (oracle/pcx_oracle_batched.c one_round, built with NMAX = 256 for these shapes), so the
// results are bit-identical to it: the reference's own orders where they are known (numpy
// pairwise sums, the OpenBLAS dgemv order of np.dot, weightedstats' sequential walk, the
// interpolation's sequential means) and the SPEC's fixed orders elsewhere (fma chains of the
// covariance and scores, the power iteration with Gram squarings, tree64 norms).
//
// Work split: one thread per event column, per reporter row or per matrix entry, as each
// step allows; the reference's sequential sums stay on one thread.  LDS holds the
// power-iteration matrices, the per-element NA flags and the row / event vectors; the filled
// matrix and the covariance live in a per-round global scratch (L2-resident).
// Algorithms: PCA, "absolute", "big-five", "fixed-variance", "cokurtosis" (the clusterings take
// the round scheduler).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pcx_internal.h"

namespace pcx {
namespace {

constexpr int MT = 256;  // threads per round
constexpr int MN = 256;  // max reporters
constexpr int MEV = 64;  // max events
constexpr double M_PI_TOL = 1e-14;
constexpr int M_PI_MAXIT = 256, M_PI_PRESQUARE = 3, M_PI_SQUARE_EVERY = 32, M_PI_MAX_SQUARINGS = 8,
              M_PI_POLISH = 4;
constexpr double M_DBL_EPS = 2.220446049250313080847e-16;
constexpr double M_DBL_MIN = 2.2250738585072014e-308;

// numpy pairwise sum (SPEC pw_sum) of g(0..n-1), n <= 256: leaves of <= 128, halves rounded
// down to multiples of 8 (the right half of n > 242 splits once more)
template <class G>
__device__ double mpw_leaf(G g, int off, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; i++) r += g(off + i);
        return r;
    }
    double r[8];
    for (int k = 0; k < 8; k++) r[k] = g(off + k);
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int k = 0; k < 8; k++) r[k] += g(off + i + k);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += g(off + i);
    return res;
}
template <class G>
__device__ double mpw_sub(G g, int off, int n) {  // n <= 256: the right half may split once more
    if (n <= 128) return mpw_leaf(g, off, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return mpw_leaf(g, off, n2) + mpw_leaf(g, off + n2, n - n2);
}
template <class G>
__device__ double mpw(G g, int n) {
    if (n <= 128) return mpw_leaf(g, 0, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return mpw_leaf(g, 0, n2) + mpw_sub(g, n2, n - n2);
}

// the same tree64 on wave 0 (lane = slot): the xor butterfly by shuffles; valid on lane 0
template <class G>
__device__ double wtree64(G g, int n) {
    const int l = threadIdx.x & 63;
    double v = l < n ? g(l) : 0.0;
    for (int s = 1; s <= 8; s <<= 1) v = v + __shfl_xor(v, s, 64);
    const double t16 = __shfl(v, 16, 64), t32 = __shfl(v, 32, 64), t48 = __shfl(v, 48, 64);
    return (v + t16) + (t32 + t48);
}

// block compaction: rows with pred(i) in row order -> out[0..m) = val(i); returns m (all threads)
template <class P, class V>
__device__ int bcompact(P pred, V val, int n, double* out, int* wcnt) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int base = 0;
    for (int i0 = 0; i0 < n; i0 += MT) {
        const int i = i0 + (int)threadIdx.x;
        const bool p = i < n && pred(i);
        const unsigned long long bal = __ballot(p);
        if (lane == 0) wcnt[w] = __popcll(bal);
        __syncthreads();
        int off = base;
        for (int k = 0; k < w; k++) off += wcnt[k];
        if (p) out[off + __popcll(bal & ((1ull << lane) - 1ull))] = val(i);
        for (int k = 0; k < MT / 64; k++) base += wcnt[k];
        __syncthreads();
    }
    return base;
}

// SPEC dot2 (compensated dot, index order)
template <class A, class B>
__device__ double mdot2(A a, B b, int n) {
    double s = 0.0, c = 0.0;
    for (int i = 0; i < n; i++) {
        const double x = a(i), y = b(i);
        const double p = x * y;
        const double pe = fma(x, y, -p);
        const double t = s + p;
        const double z = t - s;
        const double se = (s - (t - z)) + (p - z);
        s = t;
        c = c + (pe + se);
    }
    return s + c;
}

// np.dot(v, F)[j] in OpenBLAS's order (SPEC ob_vecmat)
template <class V, class X>
__device__ double mob_vecmat(V v, X F, int N, int E, int j) {
    if (E == 1) {  // numpy's ddot
        double acc8[4][8], acc4[4][4];
        for (int r = 0; r < 4; r++)
            for (int l = 0; l < 8; l++) acc8[r][l] = 0.0;
        const int n32 = N & -32, n16 = N & -16;
        for (int i = 0; i < n32; i += 32)
            for (int k = 0; k < 32; k++) acc8[k / 8][k % 8] = fma(v(i + k), F(i + k), acc8[k / 8][k % 8]);
        for (int r = 0; r < 4; r++)
            for (int l = 0; l < 4; l++) acc4[r][l] = acc8[r][l] + acc8[r][l + 4];
        for (int i = n32; i < n16; i += 16)
            for (int k = 0; k < 16; k++) acc4[k / 4][k % 4] = fma(v(i + k), F(i + k), acc4[k / 4][k % 4]);
        double A[4];
        for (int l = 0; l < 4; l++) A[l] = ((acc4[0][l] + acc4[1][l]) + acc4[2][l]) + acc4[3][l];
        double d = (A[0] + A[2]) + (A[1] + A[3]);
        for (int i = n16; i < N; i++) d = fma(v(i), F(i), d);
        return d;
    }
    if (j < (E & ~3)) {
        double y = 0.0;
        int n = 0;
        for (; n + 4 <= N; n += 4) {
            double t = F(n + 1) * v(n + 1);
            t = fma(F(n), v(n), t);
            t = fma(F(n + 2), v(n + 2), t);
            t = fma(F(n + 3), v(n + 3), t);
            y = y + t;
        }
        if (n + 2 <= N) {
            double t = F(n + 1) * v(n + 1);
            t = fma(F(n), v(n), t);
            y = y + t;
            n += 2;
        }
        if (n < N) y = y + F(n) * v(n);
        return y;
    }
    double t = 0.0;
    int i = 0;
    if (E == 2 || E == 3)
        for (; i + 4 <= N; i += 4) {
            t = t + fma(F(i), v(i), F(i + 1) * v(i + 1));
            t = t + fma(F(i + 2), v(i + 2), F(i + 3) * v(i + 3));
        }
    for (; i < N; i++) t = fma(F(i), v(i), t);
    return t;
}

__device__ __forceinline__ double mcatch(double x, double tol) {
    if (x < 1.5 - tol) return 1.0;
    if (x > 1.5 + tol) return 2.0;
    return 1.5;
}

// block reductions (max of doubles / first index)
__device__ double bmax(double v, double* sh) {
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int s = MT / 2; s >= 1; s >>= 1) {
        if ((int)threadIdx.x < s) sh[threadIdx.x] = fmax(sh[threadIdx.x], sh[threadIdx.x + s]);
        __syncthreads();
    }
    const double r = sh[0];
    __syncthreads();
    return r;
}

// weightedstats.weighted_median of n <= 256 (x, w) pairs in LDS (SPEC wmedian), the whole
// block cooperating on the stable (x, w) ranks; the result on every thread
__device__ double mwmedian(const double* x, const double* w, int n, double* xs, double* ws, double* sh) {
    __shared__ double res_s;
    if (threadIdx.x == 0) {
        double W = 0.0;
        for (int i = 0; i < n; i++) W += w[i];
        const double mid = 0.5 * W;
        int dom = 0, pos = 0;
        for (int i = 0; i < n; i++) {
            dom |= w[i] > mid;
            pos |= w[i] > 0;
        }
        double r = __builtin_nan("");
        if (dom) {
            double m = w[0];
            for (int i = 1; i < n; i++)
                if (w[i] > m) m = w[i];
            for (int i = 0; i < n; i++)
                if (w[i] == m) {
                    r = x[i];
                    break;
                }
            sh[0] = 1.0;  // decided
        } else {
            sh[0] = pos ? 0.0 : 1.0;
        }
        sh[1] = mid;
        res_s = r;
    }
    __syncthreads();
    const bool decided = sh[0] != 0.0;
    const double mid = sh[1];
    __syncthreads();
    if (decided) return res_s;
    for (int i = threadIdx.x; i < n; i += MT) {  // stable rank by (x, w)
        int r = 0;
        const double xi = x[i], wi = w[i];
        for (int m = 0; m < n; m++) {
            const bool lt = (x[m] < xi) || (x[m] == xi && w[m] < wi);
            const bool eq = (x[m] == xi) && (w[m] == wi);
            r += (lt || (eq && m < i)) ? 1 : 0;
        }
        xs[r] = xi;
        ws[r] = wi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double cum = 0.0, r;
        int k = 0;
        bool fail = false;
        while (cum <= mid) {
            if (k == n) {
                fail = true;
                break;
            }
            cum += ws[k];
            k++;
        }
        if (fail) {
            r = __builtin_nan("");
        } else {
            const double before = cum - ws[k - 1];
            if (fabs(before - mid) < M_DBL_EPS) {
                if (k >= 2) r = (xs[k - 2] + xs[k - 1]) / 2.0;
                else if (n == 1) r = xs[0] / 1.0;
                else r = __builtin_nan("");
            } else {
                r = xs[k - 1];
            }
        }
        res_s = r;
    }
    __syncthreads();
    const double r = res_s;
    __syncthreads();
    return r;
}

// "big-five" / "fixed-variance" (:373-390, :429-451), SPEC component_scores: eigenpairs of C by
// cyclic two-sided Jacobi with the round-robin pair schedule (every step's pairs disjoint: one
// thread per pair for the angles, per (pair, index) for the rotations, rows then columns), Sigma
// descending (ties by index), net_i = sum_c Sigma_c (wcd_i . loading_c) over the components.
// A = M, V = Tm (LDS, stride ES); returns the fixed-variance count, else -1.
constexpr int M_JAC_MAXSWEEP = 30;
constexpr double M_JAC_TOL = 1e-15;

__device__ __forceinline__ void mjac_pair(int i, int r, int n, int& p, int& q) {
    const int a = i == 0 ? 0 : 1 + (i - 1 + r) % (n - 1);
    const int b = 1 + (n - 2 - i + r) % (n - 1);
    p = a < b ? a : b;
    q = a < b ? b : a;
}

__device__ int component_scores(const BatchArgs& a, const double* C, double* A, double* V, int ES, const double* F,
                                const double* mu, double* net, double* sh, double* scal) {
    const int E = a.E, N = a.N, tid = threadIdx.x;
    __shared__ double cc[MEV / 2 + 1], ss[MEV / 2 + 1];
    __shared__ int pp[MEV / 2 + 1], qq[MEV / 2 + 1];
    __shared__ int order[MEV];
    __shared__ double sig[MEV];
    for (int e = tid; e < E * E; e += MT) {
        const int j = e / E, k = e % E;
        A[j * ES + k] = C[e];
        V[j * ES + k] = j == k ? 1.0 : 0.0;
    }
    __syncthreads();
    if (tid == 0) scal[0] = mpw([&](int j) { return C[j * E + j]; }, E);  // np.trace: add.reduce
    if (E >= 2) {
        const int n = E + (E & 1), npair = n / 2;
        for (int sweep = 0; sweep < M_JAC_MAXSWEEP; sweep++) {
            double off = 0.0, dg = 0.0;  // max-norms: exact in any order
            for (int e = tid; e < E * E; e += MT) {
                const int j = e / E, k = e % E;
                const double v = fabs(A[j * ES + k]);
                if (j == k) dg = fmax(dg, v);
                else off = fmax(off, v);
            }
            off = bmax(off, sh);
            dg = bmax(dg, sh);
            if (!(off > M_JAC_TOL * dg)) break;  // block-uniform
            for (int r = 0; r < n - 1; r++) {
                for (int i = tid; i < npair; i += MT) {
                    int p, q;
                    mjac_pair(i, r, n, p, q);
                    pp[i] = p;
                    qq[i] = q;
                    double c = 1.0, sn = 0.0;
                    if (q < E) {
                        const double app = A[p * ES + p], aqq = A[q * ES + q], apq = A[p * ES + q];
                        if (apq != 0.0) {
                            const double tau = (aqq - app) / (2.0 * apq);
                            const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
                            c = 1.0 / sqrt(1.0 + t * t);
                            sn = t * c;
                        }
                    }
                    cc[i] = c;
                    ss[i] = sn;
                }
                __syncthreads();
                for (int e = tid; e < npair * E; e += MT) {  // rows
                    const int i = e / E, k = e % E;
                    if (ss[i] == 0.0) continue;
                    const int p = pp[i], q = qq[i];
                    const double c = cc[i], sn = ss[i];
                    const double apk = A[p * ES + k], aqk = A[q * ES + k];
                    A[p * ES + k] = c * apk - sn * aqk;
                    A[q * ES + k] = sn * apk + c * aqk;
                }
                __syncthreads();
                for (int e = tid; e < npair * E; e += MT) {  // columns of A and V
                    const int i = e / E, j = e % E;
                    if (ss[i] == 0.0) continue;
                    const int p = pp[i], q = qq[i];
                    const double c = cc[i], sn = ss[i];
                    const double ajp = A[j * ES + p], ajq = A[j * ES + q];
                    A[j * ES + p] = c * ajp - sn * ajq;
                    A[j * ES + q] = sn * ajp + c * ajq;
                    const double vjp = V[j * ES + p], vjq = V[j * ES + q];
                    V[j * ES + p] = c * vjp - sn * vjq;
                    V[j * ES + q] = sn * vjp + c * vjq;
                }
                __syncthreads();
            }
        }
    }
    for (int j = tid; j < E; j += MT) sig[j] = fabs(A[j * ES + j]);
    __syncthreads();
    for (int j = tid; j < E; j += MT) {  // descending Sigma, ties by index
        int rk = 0;
        for (int k = 0; k < E; k++) rk += (sig[k] > sig[j]) || (sig[k] == sig[j] && k < j);
        order[rk] = j;
    }
    __syncthreads();
    const int kmax = a.algorithm == PCX_ALG_BIG_FIVE ? a.max_components : E;
    if (tid == 0) {  // fixed-variance: cumsum(Sigma / trace) >= threshold stops after that component
        int used = kmax;
        if (a.algorithm == PCX_ALG_FIXED_VARIANCE) {
            double ve = 0.0;
            for (int c = 0; c < kmax; c++) {
                ve = ve + sig[order[c]] / scal[0];
                if (ve >= a.variance_threshold) {
                    used = c + 1;
                    break;
                }
            }
        }
        scal[1] = (double)used;
    }
    __syncthreads();
    const int used = (int)scal[1];
    for (int i = tid; i < N; i += MT) {
        double acc = 0.0;
        for (int c = 0; c < used; c++) {
            const int idx = order[c];
            const double sg = sig[idx];
            const double fl = V[idx] < 0.0 ? -1.0 : 1.0;  // loading *= -1 if loading[0] < 0
            double d = 0.0;
            for (int j = 0; j < E; j++) d = fma(F[i * E + j] - mu[j], fl * V[j * ES + idx], d);
            acc = acc + sg * d;
        }
        net[i] = acc;
    }
    __syncthreads();
    return a.algorithm == PCX_ALG_FIXED_VARIANCE ? used : -1;
}

struct MedLds {  // offsets (doubles) into the dynamic LDS
    int M, T, vN, vE, flags;
};

// N-vectors (each N doubles): REP, TOK, S, SET1, SET2, NW1, NW2, U, THIS, SMOOTH, XA, WA, XS, WS
enum { VN_REP = 0, VN_TOK, VN_S, VN_SET1, VN_SET2, VN_NW1, VN_NW2, VN_U, VN_THIS, VN_SMOOTH, VN_XA, VN_WA, VN_XS,
       VN_WS, VN_COUNT };
// E-vectors (each E doubles)
enum { VE_MU = 0, VE_OLD, VE_LD, VE_X, VE_Y, VE_SQ, VE_D1, VE_D2, VE_NEW1, VE_NEW2, VE_R0, VE_R1, VE_R2, VE_E1, VE_E2,
       VE_RAW, VE_ADJ, VE_FIN, VE_CERT, VE_REWARD, VE_PC, VE_RELC, VE_COUNT };

// diagnostic phase stamps (PCX_STAMPS=1): shader-clock reads at phase boundaries
#define MSTAMP(k)                                                                 \
    do {                                                                          \
        if (a.stamps) {                                                           \
            const long long t_ = (long long)__builtin_amdgcn_s_memtime();         \
            if (threadIdx.x == 0) a.stamps[b * 32 + (k)] = t_;                    \
        }                                                                         \
    } while (0)

__global__ void __launch_bounds__(MT) medium_round_kernel(BatchArgs a, int64_t b0, double* Fscr, double* Cscr) {
    extern __shared__ __attribute__((aligned(16))) double mlds[];
    __shared__ double sh[MT];
    __shared__ double scal[16];
    const int64_t b = b0 + blockIdx.x;  // round; scratch slot blockIdx.x
    const int N = a.N, E = a.E, ES = E + 1;
    const int tid = threadIdx.x;
    double* M = mlds;
    double* Tm = M + E * ES;
    double* vN = Tm + E * ES;
    double* vE = vN + VN_COUNT * N;
    uint8_t* fl = (uint8_t*)(vE + VE_COUNT * E);  // [N][E] bit 0 NaN, bit 1 zero
    auto VNp = [&](int k) { return vN + k * N; };
    auto VEp = [&](int k) { return vE + k * E; };
    double* rep = VNp(VN_REP);
    double* tok = VNp(VN_TOK);
    const double* Rin = a.reports + b * N * E;
    double* F = a.filled ? a.filled + b * N * E : Fscr + (int64_t)blockIdx.x * N * E;
    double* C = Cscr + (int64_t)blockIdx.x * E * E;
    const int64_t bo = a.bounds_shared ? 0 : b * E;
    const bool has_bounds = a.scaled != nullptr;
    auto scaled = [&](int j) { return has_bounds && a.scaled[bo + j] != 0; };
    const int alg = a.algorithm;
    MSTAMP(0);

    // --- a1: reputation (:138-146)
    if (tid == 0) scal[0] = a.reputation ? mpw([&](int i) { return a.reputation[b * N + i]; }, N) : 0.0;
    __syncthreads();
    for (int i = tid; i < N; i += MT) {
        const double r = a.reputation ? a.reputation[b * N + i] / scal[0] : 1.0 / (double)N;
        rep[i] = r;
        tok[i] = trunc(r * 1e6);
    }
    __syncthreads();
    if (tid == 0) {
        double st = 0.0;
        for (int i = 0; i < N; i++) st += tok[i];
        scal[1] = st - 1.0;  // denom
    }
    // --- a2: rescale (:266-269), NA (:278)
    for (int e = tid; e < N * E; e += MT) {
        const int j = e % E;
        double x = Rin[e];
        if (scaled(j)) {
            x = (x - a.lo[bo + j]) / (a.hi[bo + j] - a.lo[bo + j]);
            if (a.int_dtype) x = trunc(x);
        }
        F[e] = x;
        fl[e] = (uint8_t)((__builtin_isnan(x) ? 1 : 0) | (x == 0.0 ? 2 : 0));
        if (a.original) a.original[b * N * E + e] = x;
    }
    __syncthreads();
    MSTAMP(1);
    // --- a3: interpolate (:284-313): binary columns one thread each; scaled columns one at a
    // time with the whole block (weighted median)
    double* XA = VNp(VN_XA);
    double* WA = VNp(VN_WA);
    for (int j = tid; j < E; j += MT) {
        if (scaled(j)) continue;
        int nmiss = 0;
        double tot = 0.0;
        for (int i = 0; i < N; i++) {
            const bool m = fl[i * E + j] != 0;
            nmiss += m ? 1 : 0;
            if (!m) tot += rep[i];
        }
        if (!nmiss) continue;
        double g = 0.0;
        for (int i = 0; i < N; i++)
            if (!fl[i * E + j]) g += (rep[i] / tot) * F[i * E + j];
        g = mcatch(g, a.catch_tol);
        if (a.int_dtype) g = trunc(g);
        for (int i = 0; i < N; i++)
            if (fl[i * E + j]) F[i * E + j] = g;
    }
    MSTAMP(2);
    __shared__ int wcnt[MT / 64];
    for (int j = 0; j < E; j++) {
        if (!scaled(j)) continue;
        // present values and their reputations in row order (block compaction), then the
        // sequential present total on one thread and the weights rep / total
        const int np_ = bcompact([&](int i) { return fl[i * E + j] == 0; }, [&](int i) { return F[i * E + j]; }, N, XA,
                                 wcnt);
        bcompact([&](int i) { return fl[i * E + j] == 0; }, [&](int i) { return rep[i]; }, N, WA, wcnt);
        if (tid == 0) {
            double tot = 0.0;
            for (int q = 0; q < np_; q++) tot += WA[q];
            scal[2] = tot;
        }
        __syncthreads();
        for (int q = tid; q < np_; q += MT) WA[q] = WA[q] / scal[2];
        __syncthreads();
        const int nmiss = N - np_;
        if (nmiss) {  // block-uniform
            double g = mwmedian(XA, WA, np_, VNp(VN_XS), VNp(VN_WS), sh);
            if (a.int_dtype) g = trunc(g);
            for (int i = tid; i < N; i += MT)
                if (fl[i * E + j]) F[i * E + j] = g;
        }
        __syncthreads();
    }
    __syncthreads();
    MSTAMP(3);
    // old = np.dot(rep, F) (:489)
    for (int j = tid; j < E; j += MT)
        VEp(VE_OLD)[j] = mob_vecmat([&](int i) { return rep[i]; }, [&](int i) { return F[i * E + j]; }, N, E, j);
    double* loading = VEp(VE_LD);
    double* s = VNp(VN_S);
    double* nc = VNp(VN_U);  // nc, then u
    int flags = 0, iters = 0, branch = PCX_BRANCH_NONE;
    for (int j = tid; j < E; j += MT) loading[j] = 0.0;
    for (int i = tid; i < N; i += MT) s[i] = nc[i] = 0.0;
    __syncthreads();
    MSTAMP(4);
    int comps = -1;
    if (alg == PCX_ALG_PCA || alg == PCX_ALG_BIG_FIVE || alg == PCX_ALG_FIXED_VARIANCE) {
        // --- a5: weighted mean (np.ma.average, :317-319)
        double* mu = VEp(VE_MU);
        if (tid == 0) scal[4] = mpw([&](int i) { return rep[i]; }, N);
        __syncthreads();
        for (int j = tid; j < E; j += MT) {
            double acc;
            if (E == 1) {
                acc = mpw([&](int i) { return F[i * E + j] * rep[i]; }, N);
            } else {
                acc = F[j] * rep[0];
                for (int i = 1; i < N; i++) acc = acc + F[i * E + j] * rep[i];
            }
            mu[j] = acc / scal[4];
        }
        __syncthreads();
        MSTAMP(5);
        // --- a6: covariance (:326), lower triangle mirrored
        const double denom = scal[1];
        for (int e = tid; e < E * E; e += MT) {
            const int j = e / E, k = e % E;
            if (k > j) continue;
            double acc = 0.0;
            for (int i = 0; i < N; i++) acc = fma((F[i * E + j] - mu[j]) * tok[i], F[i * E + k] - mu[k], acc);
            const double c = acc / denom;
            C[j * E + k] = c;
            C[k * E + j] = c;
        }
        __syncthreads();
        MSTAMP(6);
        // --- a7: power iteration (SPEC power_iter)
        int finite = 1, nonzero = 0;
        for (int e = tid; e < E * E; e += MT) {
            finite &= __builtin_isfinite(C[e]) ? 1 : 0;
            nonzero |= C[e] != 0.0 ? 1 : 0;
        }
        finite = __syncthreads_and(finite);
        nonzero = __syncthreads_or(nonzero);
        double* x = VEp(VE_X);
        double* y = VEp(VE_Y);
        if (!finite) {
            for (int j = tid; j < E; j += MT) x[j] = 1.0;
            flags |= PCX_FLAG_SVD_FAIL;
        } else if (!nonzero) {
            for (int j = tid; j < E; j += MT) x[j] = j == 0 ? 1.0 : 0.0;
            flags |= PCX_FLAG_ZERO_COV;
        } else {
            if (tid == 0) {
                int kd = 0;
                for (int j = 1; j < E; j++)
                    if (C[j * E + j] > C[kd * E + kd]) kd = j;
                scal[5] = (double)kd;
            }
            __syncthreads();
            if (tid < 64) {
                const int kd0 = (int)scal[5];
                const double t = sqrt(wtree64([&](int j) { const double v = C[j * E + kd0]; return v * v; }, E));
                if (tid == 0) scal[6] = t;
            }
            __syncthreads();
            const int kd = (int)scal[5];
            for (int j = tid; j < E; j += MT) x[j] = C[j * E + kd] / scal[6];
            for (int e = tid; e < E * E; e += MT) M[(e / E) * ES + e % E] = C[e];
            __syncthreads();
            auto square = [&]() {  // M <- (M M) * 2^-ilogb(max|MM|)
                double lm = 0.0;
                for (int e = tid; e < E * E; e += MT) {
                    const int j = e / E, k = e % E;
                    double acc = 0.0;
                    for (int l = 0; l < E; l++) acc = fma(M[j * ES + l], M[l * ES + k], acc);
                    Tm[j * ES + k] = acc;
                    const double v = fabs(acc);
                    if (v > lm) lm = v;
                }
                const double mx = bmax(lm, sh);
                const bool pow2 = mx >= M_DBL_MIN && __builtin_isfinite(mx);
                const double sc = pow2 ? ldexp(1.0, -ilogb(mx)) : 1.0;
                for (int e = tid; e < E * E; e += MT) {
                    const int j = e / E, k = e % E;
                    const double t = Tm[j * ES + k];
                    M[j * ES + k] = pow2 ? t * sc : (mx > 0.0 ? t / mx : t);
                }
                __syncthreads();
            };
            // y = A x / ||A x|| (tree64 norm), A = M (stride ES) or C (stride E)
            auto matvec_unit = [&](const double* A, int lda) {
                for (int j = tid; j < E; j += MT) {
                    double acc = 0.0;
                    for (int k = 0; k < E; k++) acc = fma(A[j * lda + k], x[k], acc);
                    y[j] = acc;
                }
                __syncthreads();
                if (tid < 64) {
                    const double t = sqrt(wtree64([&](int j) { return y[j] * y[j]; }, E));
                    if (tid == 0) scal[7] = t;
                }
                __syncthreads();
                for (int j = tid; j < E; j += MT) y[j] = y[j] / scal[7];
                __syncthreads();
            };
            int sqn = 0;
            for (; sqn < M_PI_PRESQUARE; sqn++) square();
            int since = 0;
            for (;;) {
                matvec_unit(M, ES);
                double ld = 0.0;
                for (int j = tid; j < E; j += MT) ld = fmax(ld, fabs(y[j] - x[j]));
                const double d = bmax(ld, sh);
                for (int j = tid; j < E; j += MT) x[j] = y[j];
                __syncthreads();
                iters++;
                since++;
                if (d <= M_PI_TOL) break;
                if (iters >= M_PI_MAXIT) {
                    flags |= PCX_FLAG_PI_MAXIT;
                    break;
                }
                if (since >= M_PI_SQUARE_EVERY && sqn < M_PI_MAX_SQUARINGS) {
                    square();
                    sqn++;
                    since = 0;
                }
            }
            for (int p = 0; p < M_PI_POLISH; p++) {
                matvec_unit(C, E);
                for (int j = tid; j < E; j += MT) x[j] = y[j];
                __syncthreads();
            }
            iters += M_PI_POLISH + sqn;  // SPEC: steps + polish + squarings
            if (tid == 0) {  // SPEC sign rule
                int f = -1, nnz = 0;
                for (int j = 0; j < E; j++)
                    if (x[j] != 0.0) {
                        nnz++;
                        if (f < 0) f = j;
                    }
                const bool neg = nnz == 1 ? x[f] < 0.0 : x[f] > 0.0;
                scal[8] = neg ? 1.0 : 0.0;
            }
            __syncthreads();
            if (scal[8] != 0.0)
                for (int j = tid; j < E; j += MT) x[j] = -x[j];
        }
        __syncthreads();
        if (tid == 0) scal[9] = sqrt(mpw([&](int j) { return x[j] * x[j]; }, E));
        __syncthreads();
        for (int j = tid; j < E; j += MT) loading[j] = x[j] / scal[9];
        __syncthreads();
        MSTAMP(7);
        if (alg == PCX_ALG_PCA) {
            for (int i = tid; i < N; i += MT) {  // scores (:337)
                double acc = 0.0;
                for (int j = 0; j < E; j++) acc = fma(F[i * E + j] - mu[j], loading[j], acc);
                s[i] = acc;
            }
        } else if (flags & PCX_FLAG_SVD_FAIL) {  // the reference's second svd raises (:375, :431)
            for (int i = tid; i < N; i += MT) s[i] = __builtin_nan("");
        } else {
            comps = component_scores(a, C, M, Tm, ES, F, mu, s, sh, scal);
        }
    } else if (alg == PCX_ALG_COKURTOSIS) {
        for (int i = tid; i < N; i += MT) s[i] = a.aux_scores[b * N + i];
    }
    __syncthreads();
    MSTAMP(8);
    if (alg != PCX_ALG_ABSOLUTE) {
        // --- a8/a9: nonconformity_rank (:487-500), tie -> nonconformity (:475-485)
        double* set1 = VNp(VN_SET1);
        double* set2 = VNp(VN_SET2);
        double* n1 = VNp(VN_NW1);
        double* n2 = VNp(VN_NW2);
        if (tid == 0) {  // NaN propagates like np.min / np.max
            double mn = s[0], mx = s[0];
            for (int i = 1; i < N; i++) {
                if (__builtin_isnan(s[i]) || s[i] < mn) mn = __builtin_isnan(mn) ? mn : s[i];
                if (__builtin_isnan(s[i]) || s[i] > mx) mx = __builtin_isnan(mx) ? mx : s[i];
            }
            scal[10] = mn;
            scal[11] = mx;
        }
        __syncthreads();
        for (int i = tid; i < N; i += MT) {
            set1[i] = s[i] + fabs(scal[10]);
            set2[i] = s[i] - scal[11];
        }
        __syncthreads();
        if (tid == 0) {  // normalize (:244-249)
            double S1 = mpw([&](int i) { return fabs(set1[i]); }, N);
            scal[12] = S1;
            scal[13] = S1 == 0 ? mpw([&](int i) { return fabs(set1[i]) + 1.0; }, N) : S1;
            double S2 = mpw([&](int i) { return fabs(set2[i]); }, N);
            scal[14] = S2;
            scal[15] = S2 == 0 ? mpw([&](int i) { return fabs(set2[i]) + 1.0; }, N) : S2;
        }
        __syncthreads();
        for (int i = tid; i < N; i += MT) {
            n1[i] = scal[12] == 0 ? (fabs(set1[i]) + 1.0) / scal[13] : fabs(set1[i]) / scal[13];
            n2[i] = scal[14] == 0 ? (fabs(set2[i]) + 1.0) / scal[15] : fabs(set2[i]) / scal[15];
        }
        __syncthreads();
        double* old = VEp(VE_OLD);
        for (int j = tid; j < E; j += MT) {
            const double a1 = mob_vecmat([&](int i) { return n1[i]; }, [&](int i) { return F[i * E + j]; }, N, E, j);
            const double a2 = mob_vecmat([&](int i) { return n2[i]; }, [&](int i) { return F[i * E + j]; }, N, E, j);
            VEp(VE_D1)[j] = a1;
            VEp(VE_D2)[j] = a2;
            const double t = 0.01 * old[j];
            VEp(VE_NEW1)[j] = a1 + t;
            VEp(VE_NEW2)[j] = a2 + t;
        }
        __syncthreads();
        double ref = 0.0;
        if (alg == PCX_ALG_PCA) {
            double* nw1 = VEp(VE_NEW1);
            double* nw2 = VEp(VE_NEW2);
            for (int j = tid; j < E; j += MT) {
                int lt0 = 0, eq0 = 0, lt1 = 0, eq1 = 0, lt2 = 0, eq2 = 0;
                for (int k = 0; k < E; k++) {
                    lt0 += old[k] < old[j];
                    eq0 += old[k] == old[j];
                    lt1 += nw1[k] < nw1[j];
                    eq1 += nw1[k] == nw1[j];
                    lt2 += nw2[k] < nw2[j];
                    eq2 += nw2[k] == nw2[j];
                }
                const double r0 = (double)lt0 + (double)(eq0 + 1) * 0.5;
                const double r1 = (double)lt1 + (double)(eq1 + 1) * 0.5;
                const double r2 = (double)lt2 + (double)(eq2 + 1) * 0.5;
                VEp(VE_E1)[j] = fabs(r1 - r0);
                VEp(VE_E2)[j] = fabs(r2 - r0);
            }
            __syncthreads();
            if (tid == 0)
                scal[2] = mpw([&](int j) { return VEp(VE_E1)[j]; }, E) - mpw([&](int j) { return VEp(VE_E2)[j]; }, E);
            __syncthreads();
            ref = scal[2];
            __syncthreads();
        }
        int pick1;
        if (ref == 0) {
            if (tid == 0) {
                const double* d1 = VEp(VE_D1);
                const double* d2 = VEp(VE_D2);
                const double q1 = mpw([&](int j) { const double v = d1[j] - old[j]; return v * v; }, E);
                const double q2 = mpw([&](int j) { const double v = d2[j] - old[j]; return v * v; }, E);
                scal[3] = (q1 - q2) <= 0 ? 1.0 : 0.0;
            }
            __syncthreads();
            pick1 = scal[3] != 0.0;
            branch = pick1 ? PCX_BRANCH_TIE_SET1 : PCX_BRANCH_TIE_SET2;
        } else {
            pick1 = ref < 0;
            branch = pick1 ? PCX_BRANCH_SET1 : PCX_BRANCH_SET2;
        }
        for (int i = tid; i < N; i += MT) nc[i] = pick1 ? set1[i] : set2[i];
    }
    __syncthreads();
    MSTAMP(9);
    // --- a10: reputation update (:460-472)
    double* thisr = VNp(VN_THIS);
    double* smooth = VNp(VN_SMOOTH);
    if (tid == 0) scal[4] = mpw([&](int i) { return rep[i]; }, N) / (double)N;
    __syncthreads();
    for (int i = tid; i < N; i += MT) nc[i] = nc[i] * (rep[i] / scal[4]);  // u (nc no longer needed)
    __syncthreads();
    if (tid == 0) {
        const double S = mpw([&](int i) { return fabs(nc[i]); }, N);
        scal[5] = S;
        scal[6] = S == 0 ? mpw([&](int i) { return fabs(nc[i]) + 1.0; }, N) : S;
    }
    __syncthreads();
    for (int i = tid; i < N; i += MT) {
        const double t = scal[5] == 0 ? (fabs(nc[i]) + 1.0) / scal[6] : fabs(nc[i]) / scal[6];
        thisr[i] = t;
        smooth[i] = a.alpha * t + (1.0 - a.alpha) * rep[i];
    }
    __syncthreads();
    MSTAMP(10);
    // --- a12/a13: outcomes (:510-538)
    double* raw = VEp(VE_RAW);
    double* adj = VEp(VE_ADJ);
    double* fin = VEp(VE_FIN);
    for (int j = tid; j < E; j += MT) {
        raw[j] = mob_vecmat([&](int i) { return smooth[i]; }, [&](int i) { return F[i * E + j]; }, N, E, j);
        if (!scaled(j)) {
            adj[j] = mcatch(raw[j], a.catch_tol);
            fin[j] = adj[j];
        }
    }
    __syncthreads();
    MSTAMP(11);
    for (int j = 0; j < E; j++) {
        if (!scaled(j)) continue;
        for (int i = tid; i < N; i += MT) XA[i] = F[i * E + j];
        __syncthreads();
        const double r = mwmedian(XA, smooth, N, VNp(VN_XS), VNp(VN_WS), sh);
        if (tid == 0) {
            raw[j] = r;
            adj[j] = r;
            double f = r * (a.hi[bo + j] - a.lo[bo + j]);
            f = f + a.lo[bo + j];
            fin[j] = f;
        }
        __syncthreads();
    }
    MSTAMP(12);
    // --- a14: certainty (:540-546): sum of smooth over the matching rows (pairwise), per event
    double* cert = VEp(VE_CERT);
    for (int j = 0; j < E; j++) {  // the matching rows' weights in row order (block compaction)
        const double aj = adj[j];
        const int m = bcompact([&](int i) { return F[i * E + j] == aj; }, [&](int i) { return smooth[i]; }, N, XA, wcnt);
        if (tid == 0)
            cert[j] = m ? mpw([&](int q) { return XA[q]; }, m) : (alg == PCX_ALG_PCA ? __builtin_nan("") : 0.0);
        __syncthreads();
    }
    MSTAMP(13);
    double* reward = VEp(VE_REWARD);
    double* pc = VEp(VE_PC);
    double* relc = VEp(VE_RELC);
    if (tid == 0) {
        const double S = mpw([&](int j) { return fabs(cert[j]); }, E);
        const double Sp = S == 0 ? mpw([&](int j) { return fabs(cert[j]) + 1.0; }, E) : S;
        for (int j = 0; j < E; j++) reward[j] = S == 0 ? (fabs(cert[j]) + 1.0) / Sp : fabs(cert[j]) / Sp;
        scal[7] = mpw([&](int j) { return cert[j]; }, E) / (double)E;  // avg certainty
    }
    // --- a15: participation and bonuses (:549-581)
    for (int j = tid; j < E; j += MT) {
        pc[j] = 1.0 - mdot2([&](int i) { return smooth[i]; }, [&](int i) { return fl[i * E + j] ? 1.0 : 0.0; }, N);
        int nz = 0;
        for (int i = 0; i < N; i++) nz += (fl[i * E + j] & 2) ? 1 : 0;
        if (a.nas_filled) a.nas_filled[b * E + j] = (double)nz;
    }
    __syncthreads();
    MSTAMP(14);
    double* pr = VNp(VN_SET1);  // reuse
    double* narow = VNp(VN_SET2);
    double* rel = VNp(VN_NW1);
    double* a2v = VNp(VN_NW2);
    double* rmask = VNp(VN_XS);
    for (int i = tid; i < N; i += MT) {
        int nz = 0, nn = 0;
        for (int j = 0; j < E; j++) {
            nz += (fl[i * E + j] & 2) ? 1 : 0;
            nn += (fl[i * E + j] & 1) ? 1 : 0;
        }
        narow[i] = (double)nz;
        pr[i] = 1.0 - narow[i] / (double)E;
        rmask[i] = nn == E ? 1.0 : 0.0;  // Q15: a fully NaN row is masked
        a2v[i] = rmask[i] != 0.0 ? 0.0 : fabs(pr[i]);
    }
    __syncthreads();
    if (tid == 0) {
        scal[8] = 1.0 - mpw([&](int j) { return pc[j]; }, E) / (double)E;  // pna
        double S = mpw([&](int i) { return a2v[i]; }, N);
        const bool bump = S == 0;
        if (bump) S = mpw([&](int i) { return rmask[i] != 0.0 ? 0.0 : fabs(pr[i]) + 1.0; }, N);
        scal[9] = S;
        scal[10] = bump ? 1.0 : 0.0;
        const double P = mpw([&](int j) { return fabs(pc[j]); }, E);
        const double Pp = P == 0 ? mpw([&](int j) { return fabs(pc[j]) + 1.0; }, E) : P;
        for (int j = 0; j < E; j++) relc[j] = P == 0 ? (fabs(pc[j]) + 1.0) / Pp : fabs(pc[j]) / Pp;
    }
    __syncthreads();
    const double pna = scal[8];
    for (int i = tid; i < N; i += MT) {
        const bool masked = rmask[i] != 0.0;
        const double ai = masked ? 0.0 : fabs(pr[i]) + (scal[10] != 0.0 ? 1.0 : 0.0);
        rel[i] = masked ? fabs(pr[i]) : ai / scal[9];
        const int64_t o = b * N + i;
        if (a.old_rep) a.old_rep[o] = rep[i];
        if (a.this_rep) a.this_rep[o] = thisr[i];
        if (a.smooth_rep) a.smooth_rep[o] = smooth[i];
        if (a.scores) a.scores[o] = s[i];
        if (a.na_row) a.na_row[o] = narow[i];
        if (a.participation_rows) a.participation_rows[o] = pr[i];
        if (a.relative_part) a.relative_part[o] = rel[i];
        if (a.reporter_bonus) a.reporter_bonus[o] = masked ? rel[i] : rel[i] * pna + smooth[i] * (1.0 - pna);
    }
    for (int j = tid; j < E; j += MT) {
        const int64_t o = b * E + j;
        if (a.adj_first_loadings) a.adj_first_loadings[o] = loading[j];
        if (a.outcomes_raw) a.outcomes_raw[o] = raw[j];
        if (a.outcomes_adjusted) a.outcomes_adjusted[o] = adj[j];
        if (a.outcomes_final) a.outcomes_final[o] = fin[j];
        if (a.certainty) a.certainty[o] = cert[j];
        if (a.consensus_reward) a.consensus_reward[o] = reward[j];
        if (a.participation_columns) a.participation_columns[o] = pc[j];
        if (a.author_bonus) a.author_bonus[o] = relc[j] * pna + reward[j] * (1.0 - pna);
    }
    MSTAMP(15);
    if (tid == 0) {
        if (a.participation) a.participation[b] = 1.0 - pna;
        if (a.avg_certainty) a.avg_certainty[b] = scal[7];
        if (a.branch) a.branch[b] = branch;
        if (a.flags) a.flags[b] = flags;
        if (a.pi_iters) a.pi_iters[b] = iters;
        if (a.components) a.components[b] = comps;
    }
}

}  // namespace

bool medium_fits(const BatchArgs& a) {
    return a.N >= 1 && a.N <= MN && a.E >= 1 && a.E <= MEV &&
           a.algorithm >= PCX_ALG_PCA && a.algorithm <= PCX_ALG_COKURTOSIS;
}

size_t medium_lds_bytes(int N, int E) {
    const size_t ES = (size_t)E + 1;
    return (2 * E * ES + (size_t)VN_COUNT * N + (size_t)VE_COUNT * E) * sizeof(double) + (size_t)N * E + 16;
}

// rounds in chunks whose scratch (filled matrix unless the caller keeps it, covariance) fits
// `scratch_bytes`; returns the chunk size used through *chunk
int64_t medium_chunk(const BatchArgs& a, size_t scratch_bytes) {
    const size_t per = ((a.filled ? 0 : (size_t)a.N * a.E) + (size_t)a.E * a.E) * sizeof(double);
    int64_t c = (int64_t)(scratch_bytes / (per ? per : 1));
    return c < 1 ? 1 : (c > a.B ? a.B : c);
}

hipError_t launch_medium(const BatchArgs& a, int64_t b0, int64_t nb, double* Fscr, double* Cscr, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    const size_t lds = medium_lds_bytes(a.N, a.E);
    // (dynamic LDS above 64 KB needs no attribute on gfx950: the launch checks it against 160 KB)
    (void)hipGetLastError();  // report launch errors only
    hipLaunchKernelGGL(medium_round_kernel, dim3((unsigned)nb), dim3(MT), lds, st, a, b0, Fscr, Cscr);
    return hipGetLastError();
}

}  // namespace pcx
