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
// Work split: one thread per event column, per reporter row, per matrix entry or per 4 x 4
// tile, as each step allows; one wave per weighted median (bitonic (x, w, index) order, the
// sequential total and walk on every lane alike) and per certainty; the power steps on one
// wave; the reference's sequential sums in their order, loads issued ahead.  LDS holds a work
// region (power-iteration matrices / median scratch / staged covariance rows / np.dot block
// partials), the per-element NA flags and the row / event vectors; the filled matrix and the
// covariance live in a per-round global scratch (L2-resident).  DESIGN.md 5.3.
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
              M_PI_POLISH = 2;
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

// the same tree64 on a register value per lane (0 beyond n); valid on lane 0
__device__ double wtree64v(double v) {
    for (int s = 1; s <= 8; s <<= 1) v = v + __shfl_xor(v, s, 64);
    const double t16 = __shfl(v, 16, 64), t32 = __shfl(v, 32, 64), t48 = __shfl(v, 48, 64);
    return (v + t16) + (t32 + t48);
}

// SPEC dot2 (compensated dot, index order)
template <class A, class B>
__device__ double mdot2(A a, B b, int n) {
    double s = 0.0, c = 0.0;
    auto step = [&](double x, double y) {
        const double p = x * y;
        const double pe = fma(x, y, -p);
        const double t = s + p;
        const double z = t - s;
        const double se = (s - (t - z)) + (p - z);
        s = t;
        c = c + (pe + se);
    };
    int i = 0;
    for (; i + 8 <= n; i += 8) {  // in index order, loads eight ahead
        double xa[8], ya[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            xa[q] = a(i + q);
            ya[q] = b(i + q);
        }
#pragma unroll
        for (int q = 0; q < 8; q++) step(xa[q], ya[q]);
    }
    for (; i < n; i++) step(a(i), b(i));
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
        for (; n + 8 <= N; n += 8) {  // two blocks of four rows, loads ahead of the adds
            double f[8], w[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                f[q] = F(n + q);
                w[q] = v(n + q);
            }
            double t0 = f[1] * w[1];
            t0 = fma(f[0], w[0], t0);
            t0 = fma(f[2], w[2], t0);
            t0 = fma(f[3], w[3], t0);
            double t1 = f[5] * w[5];
            t1 = fma(f[4], w[4], t1);
            t1 = fma(f[6], w[6], t1);
            t1 = fma(f[7], w[7], t1);
            y = y + t0;
            y = y + t1;
        }
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

// out[j] = np.dot(v, F)[j] for every column (block call, all threads): OpenBLAS's four-row
// block partials of the columns j < E & ~3 in parallel into tb ((N / 4) x (E & ~3) doubles),
// then each column's sequential sum of its partials and the row tail; the other columns (and
// E == 1) by mob_vecmat on their thread over a copy staged in LDS after the partials
// ((E - E & ~3) x N doubles).  The caller syncs before reading out.
template <class V>
__device__ void bvecmat(V v, const double* F, int N, int E, double* out, double* tb);

__device__ __forceinline__ double mcatch(double x, double tol) {
    if (x < 1.5 - tol) return 1.0;
    if (x > 1.5 + tol) return 2.0;
    return 1.5;
}

template <class V>
__device__ void bvecmat(V v, const double* F, int N, int E, double* out, double* tb) {
    const int E4 = E == 1 ? 0 : (E & ~3), nb = N >> 2, ni = nb * E4;
    for (int i0 = threadIdx.x; i0 < ni; i0 += 4 * MT) {  // four blocks' loads per round trip
        double f[4][4], w[4][4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int idx = i0 + u * MT;
            const int j = idx % E4, n = 4 * (idx / E4);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                f[u][r] = idx < ni ? F[(n + r) * E + j] : 0.0;
                w[u][r] = idx < ni ? v(n + r) : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int idx = i0 + u * MT;
            double t = f[u][1] * w[u][1];
            t = fma(f[u][0], w[u][0], t);
            t = fma(f[u][2], w[u][2], t);
            t = fma(f[u][3], w[u][3], t);
            if (idx < ni) tb[idx] = t;
        }
    }
    double* tl = tb + ni;  // the columns past E & ~3 staged from F (their chains read LDS)
    const int nt = (E - E4) * N;
    for (int idx = threadIdx.x; idx < nt; idx += MT) tl[idx] = F[(idx % N) * E + E4 + idx / N];
    __syncthreads();
    for (int j = threadIdx.x; j < E; j += MT) {
        if (j >= E4) {
            const double* col = tl + (j - E4) * N;
            out[j] = mob_vecmat(v, [&](int i) { return col[i]; }, N, E, j);
            continue;
        }
        double y = mseq([&](int b) { return tb[b * E4 + j]; }, nb);  // y = y + t, block order
        int n = 4 * nb;
        if (n + 2 <= N) {
            double t = F[(n + 1) * E + j] * v(n + 1);
            t = fma(F[n * E + j], v(n), t);
            y = y + t;
            n += 2;
        }
        if (n < N) y = y + F[n * E + j] * v(n);
        out[j] = y;
    }
}

// block reductions (max of doubles / first index)
// (max-norms of non-negative values: exact in any order)
__device__ double bmax(double v, double* sh) {
    for (int s = 1; s < 64; s <<= 1) v = fmax(v, __shfl_xor(v, s, 64));
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = sh[0];
    for (int w = 1; w < MT / 64; w++) r = fmax(r, sh[w]);
    __syncthreads();
    return r;
}

// one wave's LDS writes visible to its other lanes (LDS operations of a wave execute in issue
// order: a compiler-ordering wave barrier, no lgkmcnt drain)
__device__ __forceinline__ void mwsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// broadcast from a wave-uniform lane (v_readlane into SGPRs)
__device__ __forceinline__ double mbcast(double v, int src) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// sequential sum g(0) + g(1) + ... in index order (Python's builtin sum), the loads issued
// eight at a time ahead of the dependent adds
template <class G>
__device__ double mseq(G g, int n) {
    double s = 0.0;
    int i = 0;
    for (; i + 8 <= n; i += 8) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; q++) v[q] = g(i + q);
#pragma unroll
        for (int q = 0; q < 8; q++) s += v[q];
    }
    for (; i < n; i++) s += g(i);
    return s;
}

// weightedstats.weighted_median (SPEC wmedian) of n <= 256 (x, w) pairs in LDS on ONE wave:
// lane 0's sequential total and walk (loads batched by eight), the stable (x, w) order by a
// bitonic network over the lanes in LDS (the SPEC's rank placement when a NaN is present); sb is
// this wave's sort scratch of PN doubles x, PN doubles w and PN ints (PN = pow2 >= n); the result
// on every lane of the wave
__device__ double wv_wmedian(const double* x, const double* w, int n, double* sb, int PN,
                             long long* prof = nullptr) {
    const int lane = threadIdx.x & 63;
    double* xs = sb;
    double* ws = sb + PN;
    long long t0 = prof ? (long long)__builtin_amdgcn_s_memtime() : 0;
    const double W = mseq([&](int i) { return w[i]; }, n);  // every lane alike (broadcast loads)
    const double mid = 0.5 * W;
    bool dom = false, pos = false, nan_ = false;
    for (int i = lane; i < n; i += 64) {
        dom |= w[i] > mid;
        pos |= w[i] > 0;
        nan_ |= __builtin_isnan(x[i]) || __builtin_isnan(w[i]);
    }
    const bool anydom = __ballot(dom) != 0, anypos = __ballot(pos) != 0;
    double r = __builtin_nan("");
    if (anydom) {
        if (lane == 0) {
            double m = w[0];
            for (int i = 1; i < n; i++)
                if (w[i] > m) m = w[i];
            for (int i = 0; i < n; i++)
                if (w[i] == m) {
                    r = x[i];
                    break;
                }
        }
        return mbcast(r, 0);
    }
    if (!anypos) return r;
    if (prof) {
        const long long t = (long long)__builtin_amdgcn_s_memtime();
        prof[0] += t - t0;
        t0 = t;
    }
    if (__ballot(nan_) == 0) {
        // the stable (x, w) order is the ascending order of (x, w, index) (x, w compared with
        // < and ==): a bitonic network over P = pow2 >= n slots in LDS, padding slots last
        int* id = (int*)(sb + 2 * PN);
        int P = 2;
        while (P < n) P <<= 1;
        for (int i = lane; i < P; i += 64) {
            const bool v = i < n;
            xs[i] = v ? x[i] : 0.0;
            ws[i] = v ? w[i] : 0.0;
            id[i] = v ? i : -1;
        }
        mwsync();
        for (int k = 2; k <= P; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int t = lane; t < (P >> 1); t += 64) {
                    const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1)), l = i + j;
                    const int ia = id[i], il = id[l];
                    const double xa = xs[i], wa = ws[i], xl = xs[l], wl = ws[l];
                    bool gt;  // (x, w, id) at i after the one at l; padding after everything
                    if (ia < 0 || il < 0)
                        gt = ia < 0 && il >= 0;
                    else
                        gt = (xl < xa) || (xl == xa && (wl < wa || (wl == wa && il < ia)));
                    if (gt == ((i & k) == 0)) {
                        xs[i] = xl;
                        xs[l] = xa;
                        ws[i] = wl;
                        ws[l] = wa;
                        id[i] = il;
                        id[l] = ia;
                    }
                }
                mwsync();
            }
    } else {
        // stable rank by (x, w) as the SPEC places it: this lane's elements i = lane + 64 q in
        // registers, the compared elements m read eight at a time (LDS broadcasts)
        const int nq = (n + 63) >> 6;
        double xi[4], wi[4];
        int rk[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int i = lane + 64 * q;
            xi[q] = i < n ? x[i] : 0.0;
            wi[q] = i < n ? w[i] : 0.0;
            rk[q] = 0;
        }
        auto cmp = [&](double xm, double wm, int m) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (q >= nq) break;  // wave-uniform
                const bool lt = (xm < xi[q]) || (xm == xi[q] && wm < wi[q]);
                const bool eq = (xm == xi[q]) && (wm == wi[q]);
                rk[q] += (lt || (eq && m < lane + 64 * q)) ? 1 : 0;
            }
        };
        int m0 = 0;
        for (; m0 + 8 <= n; m0 += 8) {
            double xm[8], wm[8];
#pragma unroll
            for (int t = 0; t < 8; t++) {
                xm[t] = x[m0 + t];
                wm[t] = w[m0 + t];
            }
#pragma unroll
            for (int t = 0; t < 8; t++) cmp(xm[t], wm[t], m0 + t);
        }
        for (; m0 < n; m0++) cmp(x[m0], w[m0], m0);
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (lane + 64 * q < n) {
                xs[rk[q]] = xi[q];
                ws[rk[q]] = wi[q];
            }
    }
    mwsync();
    if (prof) {
        const long long t = (long long)__builtin_amdgcn_s_memtime();
        prof[1] += t - t0;
        t0 = t;
    }
    {
        // the walk `while cum <= mid: cum += ws[k]; k += 1` on every lane alike (no divergence):
        // branch-free steps, eight loads ahead, leaving at the first batch past the crossing
        double cum = 0.0;
        int k = 0;
        bool stop = !(cum <= mid);
        for (int i = 0; i < n && !stop; i += 8) {
            const int lim = n - i < 8 ? n - i : 8;
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; q++) v[q] = q < lim ? ws[i + q] : 0.0;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const bool go = !stop && q < lim;
                const double c2 = cum + v[q];
                cum = go ? c2 : cum;
                k += go ? 1 : 0;
                stop = stop || (go && !(cum <= mid));
            }
        }
        const bool fail = !stop;  // ran past the end with cum <= mid
        if (!fail) {
            const double before = cum - ws[k - 1];
            if (fabs(before - mid) < M_DBL_EPS) {
                if (k >= 2) r = (xs[k - 2] + xs[k - 1]) / 2.0;
                else if (n == 1) r = xs[0] / 1.0;
            } else {
                r = xs[k - 1];
            }
        }
    }
    r = mbcast(r, 0);
    mwsync();  // xs / ws free for the wave's next use
    if (prof) prof[2] += (long long)__builtin_amdgcn_s_memtime() - t0;
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

// N-vectors (each N doubles)
enum { VN_REP = 0, VN_TOK, VN_S, VN_SET1, VN_SET2, VN_NW1, VN_NW2, VN_U, VN_THIS, VN_SMOOTH, VN_XS, VN_COUNT };
// E-vectors (each E doubles)
enum { VE_MU = 0, VE_OLD, VE_LD, VE_X, VE_Y, VE_SQ, VE_D1, VE_D2, VE_NEW1, VE_NEW2, VE_R0, VE_R1, VE_R2, VE_E1, VE_E2,
       VE_RAW, VE_ADJ, VE_FIN, VE_CERT, VE_REWARD, VE_PC, VE_RELC, VE_COUNT };
// doubles of the work region: M (E x (E+1); and Tm for the Jacobi algorithms), or per wave two N-vectors (median
// operands) and the sort scratch (PN doubles x, PN doubles w, PN ints; PN = pow2 >= N), or the
// vector-matrix block partials, or the covariance's staged rows
__host__ __device__ __forceinline__ int medium_pow2(int N) {
    int p = 2;
    while (p < N) p <<= 1;
    return p;
}
__host__ __device__ __forceinline__ int medium_wave_stride(int N) {
    const int pn = medium_pow2(N);
    return 2 * N + 2 * pn + pn / 2;
}
__host__ __device__ __forceinline__ int medium_work(int N, int E, int alg) {
    const bool jac = alg == PCX_ALG_BIG_FIVE || alg == PCX_ALG_FIXED_VARIANCE;  // Tm: the eigenvectors
    const int E4 = E == 1 ? 0 : (E & ~3);
    const int mt = (jac ? 2 : 1) * E * (E + 1), wq = (MT / 64) * medium_wave_stride(N),
              vb = (N >> 2) * E4 + (E - E4) * N;
    const int m = mt > wq ? mt : wq;
    return m > vb ? m : vb;  // and bvecmat's block partials
}

// diagnostic phase stamps (PCX_STAMPS=1): shader-clock reads at phase boundaries
#define MSTAMP(k)                                                                 \
    do {                                                                          \
        if (a.stamps) {                                                           \
            const long long t_ = (long long)__builtin_amdgcn_s_memtime();         \
            if (threadIdx.x == 0) a.stamps[b * 32 + (k)] = t_;                    \
        }                                                                         \
    } while (0)

#ifndef PCX_MEDIUM_WAVES  // waves per SIMD the VGPR budget is sized for (a build parameter for A/B runs)
#define PCX_MEDIUM_WAVES 3
#endif
__global__ void __launch_bounds__(MT, PCX_MEDIUM_WAVES) medium_round_kernel(BatchArgs a, int64_t b0, double* Fscr, double* Cscr) {
    extern __shared__ __attribute__((aligned(16))) double mlds[];
    __shared__ double sh[MT];
    __shared__ double scal[16];
    const int64_t b = b0 + blockIdx.x;  // round; scratch slot blockIdx.x
    const int N = a.N, E = a.E, ES = E + 1;
    const int tid = threadIdx.x;
    double* M = mlds;
    double* Tm = M + E * ES;
    // work region: M and Tm in the power iteration / Jacobi, per wave the median operands and
    // sort scratch in the interpolation, the outcomes and the certainty
    double* vN = mlds + medium_work(N, E, a.algorithm);
    double* vE = vN + VN_COUNT * N;
    // NA flags [N][E], two bits per element (bit 0 NaN, bit 1 zero), sixteen to a word
    uint32_t* flw = (uint32_t*)(vE + VE_COUNT * E);
    auto FL = [&](int e) -> uint32_t { return (flw[e >> 4] >> ((e & 15) << 1)) & 3u; };
    auto VNp = [&](int k) { return vN + k * N; };
    auto VEp = [&](int k) { return vE + k * E; };
    double* rep = VNp(VN_REP);
    double* tok = VNp(VN_TOK);
    const double* Rin = a.reports + b * N * E;
    double* F = a.filled ? a.filled + b * N * E : Fscr + (int64_t)blockIdx.x * N * E;
    double* C = Cscr + (int64_t)blockIdx.x * E * E;
    const int64_t bo = a.bounds_shared ? 0 : b * E;
    const bool has_bounds = a.scaled != nullptr;
    const int alg = a.algorithm;
    const int lane = tid & 63, wv = tid >> 6;
    const int PN = medium_pow2(N);
    double* wb = mlds + wv * medium_wave_stride(N);  // this wave's median operands and sort scratch
    __shared__ unsigned long long scmask_s;
    __shared__ int scl[MEV], nscl_s;
    MSTAMP(0);
    if (tid < 64) {  // the scaled events: a mask and their list in index order
        const bool p = has_bounds && tid < E && a.scaled[bo + tid] != 0;
        const unsigned long long bal = __ballot(p);
        if (p) scl[__popcll(bal & ((1ull << tid) - 1ull))] = tid;
        if (tid == 0) {
            scmask_s = bal;
            nscl_s = __popcll(bal);
        }
    }
    auto scaled = [&](int j) { return ((scmask_s >> j) & 1ull) != 0; };
    long long mprof[3] = {0, 0, 0};  // diagnostic (PCX_STAMPS): median total+dom / rank / walk cycles

    for (int w = tid; w < (N * E + 15) >> 4; w += MT) flw[w] = 0u;  // (ordered by the barrier below)
    // --- a1: reputation (:138-146)
    if (tid == 0) scal[0] = a.reputation ? mpw([&](int i) { return a.reputation[b * N + i]; }, N) : 0.0;
    __syncthreads();
    for (int i = tid; i < N; i += MT) {
        const double r = a.reputation ? a.reputation[b * N + i] / scal[0] : 1.0 / (double)N;
        rep[i] = r;
        tok[i] = trunc(r * 1e6);
    }
    __syncthreads();
    if (tid == 0) scal[1] = mseq([&](int i) { return tok[i]; }, N) - 1.0;  // denom
    // --- a2: rescale (:266-269), NA (:278)
    for (int e0 = tid; e0 < N * E; e0 += 8 * MT) {  // eight reports' loads ahead of the stores
        double xv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int e = e0 + u * MT;
            xv[u] = e < N * E ? Rin[e] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int e = e0 + u * MT;
            if (e >= N * E) break;
            const int j = e % E;
            double x = xv[u];
            if (scaled(j)) {
                x = (x - a.lo[bo + j]) / (a.hi[bo + j] - a.lo[bo + j]);
                if (a.int_dtype) x = trunc(x);
            }
            F[e] = x;
            const uint32_t bits = (__builtin_isnan(x) ? 1u : 0u) | (x == 0.0 ? 2u : 0u);
            if (bits) atomicOr(&flw[e >> 4], bits << ((e & 15) << 1));
            if (a.original) a.original[b * N * E + e] = x;
        }
    }
    __syncthreads();
    MSTAMP(1);
    // --- a3: interpolate (:284-313): binary columns one thread each; scaled columns one at a
    // time with the whole block (weighted median)
    {
        // one thread per binary column (E <= 64): the present total from the LDS flags, then the
        // weighted mean over the present rows in row order, the filled matrix staged through the
        // work region in row chunks (one round trip per chunk, not per eight rows)
        const int j = tid;
        const bool act = j < E && !scaled(j);
        int nmiss = 0;
        double tot = 0.0;
        if (act) {
            int i = 0;
            for (; i + 8 <= N; i += 8) {
                uint8_t f[8];
                double r[8];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    f[q] = FL((i + q) * E + j);
                    r[q] = rep[i + q];
                }
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    nmiss += f[q] ? 1 : 0;
                    if (!f[q]) tot += r[q];
                }
            }
            for (; i < N; i++) {
                const bool m = FL(i * E + j) != 0;
                nmiss += m ? 1 : 0;
                if (!m) tot += rep[i];
            }
        }
        const bool need = act && nmiss > 0;
        double g = 0.0;
        if (__syncthreads_or(need)) {
            int CR = medium_work(N, E, a.algorithm) / E;
            CR = CR > 64 ? 64 : CR;
            double* st = mlds;
            for (int c0 = 0; c0 < N; c0 += CR) {
                const int cr = N - c0 < CR ? N - c0 : CR;
                for (int idx = tid; idx < cr * E; idx += MT) st[idx] = F[c0 * E + idx];
                __syncthreads();
                if (need) {
                    int r = 0;
                    for (; r + 8 <= cr; r += 8) {
                        uint8_t f[8];
                        double w8[8], x[8];
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            f[q] = FL((c0 + r + q) * E + j);
                            w8[q] = rep[c0 + r + q];
                            x[q] = st[(r + q) * E + j];
                        }
#pragma unroll
                        for (int q = 0; q < 8; q++)
                            if (!f[q]) g += (w8[q] / tot) * x[q];
                    }
                    for (; r < cr; r++)
                        if (!FL((c0 + r) * E + j)) g += (rep[c0 + r] / tot) * st[r * E + j];
                }
                __syncthreads();
            }
        }
        if (need) {
            g = mcatch(g, a.catch_tol);
            if (a.int_dtype) g = trunc(g);
            for (int i = 0; i < N; i++)
                if (FL(i * E + j)) F[i * E + j] = g;
        }
    }
    MSTAMP(2);
    const int nscl = nscl_s;
    for (int c = wv; c < nscl; c += MT / 64) {  // one wave per scaled column
        const int j = scl[c];
        // present values and their reputations in row order (wave compaction), then the
        // sequential present total on lane 0 and the weights rep / total
        int np_ = 0;
        for (int i0 = 0; i0 < N; i0 += 64) {
            const int i = i0 + lane;
            const bool p = i < N && FL(i * E + j) == 0;
            const unsigned long long bal = __ballot(p);
            if (p) {
                const int o = np_ + __popcll(bal & ((1ull << lane) - 1ull));
                wb[o] = F[i * E + j];
                wb[N + o] = rep[i];
            }
            np_ += __popcll(bal);
        }
        mwsync();
        double tot = 0.0;
        if (lane == 0) tot = mseq([&](int q) { return wb[N + q]; }, np_);
        tot = mbcast(tot, 0);
        for (int q = lane; q < np_; q += 64) wb[N + q] = wb[N + q] / tot;
        mwsync();
        if (np_ < N) {  // wave-uniform
            double g = wv_wmedian(wb, wb + N, np_, wb + 2 * N, PN);
            if (a.int_dtype) g = trunc(g);
            for (int i = lane; i < N; i += 64)
                if (FL(i * E + j)) F[i * E + j] = g;
        }
        mwsync();
    }
    __syncthreads();
    MSTAMP(3);
    // old = np.dot(rep, F) (:489)
    bvecmat([&](int i) { return rep[i]; }, F, N, E, VEp(VE_OLD), mlds);
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
        // --- a6: covariance (:326), lower triangle mirrored: one 4 x 4 tile (J >= K) per thread,
        // rows staged through the work region in chunks (A = (F - mu) * tok, D = F - mu), each
        // entry's fma chain in row order
        {
            const double denom = scal[1];
            const int nT = (E + 3) >> 2, ntiles = nT * (nT + 1) / 2;
            int tJ = 0, tK = tid;
            while (tK > tJ) {
                tK -= tJ + 1;
                tJ++;
            }
            double acc[4][4];
#pragma unroll
            for (int p = 0; p < 4; p++)
#pragma unroll
                for (int q = 0; q < 4; q++) acc[p][q] = 0.0;
            int CR = medium_work(N, E, a.algorithm) / (2 * E);
            CR = CR > 32 ? 32 : CR;
            double* Al = mlds;
            double* Dl = mlds + CR * E;
            for (int c0 = 0; c0 < N; c0 += CR) {
                const int cr = N - c0 < CR ? N - c0 : CR;
                for (int idx = tid; idx < cr * E; idx += MT) {
                    const int i = c0 + idx / E, j = idx % E;
                    const double d = F[i * E + j] - mu[j];
                    Dl[idx] = d;
                    Al[idx] = d * tok[i];
                }
                __syncthreads();
                if (tid < ntiles)
                    for (int r = 0; r < cr; r++) {
                        double av[4], dv[4];
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int j = 4 * tJ + q, k = 4 * tK + q;
                            av[q] = j < E ? Al[r * E + j] : 0.0;
                            dv[q] = k < E ? Dl[r * E + k] : 0.0;
                        }
#pragma unroll
                        for (int p = 0; p < 4; p++)
#pragma unroll
                            for (int q = 0; q < 4; q++) acc[p][q] = fma(av[p], dv[q], acc[p][q]);
                    }
                __syncthreads();
            }
            if (tid < ntiles)
#pragma unroll
                for (int p = 0; p < 4; p++)
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int j = 4 * tJ + p, k = 4 * tK + q;
                        if (j < E && k <= j) {
                            const double c = acc[p][q] / denom;
                            C[j * E + k] = c;
                            C[k * E + j] = c;
                        }
                    }
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
            auto square = [&]() {  // M <- (M M) * 2^-ilogb(max|MM|): one 4 x 4 tile per thread
                // (E <= 64: at most 16 x 16 tiles, one per thread; the product stays in registers
                // across the block max, then overwrites M)
                double lm = 0.0;
                const int nT = (E + 3) >> 2, J = tid / nT, K = tid % nT;
                const bool own = tid < nT * nT;
                double acc[4][4];
#pragma unroll
                for (int p = 0; p < 4; p++)
#pragma unroll
                    for (int q = 0; q < 4; q++) acc[p][q] = 0.0;
                if (own) {
                    for (int l = 0; l < E; l++) {
                        double mr[4], mc[4];
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int j = 4 * J + q, k = 4 * K + q;
                            mr[q] = j < E ? M[j * ES + l] : 0.0;
                            mc[q] = k < E ? M[l * ES + k] : 0.0;
                        }
#pragma unroll
                        for (int p = 0; p < 4; p++)
#pragma unroll
                            for (int q = 0; q < 4; q++) acc[p][q] = fma(mr[p], mc[q], acc[p][q]);
                    }
#pragma unroll
                    for (int p = 0; p < 4; p++)
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const double v = fabs(acc[p][q]);
                            if (4 * J + p < E && 4 * K + q < E && v > lm) lm = v;
                        }
                }
                const double mx = bmax(lm, sh);  // (its barriers: every read of M is done)
                const bool pow2 = mx >= M_DBL_MIN && __builtin_isfinite(mx);
                const double sc = pow2 ? ldexp(1.0, -ilogb(mx)) : 1.0;
                if (own)
#pragma unroll
                    for (int p = 0; p < 4; p++)
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int j = 4 * J + p, k = 4 * K + q;
                            const double t = acc[p][q];
                            if (j < E && k < E) M[j * ES + k] = pow2 ? t * sc : (mx > 0.0 ? t / mx : t);
                        }
                __syncthreads();
            };
            int sqn = 0;
            for (; sqn < M_PI_PRESQUARE; sqn++) square();
            MSTAMP(28);
            // the power steps between squarings and the polish on wave 0: lane j = row j, x in
            // registers (x_k broadcast by readlane), tree64 norm and max-norm by shuffles
            __shared__ int pi_s[3];
            auto step = [&](const double* A, int lda, double xr) {  // (A x) / ||A x||
                const int row = lane < E ? lane : 0;
                double acc = 0.0;
                for (int k = 0; k < E; k++) acc = fma(A[row * lda + k], mbcast(xr, k), acc);
                const double yv = lane < E ? acc : 0.0;
                const double t = mbcast(sqrt(wtree64v(yv * yv)), 0);
                return yv / t;
            };
            int since = 0;
            for (;;) {
                if (wv == 0) {
                    double xr = lane < E ? x[lane] : 0.0;
                    int it = iters, sn = since, st = 0;
                    for (;;) {
                        const double yn = step(M, ES, xr);
                        double dl = lane < E ? fabs(yn - xr) : 0.0;
                        for (int s2 = 1; s2 < 64; s2 <<= 1) dl = fmax(dl, __shfl_xor(dl, s2, 64));
                        xr = yn;
                        it++;
                        sn++;
                        if (dl <= M_PI_TOL) {
                            st = 1;
                            break;
                        }
                        if (it >= M_PI_MAXIT) {
                            st = 2;
                            break;
                        }
                        if (sn >= M_PI_SQUARE_EVERY && sqn < M_PI_MAX_SQUARINGS) break;
                    }
                    if (lane < E) x[lane] = xr;
                    if (lane == 0) {
                        pi_s[0] = st;
                        pi_s[1] = it;
                        pi_s[2] = sn;
                    }
                }
                __syncthreads();
                const int st = pi_s[0];
                iters = pi_s[1];
                since = pi_s[2];
                __syncthreads();
                if (st == 1) break;
                if (st == 2) {
                    flags |= PCX_FLAG_PI_MAXIT;
                    break;
                }
                square();
                sqn++;
                since = 0;
            }
            MSTAMP(29);
            for (int e = tid; e < E * E; e += MT) M[(e / E) * ES + e % E] = C[e];  // C into LDS
            __syncthreads();
            if (wv == 0) {
                double xr = lane < E ? x[lane] : 0.0;
                for (int p = 0; p < M_PI_POLISH; p++) xr = step(M, ES, xr);
                if (lane < E) x[lane] = xr;
            }
            __syncthreads();
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
            auto upd = [&](double v) {
                if (__builtin_isnan(v) || v < mn) mn = __builtin_isnan(mn) ? mn : v;
                if (__builtin_isnan(v) || v > mx) mx = __builtin_isnan(mx) ? mx : v;
            };
            int i = 1;
            for (; i + 8 <= N; i += 8) {  // in row order, loads eight ahead
                double v[8];
#pragma unroll
                for (int q = 0; q < 8; q++) v[q] = s[i + q];
#pragma unroll
                for (int q = 0; q < 8; q++) upd(v[q]);
            }
            for (; i < N; i++) upd(s[i]);
            scal[10] = mn;
            scal[11] = mx;
        }
        __syncthreads();
        for (int i = tid; i < N; i += MT) {
            set1[i] = s[i] + fabs(scal[10]);
            set2[i] = s[i] - scal[11];
        }
        __syncthreads();
        if (tid == 0) {  // normalize (:244-249); the two sets on two waves
            double S1 = mpw([&](int i) { return fabs(set1[i]); }, N);
            scal[12] = S1;
            scal[13] = S1 == 0 ? mpw([&](int i) { return fabs(set1[i]) + 1.0; }, N) : S1;
        } else if (tid == 64) {
            double S2 = mpw([&](int i) { return fabs(set2[i]); }, N);
            scal[14] = S2;
            scal[15] = S2 == 0 ? mpw([&](int i) { return fabs(set2[i]) + 1.0; }, N) : S2;
        }
        __syncthreads();
        MSTAMP(24);
        for (int i = tid; i < N; i += MT) {
            n1[i] = scal[12] == 0 ? (fabs(set1[i]) + 1.0) / scal[13] : fabs(set1[i]) / scal[13];
            n2[i] = scal[14] == 0 ? (fabs(set2[i]) + 1.0) / scal[15] : fabs(set2[i]) / scal[15];
        }
        __syncthreads();
        double* old = VEp(VE_OLD);
        MSTAMP(25);
        bvecmat([&](int i) { return n1[i]; }, F, N, E, VEp(VE_D1), mlds);
        __syncthreads();
        bvecmat([&](int i) { return n2[i]; }, F, N, E, VEp(VE_D2), mlds);
        __syncthreads();
        for (int j = tid; j < E; j += MT) {
            const double a1 = VEp(VE_D1)[j], a2 = VEp(VE_D2)[j];
            const double t = 0.01 * old[j];
            VEp(VE_NEW1)[j] = a1 + t;
            VEp(VE_NEW2)[j] = a2 + t;
        }
        __syncthreads();
        MSTAMP(26);
        double ref = 0.0;
        if (alg == PCX_ALG_PCA) {
            double* nw1 = VEp(VE_NEW1);
            double* nw2 = VEp(VE_NEW2);
            for (int j = tid; j < E; j += MT) {
                int lt0 = 0, eq0 = 0, lt1 = 0, eq1 = 0, lt2 = 0, eq2 = 0;
                const double o = old[j], v1 = nw1[j], v2 = nw2[j];
                auto cnt = [&](double a0, double a1, double a2) {
                    lt0 += a0 < o;
                    eq0 += a0 == o;
                    lt1 += a1 < v1;
                    eq1 += a1 == v1;
                    lt2 += a2 < v2;
                    eq2 += a2 == v2;
                };
                int k = 0;
                for (; k + 8 <= E; k += 8) {  // broadcast loads eight ahead
                    double b0[8], b1[8], b2[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        b0[q] = old[k + q];
                        b1[q] = nw1[k + q];
                        b2[q] = nw2[k + q];
                    }
#pragma unroll
                    for (int q = 0; q < 8; q++) cnt(b0[q], b1[q], b2[q]);
                }
                for (; k < E; k++) cnt(old[k], nw1[k], nw2[k]);
                const double r0 = (double)lt0 + (double)(eq0 + 1) * 0.5;
                const double r1 = (double)lt1 + (double)(eq1 + 1) * 0.5;
                const double r2 = (double)lt2 + (double)(eq2 + 1) * 0.5;
                // rankdata propagates NaN (every rank NaN): a NaN value makes the rule's sums NaN
                const bool nan = __builtin_isnan(o) || __builtin_isnan(v1) || __builtin_isnan(v2);
                VEp(VE_E1)[j] = nan ? __builtin_nan("") : fabs(r1 - r0);
                VEp(VE_E2)[j] = nan ? __builtin_nan("") : fabs(r2 - r0);
            }
            __syncthreads();
            if (tid == 0)
                scal[2] = mpw([&](int j) { return VEp(VE_E1)[j]; }, E) - mpw([&](int j) { return VEp(VE_E2)[j]; }, E);
            __syncthreads();
            ref = scal[2];
            __syncthreads();
        }
        MSTAMP(27);
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
    bvecmat([&](int i) { return smooth[i]; }, F, N, E, raw, mlds);
    __syncthreads();
    for (int j = tid; j < E; j += MT) {
        if (!scaled(j)) {
            adj[j] = mcatch(raw[j], a.catch_tol);
            fin[j] = adj[j];
        }
    }
    __syncthreads();
    MSTAMP(11);
    for (int c = wv; c < nscl; c += MT / 64) {  // one wave per scaled column
        const int j = scl[c];
        for (int i = lane; i < N; i += 64) wb[i] = F[i * E + j];
        mwsync();
        const double r = wv_wmedian(wb, smooth, N, wb + 2 * N, PN, a.stamps ? mprof : nullptr);
        if (lane == 0) {
            raw[j] = r;
            adj[j] = r;
            double f = r * (a.hi[bo + j] - a.lo[bo + j]);
            f = f + a.lo[bo + j];
            fin[j] = f;
        }
    }
    __syncthreads();
    MSTAMP(12);
    // --- a14: certainty (:540-546): sum of smooth over the matching rows (pairwise), per event
    double* cert = VEp(VE_CERT);
    for (int j = wv; j < E; j += MT / 64) {  // one wave per event: the matching rows' weights in row order
        const double aj = adj[j];
        int m = 0;
        for (int i0 = 0; i0 < N; i0 += 64) {
            const int i = i0 + lane;
            const bool p = i < N && F[i * E + j] == aj;
            const unsigned long long bal = __ballot(p);
            if (p) wb[m + __popcll(bal & ((1ull << lane) - 1ull))] = smooth[i];
            m += __popcll(bal);
        }
        mwsync();
        if (lane == 0)
            cert[j] = m ? mpw([&](int q) { return wb[q]; }, m) : (alg == PCX_ALG_PCA ? __builtin_nan("") : 0.0);
        mwsync();
    }
    __syncthreads();
    MSTAMP(13);
    double* reward = VEp(VE_REWARD);
    double* pc = VEp(VE_PC);
    double* relc = VEp(VE_RELC);
    if (tid == 64) {  // (wave 1: wave 0 runs the participation columns meanwhile)
        const double S = mpw([&](int j) { return fabs(cert[j]); }, E);
        const double Sp = S == 0 ? mpw([&](int j) { return fabs(cert[j]) + 1.0; }, E) : S;
        for (int j = 0; j < E; j++) reward[j] = S == 0 ? (fabs(cert[j]) + 1.0) / Sp : fabs(cert[j]) / Sp;
        scal[7] = mpw([&](int j) { return cert[j]; }, E) / (double)E;  // avg certainty
    }
    // --- a15: participation and bonuses (:549-581)
    for (int j = tid; j < E; j += MT) {
        pc[j] = 1.0 - mdot2([&](int i) { return smooth[i]; }, [&](int i) { return FL(i * E + j) ? 1.0 : 0.0; }, N);
        int nz = 0;
        for (int i = 0; i < N; i++) nz += (FL(i * E + j) & 2) ? 1 : 0;
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
            nz += (FL(i * E + j) & 2) ? 1 : 0;
            nn += (FL(i * E + j) & 1) ? 1 : 0;
        }
        narow[i] = (double)nz;
        pr[i] = 1.0 - narow[i] / (double)E;
        rmask[i] = nn == E ? 1.0 : 0.0;  // Q15: a fully NaN row is masked
        a2v[i] = rmask[i] != 0.0 ? 0.0 : fabs(pr[i]);
    }
    __syncthreads();
    if (tid == 0) {  // the three totals on three waves
        scal[8] = 1.0 - mpw([&](int j) { return pc[j]; }, E) / (double)E;  // pna
    } else if (tid == 64) {
        double S = mpw([&](int i) { return a2v[i]; }, N);
        const bool bump = S == 0;
        if (bump) S = mpw([&](int i) { return rmask[i] != 0.0 ? 0.0 : fabs(pr[i]) + 1.0; }, N);
        scal[9] = S;
        scal[10] = bump ? 1.0 : 0.0;
    } else if (tid == 128) {
        const double P = mpw([&](int j) { return fabs(pc[j]); }, E);
        const double Pp = P == 0 ? mpw([&](int j) { return fabs(pc[j]) + 1.0; }, E) : P;
        for (int j = 0; j < E; j++) relc[j] = P == 0 ? (fabs(pc[j]) + 1.0) / Pp : fabs(pc[j]) / Pp;
    }
    __syncthreads();
    const double pna = scal[8];
    // PCA: a NaN total of |u| (scal[5]) leaves the reference's this_rep / smooth_rep fully MASKED
    // (SPEC rep_masked: participation_columns, reporter_bonus, author_bonus are numpy.ma's data)
    const bool rep_masked = alg == PCX_ALG_PCA && __builtin_isnan(scal[5]);
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
        if (a.reporter_bonus) a.reporter_bonus[o] = (masked || rep_masked) ? rel[i] : rel[i] * pna + smooth[i] * (1.0 - pna);
    }
    for (int j = tid; j < E; j += MT) {
        const int64_t o = b * E + j;
        if (a.adj_first_loadings) a.adj_first_loadings[o] = loading[j];
        if (a.outcomes_raw) a.outcomes_raw[o] = raw[j];
        if (a.outcomes_adjusted) a.outcomes_adjusted[o] = adj[j];
        if (a.outcomes_final) a.outcomes_final[o] = fin[j];
        if (a.certainty) a.certainty[o] = cert[j];
        if (a.consensus_reward) a.consensus_reward[o] = reward[j];
        if (a.participation_columns) a.participation_columns[o] = rep_masked ? 1.0 : pc[j];
        if (a.author_bonus) a.author_bonus[o] = rep_masked ? 1.0 : relc[j] * pna + reward[j] * (1.0 - pna);
    }
    MSTAMP(15);
    if (a.stamps && tid == 0)
        for (int k = 0; k < 3; k++) a.stamps[b * 32 + 20 + k] = mprof[k];
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

size_t medium_lds_bytes(int N, int E, int alg) {
    return ((size_t)medium_work(N, E, alg) + (size_t)VN_COUNT * N + (size_t)VE_COUNT * E) * sizeof(double) +
           (size_t)((N * E + 15) >> 4) * 4 + 16;
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
    const size_t lds = medium_lds_bytes(a.N, a.E, a.algorithm);
    // (dynamic LDS above 64 KB needs no attribute on gfx950: the launch checks it against 160 KB)
    (void)hipGetLastError();  // report launch errors only
    hipLaunchKernelGGL(medium_round_kernel, dim3((unsigned)nb), dim3(MT), lds, st, a, b0, Fscr, Cscr);
    return hipGetLastError();
}

}  // namespace pcx
