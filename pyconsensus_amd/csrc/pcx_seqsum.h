// pcx_seqsum.h -- sequential float sums of a constant, in O(log k).
//
// weightedstats.weighted_median (called at pyconsensus/__init__.py:303, :520-523) and
// the interpolation loop (:292-299) add weights one at a time with builtin float
// arithmetic: S(k) = (((0 + c) + c) + ...) + c, each addition rounded to nearest-even.
// When every weight of a column is the same double c (reputation=None, config C5) the
// whole walk is a function of the count alone, so the reference's decisions can be
// replayed without sorting or touching the data:
//
//   * inside one binade [2^e, 2^(e+1)) the spacing U is fixed and S is a multiple of
//     U, so fl(S + c) = S + RN_U(c): a constant increment d (a tie c mod U = U/2 rounds
//     to even, which leaves S/U even after one step, so from then on d is constant too);
//   * two real additions confirm the increment, then j steps advance S by exactly j*d
//     while S + c stays below the binade top; the few steps at each binade edge are
//     real additions.  ~2 * log2(k) binades are crossed, each in O(1).
//
// Everything is plain IEEE fp64 (the file is compiled with -ffp-contract=off); the
// host build is tested against the brute-force loop (tests/test_seqsum.py).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace pcx {

__host__ __device__ inline double seq_binade_top(double S) {  // least power of two > S > 0
    int e;
    (void)frexp(S, &e);
    return ldexp(1.0, e);
}

// largest m >= 0 such that the m steps S -> S + d -> ... from S are all exact bulk steps
// (S + (m-1)*d + c < top), minus one for the rounding of this estimate
__host__ __device__ inline int64_t seq_room(double S, double c, double d, double top) {
    const double r = floor((top - S - c) / d) - 1.0;
    return r > 0.0 ? (r > 9.0e15 ? (int64_t)9e15 : (int64_t)r) : 0;
}

// S(K) for K >= 0 (S(0) = 0: the builtin sum of nothing)
__host__ __device__ inline double seqsum_const(double c, int64_t K) {
    if (K <= 0) return 0.0;
    if (!(c > 0.0) || !isfinite(c)) {  // zero, negative, NaN, inf: no bulk stepping
        double S = 0.0;
        for (int64_t k = 0; k < K && k < 4; k++) S = S + c;
        if (K <= 4 || c == 0.0 || !isfinite(c)) return K <= 4 ? S : (c == 0.0 ? 0.0 : c * (double)K);
        S = 0.0;
        for (int64_t k = 0; k < K; k++) S = S + c;  // negative c (not a weight): plain loop
        return S;
    }
    double S = c;
    int64_t k = 1;
    while (k < K) {
        const double S1 = S + c;
        const double S2 = S1 + c;
        const double d = S1 - S, d2 = S2 - S1;
        const double top = seq_binade_top(S);
        if (d == d2 && d > 0.0 && S2 < top) {
            int64_t m = seq_room(S, c, d, top);
            if (m > K - k) m = K - k;
            if (m >= 2) {
                S = S + (double)m * d;  // exact: a multiple of U below the binade top
                k += m;
                continue;
            }
        }
        S = S1;
        k++;
    }
    return S;
}

// least k >= 1 with S(k) > t; kmax + 1 if S(k) <= t for every k <= kmax
__host__ __device__ inline int64_t seqsum_first_above(double c, double t, int64_t kmax) {
    if (kmax <= 0) return kmax + 1;
    if (!(c > 0.0) || !isfinite(c)) {
        double S = 0.0;
        for (int64_t k = 1; k <= kmax; k++) {
            S = S + c;
            if (S > t) return k;
            if (!(c > 0.0) && k > 4) break;  // never grows
        }
        return kmax + 1;
    }
    double S = c;
    int64_t k = 1;
    while (true) {
        if (S > t) return k;
        if (k >= kmax) return kmax + 1;
        const double S1 = S + c;
        const double S2 = S1 + c;
        const double d = S1 - S, d2 = S2 - S1;
        const double top = seq_binade_top(S);
        if (d == d2 && d > 0.0 && S2 < top) {
            int64_t m = seq_room(S, c, d, top);
            // stay at or below t: S + m*d <= t for m <= (t - S)/d, minus one for rounding
            const double q = floor((t - S) / d) - 1.0;
            const int64_t mt = q > 0.0 ? (q > 9.0e15 ? (int64_t)9e15 : (int64_t)q) : 0;
            if (m > mt) m = mt;
            if (m > kmax - k) m = kmax - k;
            if (m >= 2) {
                S = S + (double)m * d;
                k += m;
                continue;
            }
        }
        S = S1;
        k++;
    }
}

}  // namespace pcx
