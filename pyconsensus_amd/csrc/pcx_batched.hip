// pcx_batched.hip -- batched oracle rounds on MI355X (gfx950): one wavefront per
// independent round (Simulator.jl-style Monte Carlo, README.rst:52-56).
//
// Each workgroup is ONE wave64 that runs a complete
// Oracle(reports, event_bounds, reputation).consensus()
// (pyconsensus/__init__.py:102-611, algorithm="PCA") for one N x E round held in
// LDS (N <= 64 reporters: one lane per reporter row; E <= 32 events: one lane per
// event column).  All arithmetic is IEEE fp64; the file is compiled with
// -ffp-contract=off and every fma() is deliberate.  The arithmetic order is the
// one written down in oracle/pcx_oracle_batched.c (the "SPEC"), so results are
// bit-identical to that CPU restatement; see there for which steps replay the
// reference's numpy order exactly and which use compensated dots / power
// iteration in place of OpenBLAS / LAPACK.
//
// Lane roles per phase:
//   row phase    lane i = reporter i      (rescale, fill, scores, bonuses)
//   column phase lane j = event j         (sequential column sums, GEMV^T, ranks)
//   entry phase  lane o = matrix entry o  (covariance, matrix squaring)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "pcx_internal.h"

namespace pcx {

namespace {

constexpr int W = 64;        // wavefront
constexpr int NMAX = 64;  // reporters per round (one lane each)
constexpr int EMAX = 32;  // events per round (MFMA tiles 2 x 16; pcx_api.cpp validates)
static_assert(EMAX <= 2 * 16, "2 x 2 grid of 16 x 16 MFMA tiles");
static_assert(NMAX == W, "one reporter per lane");

// power iteration constants (SPEC; equal to oracle/pcx_oracle_batched.c)
constexpr double PI_TOL = 1e-14;
constexpr int PI_MAXIT = 256;
constexpr int PI_PRESQUARE = 3;
constexpr int PI_SQUARE_EVERY = 32;
constexpr int PI_MAX_SQUARINGS = 8;
constexpr int PI_POLISH = 2;
constexpr double DBL_MIN_ = 2.2250738585072014e-308;
constexpr double DBL_EPS = 2.220446049250313080847e-16;

__device__ __forceinline__ int lane_id() { return threadIdx.x; }

// The round's helpers run inlined: the 50 x 20 kernel is ~83 KB of code, yet the instruction
// cache misses 0.14 % of its fetches (SQC_ICACHE_MISSES / HITS, profiles/r3); outlined (calls,
// __noinline__, 49 KB + shared helpers) the call ABI spills and the kernel ran 29 %
// slower (24.4 M vs 34.4 M rounds/s).
#define PCX_OUTLINE __forceinline__

// diagnostic phase stamps (PCX_STAMPS=1): shader-clock reads at phase boundaries
#define STAMP(k)                                                                  \
    do {                                                                          \
        if (a.stamps) {                                                           \
            const long long t_ = (long long)__builtin_amdgcn_s_memtime();         \
            if (threadIdx.x == 0) a.stamps[b * 32 + (k)] = t_;                    \
        }                                                                         \
    } while (0)

// One wave per workgroup: the LDS operations of a wave execute in issue order, so a
// compiler-ordering wave barrier suffices between an LDS write and another lane's read
// (no lgkmcnt(0) drain, which __syncthreads() emits).
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ int popc(uint64_t m) { return __popcll(m); }

// broadcast from a wave-uniform lane: v_readlane into SGPRs (no LDS-pipe round trip)
__device__ __forceinline__ double bcast(double v, int src) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// lane l <- lane l ^ S inside a 16-lane row, DPP only (VALU, no LDS-pipe round trip):
// quad_perm (1, 2), row_shr:4 / row_shl:4 selected by lane bit 2 (4), row_ror:8 (8)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
template <int S>
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v) {
    if constexpr (S == 1) return dpp32<0xB1>(v);
    else if constexpr (S == 2) return dpp32<0x4E>(v);
    else if constexpr (S == 8) return dpp32<0x128>(v);
    else {
        static_assert(S == 4, "row-local distances only");
        const uint32_t up = dpp32<0x114>(v), dn = dpp32<0x104>(v);  // lane l-4 | lane l+4
        return (threadIdx.x & 4) ? up : dn;
    }
}

template <int S>
__device__ __forceinline__ double xor_lane(double v) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = xor_lane32<S>((uint32_t)u), hi = xor_lane32<S>((uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ double lane_value(double v, int k) {  // lane k's v (k wave-uniform)
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, k);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), k);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// SPEC tree64: a butterfly inside each 16-lane row (xor 1, 2, 4, 8: every lane of a row
// ends with the same row sum R_r), then (R0 + R1) + (R2 + R3) from lanes 0, 16, 32, 48
__device__ __forceinline__ double tree_sum(double v) {
    v = v + xor_lane<1>(v);
    v = v + xor_lane<2>(v);
    v = v + xor_lane<4>(v);
    v = v + xor_lane<8>(v);
    return (lane_value(v, 0) + lane_value(v, 16)) + (lane_value(v, 32) + lane_value(v, 48));
}

// inclusive prefix sum over the lanes in lane order (row_shr DPP inside each 16-lane row, then the
// rows' totals by readlane): a fixed tree order, deterministic, within ~6 u of the exact sums
template <int D>
__device__ __forceinline__ double shr_lane(double v) {  // lane l <- lane l - D of its row, else +0.0
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, 0x110 + D, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), 0x110 + D, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double wave_scan_d(double v) {
    v = v + shr_lane<1>(v);
    v = v + shr_lane<2>(v);
    v = v + shr_lane<4>(v);
    v = v + shr_lane<8>(v);
    const double r0 = lane_value(v, 15), r1 = lane_value(v, 31), r2 = lane_value(v, 47);
    const int row = threadIdx.x >> 4;
    const double r01 = r0 + r1;
    return row == 0 ? v : v + (row == 1 ? r0 : row == 2 ? r01 : r01 + r2);
}

__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, xor_lane<1>(v));
    v = fmax(v, xor_lane<2>(v));
    v = fmax(v, xor_lane<4>(v));
    v = fmax(v, xor_lane<8>(v));
    return fmax(fmax(lane_value(v, 0), lane_value(v, 16)), fmax(lane_value(v, 32), lane_value(v, 48)));
}

__device__ __forceinline__ double catch_(double x, double tol) {  // __init__.py:251-258
    if (x < 1.5 - tol) return 1.0;
    if (x > 1.5 + tol) return 2.0;
    return 1.5;
}

__device__ __forceinline__ double readlane_d(double v, int k) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, k);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), k);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ double shr1_d(double v) {  // lane l <- lane l-1 (lane 0 <- 0.0)
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, 0x138, 0xf, 0xf, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), 0x138, 0xf, 0xf, true);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ double permute_d(int dst_lane, double v) {  // forward permute
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_permute(dst_lane * 4, (int)(uint32_t)u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_permute(dst_lane * 4, (int)(uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ int mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// numpy pairwise add.reduce (n <= 128 branch: 8 accumulators) of the lanes that
// have `sel` set, taken in lane order.  All 64 lanes call it; every lane gets the
// result.  Register-only: element p (p-th selected lane) is permuted to lane
// 8*(p%8) + p/8, so accumulator k's chain a_k, a_{k+8}, ... sits in lanes 8k..8k+7 and
// runs as a DPP wave_shr chain (each step recomputes final lanes identically); the
// accumulators, the fixed tree and the tail are then read back wave-uniformly.
// Same additions in the same order as numpy (and the C oracle's pw_sum).
__device__ PCX_OUTLINE double wave_pw_sum(double v, bool sel) {
    const int l = lane_id();
    const uint64_t m = ballot(sel);
    const int n = popc(m);
    if (n < 8) {
        double res = 0.0;
        uint64_t mm = m;
        while (mm) {
            const int k = __builtin_ctzll(mm);
            mm &= mm - 1;
            res += readlane_d(v, k);
        }
        return res;
    }
    const int p = sel ? mbcnt64(m) : n + mbcnt64(~m);
    const double a = permute_d((p & 7) * 8 + (p >> 3), v);
    const int T = n >> 3;  // full rounds of 8: positions < 8T feed the accumulators
    double c = a;
    for (int t = 1; t < T; t++) {
        const double prev = shr1_d(c);
        c = (l & 7) == 0 ? a : prev + a;
    }
    const double r0 = readlane_d(c, 0 * 8 + T - 1), r1 = readlane_d(c, 1 * 8 + T - 1);
    const double r2 = readlane_d(c, 2 * 8 + T - 1), r3 = readlane_d(c, 3 * 8 + T - 1);
    const double r4 = readlane_d(c, 4 * 8 + T - 1), r5 = readlane_d(c, 5 * 8 + T - 1);
    const double r6 = readlane_d(c, 6 * 8 + T - 1), r7 = readlane_d(c, 7 * 8 + T - 1);
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (int q = 8 * T; q < n; q++) res += readlane_d(a, (q & 7) * 8 + (q >> 3));
    return res;
}

// SPEC dot2 over rows i < N of column-strided data: a[i] * b[i*bs]
__device__ __forceinline__ double dot2(const double* a, const double* b, int bs, int n) {
    double s = 0.0, c = 0.0;
    for (int i = 0; i < n; i++) {
        const double x = a[i], y = b[i * bs];
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

// np.dot(v, F) for one event column j, in the operation order of numpy 2.2 / OpenBLAS
// 0.3.29 (SkylakeX kernels) in the build container, where the goldens come from -- the
// SPEC's ob_vecmat (oracle/pcx_oracle_batched.c), fitted bit for bit by
// tests/golden/probe_openblas_order.py.  Events j < E & ~3: reporters in blocks of 4, the
// second product rounded then fma with the 1st, 3rd, 4th, y = y + block; tails of 2 / 1.
// The last E % 4 events: a sequential fma chain (E == 2, 3: pairs y + fma(a, x, a' x')).
// E == 1: numpy's ddot (32-wide, then 16-wide fma accumulators, lanes (0+2)+(1+3), fma tail).
__device__ __noinline__ double ob_ddot(const double* v, const double* f, int ld, int n) {
    double acc8[4][8], acc4[4][4];
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int q = 0; q < 8; q++) acc8[r][q] = 0.0;
    const int n32 = n & -32, n16 = n & -16;
    for (int i = 0; i < n32; i += 32)
#pragma unroll
        for (int k = 0; k < 32; k++) acc8[k / 8][k % 8] = fma(v[i + k], f[(i + k) * ld], acc8[k / 8][k % 8]);
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int q = 0; q < 4; q++) acc4[r][q] = acc8[r][q] + acc8[r][q + 4];
    for (int i = n32; i < n16; i += 16)
#pragma unroll
        for (int k = 0; k < 16; k++) acc4[k / 4][k % 4] = fma(v[i + k], f[(i + k) * ld], acc4[k / 4][k % 4]);
    double A[4];
#pragma unroll
    for (int q = 0; q < 4; q++) A[q] = ((acc4[0][q] + acc4[1][q]) + acc4[2][q]) + acc4[3][q];
    double d = (A[0] + A[2]) + (A[1] + A[3]);
    for (int i = n16; i < n; i++) d = fma(v[i], f[i * ld], d);
    return d;
}

__device__ PCX_OUTLINE double ob_vecmat(const double* v, const double* f, int ld, int N, int E, int j) {
    if (E == 1) return ob_ddot(v, f, ld, N);
    if (j < (E & ~3)) {
        double y = 0.0;
        int n = 0;
        for (; n + 4 <= N; n += 4) {
            double t = f[(n + 1) * ld] * v[n + 1];
            t = fma(f[n * ld], v[n], t);
            t = fma(f[(n + 2) * ld], v[n + 2], t);
            t = fma(f[(n + 3) * ld], v[n + 3], t);
            y = y + t;
        }
        if (n + 2 <= N) {
            double t = f[(n + 1) * ld] * v[n + 1];
            t = fma(f[n * ld], v[n], t);
            y = y + t;
            n += 2;
        }
        if (n < N) y = y + f[n * ld] * v[n];
        return y;
    }
    double t = 0.0;
    int i = 0;
    if (E == 2 || E == 3)
        for (; i + 4 <= N; i += 4) {
            t = t + fma(f[i * ld], v[i], f[(i + 1) * ld] * v[i + 1]);
            t = t + fma(f[(i + 2) * ld], v[i + 2], f[(i + 3) * ld] * v[i + 3]);
        }
    for (; i < N; i++) t = fma(f[i * ld], v[i], t);
    return t;
}

// weightedstats.weighted_median restated (oracle/pcx_oracle.py): lane i holds the
// pair (x, w) if `sel`; W is the builtin sequential sum of the selected weights in
// lane order (computed by the caller).  Scratch: sx, sw (64 doubles each).
__device__ __noinline__ double wave_wmedian(double x, double w, bool sel, double W, double* sx, double* sw) {
    const int l = lane_id();
    const double mid = 0.5 * W;
    const uint64_t dom = ballot(sel && w > mid);
    if (dom) {
        // Python max(weights) then .index(): the first maximal weight
        double mx = wave_max(sel ? w : -__builtin_inf());
        const uint64_t at = ballot(sel && w == mx);
        return bcast(x, __builtin_ctzll(at));
    }
    if (!ballot(sel && w > 0.0)) return __builtin_nan("");
    const uint64_t selm = ballot(sel);
    const int n = popc(selm);
    wsync();
    if (sel) {
        sx[l] = x;
        sw[l] = w;
    }
    wsync();
    int r = 0;
    if (sel) {  // stable rank by (x, w)
        uint64_t rest = selm;
        while (rest) {
            const int mrow = __builtin_ctzll(rest);
            rest &= rest - 1;
            const double xm = sx[mrow], wm = sw[mrow];
            const bool lt = (xm < x) || (xm == x && wm < w);
            const bool eq = (xm == x) && (wm == w);
            r += (lt || (eq && mrow < l)) ? 1 : 0;
        }
    }
    wsync();
    if (sel) {
        sx[r] = x;
        sw[r] = w;
    }
    wsync();
    double res = 0.0;
    if (l == 0) {
        double cum = 0.0;
        int k = 0;
        bool fail = false;
        while (cum <= mid) {
            if (k == n) {
                fail = true;
                break;
            }
            cum += sw[k];
            k++;
        }
        if (fail) {
            res = __builtin_nan("");
        } else {
            const double before = cum - sw[k - 1];
            if (fabs(before - mid) < DBL_EPS) {
                if (k >= 2)
                    res = (sx[k - 2] + sx[k - 1]) / 2.0;
                else
                    res = n == 1 ? sx[0] / 1.0 : __builtin_nan("");
            } else {
                res = sx[k - 1];
            }
        }
    }
    return bcast(res, 0);
}

// The same weighted median as wave_wmedian, with the sort and the walk spread over
// the wave:
//  * rank: every selected lane counts the selected pairs strictly below its own in
//    the (x, w) order, one LDS-broadcast pass over the rows (unselected rows hold
//    (+inf, +inf), which no selected pair exceeds, so they need no mask);
//  * compare-equal pairs share that count; an LDS atomic on a per-rank counter
//    spreads them over [r, r + d).  Equal pairs are bitwise equal here (x and w are
//    never +-0 with equal partners: zero reports are missing), so their order cannot
//    change the walk;
//  * each pair is scattered to its rank (ox, ow), and the cumulative weight runs
//    left to right, eight broadcast loads per step group, stopping at the first
//    cum > mid: the SPEC's sequential sums bit for bit; `before` is the same subtraction.
// NaN keys have no total order: rounds with a NaN among the selected pairs take
// wave_wmedian (in ox / ow).  NR = compile-time row count bound (64 when the shape is dynamic).
// scr: med_scr(NR) doubles of LDS: ox [NR] | ow [med_ow(NR)] | NR int counters
// (ow holds the zero-padded walk groups: every prefetched group of eight).
__host__ __device__ constexpr int med_ow(int NR) { return (NR + 7) / 8 * 8 + 8; }
__host__ __device__ constexpr int med_scr(int NR) { return NR + med_ow(NR) + (NR + 1) / 2; }

// top 32 bits of the order-preserving key of a double (-0.0 folded onto +0.0)
__device__ __forceinline__ uint32_t key_hi32(double x) {
    uint64_t u = __double_as_longlong(x == 0.0 ? 0.0 : x);
    u = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
    return (uint32_t)(u >> 32);
}

// use_rank (wave-uniform): `rank` is already each selected lane's count of selected keys below
// its own (the rank loop is skipped); rank_out: when the rank loop runs, each lane's count
// wlazy: Wtot is not given; weightedstats' total (the selected weights summed in row order, an
// absent row adding +0.0) is formed only where a decision needs it.  A tree-order total Wt differs
// from it by < (N + 6) u Wt, so every comparison against mid = Wt / 2 that clears the slack
// 2^-45 Wt is the one the exact total would make.
template <int NR>
__device__ PCX_OUTLINE double wave_wmedian_rank(double x, double w, bool sel, double Wtot, int N, double* scr,
                                                    long long* prof = nullptr, bool use_rank = false, int rank = 0,
                                                    int* rank_out = nullptr, bool wlazy = false) {
    const int l = lane_id();
    double *ox = scr, *ow = scr + NR;
    int* cnt = reinterpret_cast<int*>(scr + NR + med_ow(NR));
    const long long t0 = prof ? (long long)__builtin_amdgcn_s_memtime() : 0;
    double slack = 0.0;
    // the exact total (row order, an absent row adding +0.0), read lane by lane: a near tie or
    // NaN data only, so it needs no LDS of its own (the sorted pairs may already fill ox / ow)
    auto exact_total = [&]() {
        const double v = sel ? w : 0.0;
        double t = 0.0;
        for (int i = 0; i < N; i++) t = t + readlane_d(v, i);
        slack = 0.0;
        return t;
    };
    if (wlazy) {
        Wtot = tree_sum(sel ? w : 0.0);
        slack = 0x1p-45 * Wtot;
        if (!(slack < __builtin_inf()) || ballot(sel && fabs(w - 0.5 * Wtot) <= slack)) Wtot = exact_total();
    }
    double mid = 0.5 * Wtot;
    if (ballot(sel && w > mid)) {  // weightedstats: a weight above half the total wins outright
        const double mx = wave_max(sel ? w : -__builtin_inf());
        return bcast(x, __builtin_ctzll(ballot(sel && w == mx)));  // first maximal weight
    }
    if (!ballot(sel && w > 0.0)) return __builtin_nan("");
    if (ballot(sel && (__builtin_isnan(x) || __builtin_isnan(w)))) {
        if (slack != 0.0) Wtot = exact_total();
        return wave_wmedian(x, w, sel, Wtot, ox, ow);
    }
    const int n = popc(ballot(sel));
    // rank by the top 32 bits of x's order-preserving key (one 32-bit compare per row,
    // four keys per LDS read; unselected rows hold the largest key, below no selected
    // one); pairs whose keys collide -- the atomic hands a rank out twice -- are rare and
    // take the (x, w) lexicographic pass
    uint32_t* kx = reinterpret_cast<uint32_t*>(ox);
    const uint32_t key = sel ? key_hi32(x) : 0xffffffffu;
    wsync();
    if (l < NR) {
        cnt[l] = 0;
        kx[l] = key;
    }
    for (int q = l; q < med_ow(NR); q += 64) ow[q] = 0.0;  // slots past n add +0.0 in the walk
    wsync();
    int r = 0;
    if (use_rank) {
        r = rank;
    } else {
#pragma unroll
        for (int m = 0; m < NR; m++) {
            if (NR == 64 && m >= N) break;
            r += kx[m] < key ? 1 : 0;
        }
        if (rank_out) *rank_out = r;
    }
    if (sel) atomicAdd(&cnt[r], 1);
    wsync();
    // rows sharing a key (equal x: e.g. the filled guesses of the outcome median, or a
    // 32-bit key collision) are ordered among themselves by (x, w, row), one step per
    // such row
    const bool tied = sel && cnt[r] > 1;
    uint64_t T = ballot(tied);
    int sub = 0;
    // (the tied rows' x, w and rank read from their lanes' registers: no LDS round trip per row)
    while (T) {
        const int m = __builtin_ctzll(T);
        T &= T - 1;
        const double xm = bcast(x, m), wm = bcast(w, m);
        const int rm = __builtin_amdgcn_readlane(r, m);
        const bool before = (xm < x) | ((xm == x) & ((wm < w) | ((wm == w) & (m < l))));
        sub += (tied && rm == r && before) ? 1 : 0;
    }
    if (sel) {
        ox[r + sub] = x;
        ow[r + sub] = w;
    }
    wsync();
    if (prof) {
        const long long t1 = (long long)__builtin_amdgcn_s_memtime();
        prof[0] += t1 - t0;
        prof[2] = t1;
    }
    // wave-uniform walk: cum_k = (((0 + w_0) + w_1) + ... + w_{k-1}), eight sorted
    // weights per step group as LDS broadcasts, the next group's loads issued before
    // the current group's dependent adds
    double cum = 0.0, before = 0.0;
    int k = 0;
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) v[q] = ow[q];
    bool walked = false;
    if (!ballot(sel && !(w >= 0.0))) {
        // non-negative weights.  First the prefix sums of the sorted weights in a tree order
        // (slot l on lane l; slots past n hold +0.0): they differ from the walk's sequential
        // sums by < (n + 6) u W, so when the tree sum crossing mid lies more than 2^-44 W above
        // it and its predecessor more than 2^-44 W + DBL_EPS below, the sequential walk crosses
        // at the same slot and the half test below fails -- decided without the serial chain.
        // Otherwise (a near tie) the walk runs.
        const double ps = wave_scan_d(ow[l]);  // (ow holds med_ow(NR) >= 64 slots)
        const double W = lane_value(ps, 63);
        const double margin = 0x1p-44 * W + slack;
        const uint64_t above = ballot(ps > mid);
        if (above) {
            const int j = __builtin_ctzll(above);
            const double sj = bcast(ps, j), sp = j > 0 ? bcast(ps, j - 1) : 0.0;
            if (j < n && sj - mid > margin && (j == 0 || mid - sp > margin + DBL_EPS)) {
                k = j + 1;
                before = j == 0 ? 0.0 : sp;  // j = 0: the walk's c_0 - w_0 = 0 exactly
                walked = true;
            }
        } else if (mid - W > margin) {
            walked = true;  // no crossing: k = 0
        }
    }
    if (!walked && slack != 0.0) {  // a near tie: the walk needs the exact total
        Wtot = exact_total();
        mid = 0.5 * Wtot;
    }
    if (walked) {
    } else if (!ballot(sel && !(w >= 0.0))) {
        // non-negative weights: the running sums only grow (slots past n add +0.0), so a
        // group holds the first cum > mid iff its last sum exceeds mid
        for (int t = 0; t < n; t += 8) {
            double nv[8], c[8];
#pragma unroll
            for (int q = 0; q < 8; q++) nv[q] = ow[t + 8 + q];
            c[0] = cum + v[0];
#pragma unroll
            for (int q = 1; q < 8; q++) c[q] = c[q - 1] + v[q];
            if (c[7] > mid) {
                int hit = 7;
#pragma unroll
                for (int q = 6; q >= 0; q--)
                    if (c[q] > mid) hit = q;
                k = t + hit + 1;
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (q == hit) before = c[q] - v[q];
                break;
            }
            cum = c[7];
#pragma unroll
            for (int q = 0; q < 8; q++) v[q] = nv[q];
        }
    } else
    for (int t = 0; t < n; t += 8) {
        double nv[8], c[8];
#pragma unroll
        for (int q = 0; q < 8; q++) nv[q] = ow[t + 8 + q];
        c[0] = cum + v[0];
#pragma unroll
        for (int q = 1; q < 8; q++) c[q] = c[q - 1] + v[q];
        int hit = 8;
#pragma unroll
        for (int q = 7; q >= 0; q--)
            if (t + q < n && c[q] > mid) hit = q;
        if (hit < 8) {
            k = t + hit + 1;
#pragma unroll
            for (int q = 0; q < 8; q++)
                if (q == hit) before = c[q] - v[q];
            break;
        }
        cum = c[7];
#pragma unroll
        for (int q = 0; q < 8; q++) v[q] = nv[q];
    }
    if (prof) prof[1] += (long long)__builtin_amdgcn_s_memtime() - prof[2];
    if (!k) return __builtin_nan("");
    if (fabs(before - mid) < DBL_EPS) {
        if (k >= 2) return (ox[k - 2] + ox[k - 1]) / 2.0;
        return n == 1 ? ox[0] / 1.0 : __builtin_nan("");
    }
    return ox[k - 1];
}


// the N x E round in LDS (row pitch ES) -> dst [N][E] row-major, lane-contiguous: each store
// instruction covers 64 consecutive elements (16-byte pairs when N * E is even and the
// shape is compiled in)
__device__ __forceinline__ void round_to_global(double* dst, const double* F, int N, int E, int ES, int NT, int ET) {
    const int l = lane_id();
    if (NT > 0 && ET > 0 && (NT * ET) % 2 == 0 && ((uintptr_t)dst & 15) == 0) {
        const int tot2 = NT * ET / 2;
        for (int q = l; q < tot2; q += W) {
            const int idx = 2 * q;
            const int i0 = idx / ET, j0 = idx - i0 * ET;
            const int i1 = (idx + 1) / ET, j1 = idx + 1 - i1 * ET;
            reinterpret_cast<double2*>(dst)[q] = double2{F[i0 * ES + j0], F[i1 * ES + j1]};
        }
    } else {
        for (int idx = l; idx < N * E; idx += W) {
            const int i = idx / E, j = idx - i * E;
            dst[idx] = F[i * ES + j];
        }
    }
}

// scipy.stats.rankdata(method='average') of v[0..E) in LDS; lane j < E returns rank j
__device__ PCX_OUTLINE double rank_avg(const double* v, int E) {
    const int l = lane_id();
    double r = 0.0;
    if (l < E) {
        const double x = v[l];
        int lt = 0, eq = 0;
        for (int k = 0; k < E; k++) {
            const double y = v[k];
            lt += y < x;
            eq += y == x;
        }
        r = (double)lt + (double)(eq + 1) * 0.5;
        if (__builtin_isnan(x)) r = __builtin_nan("");  // rankdata propagates NaN: the rule's sums go NaN
    }
    return r;
}

struct Smem {
    double* F;      // [N][ES] rescaled, then filled reports
    double* C;      // [E][ES] covariance (phase aliases: see carve)
    double* M;      // [max(E*ES, MED_SCR)] power-iteration / Jacobi working matrix
    double* rep;    // [N] (aliases C: dead once the covariance has its tokens)
    double* n1;     // [N] normalize(set1) (aliases C)
    double* n2;     // [N] normalize(set2) (aliases C)
    double* smooth; // [N] (aliases C)
    double* mu;     // [E] full layout only (the clusterings' mean; the rest read lane registers)
    double* tot;    // [E] present-reputation totals of the interpolation medians (aliases M)
    double* guess;  // [E] (aliases C)
    double* x;      // [E] full layout only: the Jacobi rotations' cos
    double* ld;     // [E] full layout only: the Jacobi rotations' sin
    double* old;    // [E] (aliases C)
    double* nv1;    // [E] (aliases M)
    double* nv2;    // [E] (aliases M)
    double* adj;    // [E] (aliases C)
    uint64_t* miss; // [E] bit i = report (i, j) is NaN or 0.0 (the per-row / per-column counts
                    // of each kind are lane registers)
};

// LDS per round, by phase.  The kernel is latency bound: throughput scales with the
// rounds resident per CU (tools/occupancy_batched.py), and LDS is what bounds them, so
// vectors whose lifetimes do not overlap the matrices' share their space:
//   C  (covariance, Jacobi V) is live from the covariance to the scores only; before
//      it holds guess | rep (load to fill | load to the covariance's tokens), after it
//      n1 | n2 | smooth | adj | old;
//   M  (squared matrix, Jacobi A) is dead in both median phases, where the median
//      scratch (med_scr doubles) lives, and after the eigenpairs, where nv1 | nv2 live;
//   the power-iteration vector, the loading and the weighted mean are lane registers, read
//      by other lanes through readlane / ds_bpermute (no LDS); the full layout keeps mu
//      (the clusterings read it) and x | ld as the Jacobi rotations' cos | sin.
// The integer tokens are recomputed from rep where the covariance needs them.  Per-row
// vectors hold N entries, per-event vectors E (rounded up to even).  LDS is allocated in
// 1,280-byte units (160 KiB / 128; measured with PCX_BATCHED_LDS_PAD: a 50 x 20 round of
// 12,800 bytes ran twelve to a CU, one of 13,192 eleven).
__host__ __device__ inline int smem_rows(int N) { return (N + 1) & ~1; }
// F also holds the certainty phase's compacted hit lists, [E][cert_stride] (an odd stride with
// the odd row pitch; the even pitch of PCX_BATCHED_ES_EVEN keeps N)
__host__ __device__ inline int cert_stride(int N, int ES) { return (ES & 1) ? (N | 1) : N; }
__host__ __device__ inline int smem_f_size(int N, int E, int ES) {
    return N * ES > E * cert_stride(N, ES) ? N * ES : E * cert_stride(N, ES);
}
__host__ __device__ inline int smem_evs(int E) { return (E + 1) & ~1; }
// C and M: full [E][ES] (the Jacobi eigenpairs of big-five / fixed-variance need a
// general V), or -- every other algorithm -- packed lower triangles (both are symmetric:
// the squared M bitwise too).
__host__ __device__ inline int smem_mat(int E, int ES, bool pk) { return pk ? E * (E + 1) / 2 : E * ES; }
__host__ __device__ inline int smem_c_size(int N, int E, int ES, bool pk) {
    const int need = 3 * smem_rows(N) + 2 * smem_evs(E);
    return smem_mat(E, ES, pk) > need ? smem_mat(E, ES, pk) : need;
}
__host__ __device__ inline int smem_m_size(int E, int ES, int NR, bool pk) {
    const int scr = med_scr(NR) + smem_evs(E);  // the median scratch and the totals beside it
    const int need = scr > 2 * smem_evs(E) ? scr : 2 * smem_evs(E);
    return smem_mat(E, ES, pk) > need ? smem_mat(E, ES, pk) : need;
}

__host__ __device__ inline size_t smem_doubles(int N, int E, int ES, int NR, bool pk) {
    return (size_t)smem_f_size(N, E, ES) + smem_c_size(N, E, ES, pk) + smem_m_size(E, ES, NR, pk) +
           (pk ? 1 : 4) * (size_t)smem_evs(E);
}

// entry (j, k) of the symmetric C / M
template <bool PK>
__device__ __forceinline__ int sym_at(int j, int k, int ES) {
    if constexpr (PK)
        return j >= k ? j * (j + 1) / 2 + k : k * (k + 1) / 2 + j;
    else
        return j * ES + k;
}

__device__ Smem carve(double* base, int N, int E, int ES, int NR, bool pk) {
    const int nr = smem_rows(N), ne = smem_evs(E);
    Smem s;
    double* p = base;
    s.F = p; p += smem_f_size(N, E, ES);
    s.C = p; p += smem_c_size(N, E, ES, pk);
    s.M = p; p += smem_m_size(E, ES, NR, pk);
    s.miss = reinterpret_cast<uint64_t*>(p); p += ne;
    s.mu = s.x = s.ld = nullptr;
    if (!pk) {
        s.mu = p; p += ne;
        s.x = p; p += ne;
        s.ld = p; p += ne;
    }
    // phase aliases (see above)
    s.tot = s.M + med_scr(NR);
    s.rep = s.C + ne;  // (beside guess, C[0, E))
    s.guess = s.C;
    s.n1 = s.C;
    s.n2 = s.C + nr;
    s.smooth = s.C + 2 * nr;
    s.adj = s.C + 3 * nr;
    s.old = s.C + 3 * nr + ne;
    s.nv1 = s.M;
    s.nv2 = s.M + ne;
    return s;
}

// y = normalize(M x) for lane j < E, x_k on lane k; returns y_j (0 on other lanes)
template <bool PK>
__device__ PCX_OUTLINE double matvec_unit(const double* M, int ES, double xv, int E) {
    const int l = lane_id(), r = l < E ? l : 0;  // (every lane runs the chain: readlane is wave-wide)
    double acc = 0.0;
    for (int k = 0; k < E; k++) acc = fma(M[sym_at<PK>(r, k, ES)], lane_value(xv, k), acc);
    const double y = l < E ? acc : 0.0;
    const double nrm = sqrt(tree_sum(l < E ? y * y : 0.0));
    return l < E ? y / nrm : 0.0;
}

typedef double d4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4v mfma_f64(double a, double b, d4v c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// M <- (M M) / max|M M| (SPEC square_scaled) on fp64 MFMA.  v_mfma_f64_16x16x4_f64
// accumulates exactly like the SPEC's fma chain over m (tools/probes/mfma_f64_order:
// bitwise equal), and the zero padding of the 32 x 32 tile adds exact zeros, so every
// entry is bit-identical to the VALU loop.  E <= 32: a 2 x 2 grid of 16 x 16 tiles.
// M symmetric: A[ml][mm] = B[mm][ml], one read per operand pair.
template <bool PK>
__device__ PCX_OUTLINE void square_scaled(double* M, int ES, int E) {
    const int l = lane_id(), ml = l & 15, kq = l >> 4;
    const bool two = E > 16;
    d4v t00 = {0, 0, 0, 0}, t01 = {0, 0, 0, 0}, t10 = {0, 0, 0, 0}, t11 = {0, 0, 0, 0};
    for (int m0 = 0; m0 < E; m0 += 4) {
        const int mm = m0 + kq;
        const bool ok = mm < E;
        const double a0 = (ok && ml < E) ? M[sym_at<PK>(ml, mm, ES)] : 0.0;
        const double b0 = a0;
        t00 = mfma_f64(a0, b0, t00);
        if (two) {
            const double a1 = (ok && 16 + ml < E) ? M[sym_at<PK>(16 + ml, mm, ES)] : 0.0;
            const double b1 = a1;
            // PK: the upper tile t01 = t10^T bit for bit (the same products in the same m
            // order), neither stored nor needed for the maximum (C3: 1.826 -> 1.786 ms)
            if (!PK) t01 = mfma_f64(a0, b1, t01);
            t10 = mfma_f64(a1, b0, t10);
            t11 = mfma_f64(a1, b1, t11);
        }
    }
    double mx = 0.0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int j0 = kq + 4 * r, j1 = 16 + kq + 4 * r, k0 = ml, k1 = 16 + ml;
        if (j0 < E && k0 < E) mx = fmax(mx, fabs(t00[r]));
        if (!PK && j0 < E && k1 < E) mx = fmax(mx, fabs(t01[r]));
        if (j1 < E && k0 < E) mx = fmax(mx, fabs(t10[r]));
        if (j1 < E && k1 < E) mx = fmax(mx, fabs(t11[r]));
    }
    mx = wave_max(mx);
    // SPEC: scale by the power of two that brings max|MM| into [1, 2) (exact); a zero,
    // subnormal or non-finite maximum divides instead
    const bool pow2 = mx >= DBL_MIN_ && __builtin_isfinite(mx);
    const double sc = pow2 ? ldexp(1.0, -ilogb(mx)) : 1.0;
    auto scaled = [&](double t) { return pow2 ? t * sc : (mx > 0.0 ? t / mx : t); };
    wsync();
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int j0 = kq + 4 * r, j1 = 16 + kq + 4 * r, k0 = ml, k1 = 16 + ml;
        if (j0 < E && k0 < E && (!PK || k0 <= j0)) M[sym_at<PK>(j0, k0, ES)] = scaled(t00[r]);
        if (j0 < E && k1 < E && !PK) M[sym_at<PK>(j0, k1, ES)] = scaled(t01[r]);
        if (j1 < E && k0 < E) M[sym_at<PK>(j1, k0, ES)] = scaled(t10[r]);
        if (j1 < E && k1 < E && (!PK || k1 <= j1)) M[sym_at<PK>(j1, k1, ES)] = scaled(t11[r]);
    }
    wsync();
}

// ---- "big-five" / "fixed-variance" eigenpairs: SPEC jacobi_eig of
// oracle/pcx_oracle_batched.c (cyclic two-sided Jacobi, round-robin pairs; each
// step's angles from the matrix at the step's start, rows then columns), one lane
// per (pair, row/column) element -- the same arithmetic, so bit-identical.
constexpr int JAC_MAXSWEEP = 30;
constexpr double JAC_TOL = 1e-15;

__device__ __forceinline__ void jac_pair(int i, int r, int n, int& p, int& q) {
    const int a = i == 0 ? 0 : 1 + (i - 1 + r) % (n - 1);
    const int b = 1 + (n - 2 - i + r) % (n - 1);
    p = a < b ? a : b;
    q = a < b ? b : a;
}

// A (E x E, row stride ES) -> eigenvalues on its diagonal; V -> eigenvectors (columns).
// pc, ps: rotation cosines and sines, npair <= 16 doubles of LDS each.
__device__ void jacobi_eig_wave(double* A, double* V, int ES, int E, double* pc, double* ps) {
    const int l = lane_id();
    for (int o = l; o < E * E; o += W) {
        const int j = o / E, k = o - j * E;
        V[j * ES + k] = j == k ? 1.0 : 0.0;
    }
    wsync();
    if (E < 2) return;
    const int n = E + (E & 1), npair = n / 2;
    for (int sweep = 0; sweep < JAC_MAXSWEEP; sweep++) {
        double off = 0.0, dg = 0.0;  // max-norms: exact in any order
        for (int o = l; o < E * E; o += W) {
            const int j = o / E, k = o - j * E;
            const double v = fabs(A[j * ES + k]);
            if (j == k)
                dg = fmax(dg, v);
            else
                off = fmax(off, v);
        }
        off = wave_max(off);
        dg = wave_max(dg);
        if (!(off > JAC_TOL * dg)) break;
        for (int r = 0; r < n - 1; r++) {
            if (l < npair) {
                int p, q;
                jac_pair(l, r, n, p, q);
                double c = 1.0, s = 0.0;
                if (q < E) {
                    const double apq = A[p * ES + q];
                    if (apq != 0.0) {
                        const double app = A[p * ES + p], aqq = A[q * ES + q];
                        const double tau = (aqq - app) / (2.0 * apq);
                        const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
                        c = 1.0 / sqrt(1.0 + t * t);
                        s = t * c;
                    }
                }
                pc[l] = c;
                ps[l] = s;
            }
            wsync();
            for (int o = l; o < npair * E; o += W) {  // rows p, q
                const int i = o / E, k = o - i * E;
                const double s = ps[i];
                if (s == 0.0) continue;
                int p, q;
                jac_pair(i, r, n, p, q);
                const double c = pc[i];
                const double apk = A[p * ES + k], aqk = A[q * ES + k];
                A[p * ES + k] = c * apk - s * aqk;
                A[q * ES + k] = s * apk + c * aqk;
            }
            wsync();
            for (int o = l; o < npair * E; o += W) {  // columns p, q of A and V
                const int i = o / E, j = o - i * E;
                const double s = ps[i];
                if (s == 0.0) continue;
                int p, q;
                jac_pair(i, r, n, p, q);
                const double c = pc[i];
                const double ajp = A[j * ES + p], ajq = A[j * ES + q];
                A[j * ES + p] = c * ajp - s * ajq;
                A[j * ES + q] = s * ajp + c * ajq;
                const double vjp = V[j * ES + p], vjq = V[j * ES + q];
                V[j * ES + p] = c * vjp - s * vjq;
                V[j * ES + q] = s * vjp + c * vjq;
            }
            wsync();
        }
    }
}

// ---- clustering algorithms (SPEC: oracle/pcx_oracle_batched.c) ------
// k-means (:392-405), hierarchical (:407-419) and clusterfeck (:148-242, :421-424) each
// turn the filled reports into the nonconformity vector; they run in their own kernel
// instantiation (CLUS = true) with an extra LDS region X, so the PCA kernel is untouched.
constexpr int KMAX = 8;  // k-means code books: ceil(sqrt(64))
constexpr int KMEANS_MAXIT = 4096;  // Lloyd steps per restart (a guard; scipy has none)

__host__ __device__ inline int cluster_lds_doubles(int N, int E, int ES) {
    const int nr = smem_rows(N), ne = smem_evs(E);
    const int feck = N * ES + 6 * nr + 2 * ne;                          // sums, 6 row vectors, outcomes
    const int km = N * ES + 2 * KMAX * ES + ne + 2 * nr + 2 * KMAX;     // obs, books, sd, labels, counts
    return feck > km ? feck : km;
}

// numpy pairwise add.reduce of get(0..n-1) on ONE lane (n <= 128: eight accumulators)
template <class G>
__device__ __forceinline__ double lane_pw_sum(G get, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; i++) r += get(i);
        return r;
    }
    double r0 = get(0), r1 = get(1), r2 = get(2), r3 = get(3), r4 = get(4), r5 = get(5), r6 = get(6), r7 = get(7);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
        r0 += get(i); r1 += get(i + 1); r2 += get(i + 2); r3 += get(i + 3);
        r4 += get(i + 4); r5 += get(i + 5); r6 += get(i + 6); r7 += get(i + 7);
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; i++) res += get(i);
    return res;
}

// (size - min size) / sum over the row lanes (:398-405); the integer sum is exact, and
// equal sizes give 0/0 = NaN as numpy does
__device__ __forceinline__ double nc_from_sizes(double size, bool row) {
    const double mn = -wave_max(row ? -size : -__builtin_inf());
    const double tot = tree_sum(row ? size - mn : 0.0);
    return row ? (size - mn) / tot : 0.0;
}

// hierarchical: single-linkage flat clusters at cophenetic distance <= t = connected
// components of {d_ij <= t}, d_ij = sqrt(sequential sum of squared wcd differences)
// (scipy pdist order).  Lane i owns row i's adjacency mask; masks are closed under
// "OR the masks of my members" until no lane changes.
__device__ __noinline__ double hier_nc(const double* F, const double* mu, int ES, int N, int E, double t,
                                       uint64_t* comp) {
    const int l = lane_id();
    const bool row = l < N;
    uint64_t adj = 0;
    if (row) {
        adj = 1ull << l;
        for (int j = 0; j < N; j++) {
            double d2 = 0.0;
            for (int k = 0; k < E; k++) {
                const double df = (F[l * ES + k] - mu[k]) - (F[j * ES + k] - mu[k]);
                d2 = d2 + df * df;
            }
            if (sqrt(d2) <= t) adj |= 1ull << j;
        }
        comp[l] = adj;
    }
    wsync();
    for (;;) {
        uint64_t nw = adj;
        if (row) {
            uint64_t m = adj;
            while (m) {
                const int j = __builtin_ctzll(m);
                m &= m - 1;
                nw |= comp[j];
            }
        }
        const bool changed = nw != adj;
        wsync();
        if (row) comp[l] = nw;
        adj = nw;
        wsync();
        if (!ballot(changed)) break;
    }
    return nc_from_sizes(row ? (double)popc(adj) : 0.0, row);
}

// scipy _vq.vq distance^2 as built in the goldens' container: naive for E < 5, else
// -2 x.c (OpenBLAS: one fma chain for K < 32, eight chains + tree at K = 32) + |x|^2 + |c|^2
__device__ __forceinline__ double vq_d2(const double* x, const double* c, int E, double xs, double cs) {
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
        double q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < E; k += 8)
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (k + u < E) q[u] = fma(x[k + u], c[k + u], q[u]);
        dot = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
    }
    return (-2.0 * dot + xs) + cs;
}

__device__ __forceinline__ double sqsum(const double* x, int E) {
    double s = 0.0;
    for (int k = 0; k < E; k++) s = s + x[k] * x[k];
    return s;
}

// k-means: whiten(wcd), scipy kmeans(obs, k) over the host-drawn restarts (best mean
// distortion, strict <), vq labels, cluster sizes.  Lane i = observation i in vq;
// lanes take (code, feature) pairs in the mean update.
__device__ __noinline__ double kmeans_nc(const BatchArgs& a, int64_t b, const double* F, const double* mu, int ES,
                                         int N, int E, double* X) {
    const int l = lane_id();
    const bool row = l < N, col = l < E;
    const int nr = smem_rows(N), ne = smem_evs(E);
    double* obs = X;                       // [N][ES]
    double* book = obs + N * ES;           // [KMAX][ES]
    double* best = book + KMAX * ES;       // [KMAX][ES]
    double* sd = best + KMAX * ES;         // [E]
    int* lab = reinterpret_cast<int*>(sd + ne);  // [N]
    double* csq = sd + ne + 2 * nr;        // [KMAX]
    int* cntv = reinterpret_cast<int*>(csq + KMAX);  // [KMAX]
    // np.std(wcd, axis=0): sequential column sums (pairwise when E == 1); 0 -> 1
    double sdj = 0.0;
    if (E == 1) {
        const double w = row ? F[l * ES] - mu[0] : 0.0;
        const double m = wave_pw_sum(w, row) / (double)N;
        const double q = row ? (w - m) * (w - m) : 0.0;
        sdj = sqrt(wave_pw_sum(q, row) / (double)N);
    } else if (col) {
        double s = 0.0;
        for (int i = 0; i < N; i++) s = s + (F[i * ES + l] - mu[l]);
        const double m = s / (double)N;
        double v = 0.0;
        for (int i = 0; i < N; i++) {
            const double d = (F[i * ES + l] - mu[l]) - m;
            v = v + d * d;
        }
        sdj = sqrt(v / (double)N);
    }
    if (sdj == 0.0) sdj = 1.0;
    if (col) sd[l] = sdj;
    wsync();
    for (int o = l; o < N * E; o += W) {
        const int i = o / E, k = o - i * E;
        obs[i * ES + k] = (F[i * ES + k] - mu[k]) / sd[k];
    }
    wsync();
    const double xs = row ? sqsum(obs + l * ES, E) : 0.0;
    const int K = a.kmeans_k, RS = a.kmeans_restarts;
    const int32_t* init = a.kmeans_init + b * (int64_t)RS * K;
    double best_d = __builtin_inf();
    int best_n = 0;
    for (int r = 0; r < RS; r++) {
        for (int o = l; o < K * E; o += W) {
            const int c = o / E, k = o - c * E;
            const int row0 = init[r * K + c];
            book[c * ES + k] = obs[(row0 < 0 ? 0 : row0 >= N ? N - 1 : row0) * ES + k];
        }
        int nc = K;
        double prev0 = __builtin_inf(), prev1 = __builtin_inf();
        for (int it = 0;; it++) {
            wsync();
            if (l < nc) csq[l] = sqsum(book + l * ES, E);
            wsync();
            int li = 0;
            double low = __builtin_inf();
            if (row)
                for (int c = 0; c < nc; c++) {
                    const double d = vq_d2(obs + l * ES, book + c * ES, E, xs, csq[c]);
                    if (d < low) {
                        low = d;
                        li = c;
                    }
                }
            const double dist = row ? (low > 0 ? sqrt(low) : 0.0) : 0.0;
            prev0 = prev1;
            prev1 = wave_pw_sum(dist, row) / (double)N;
            if (row) lab[l] = li;
            wsync();
            // update_cluster_means: member sums in row order, / count; empty codes dropped
            int cnt = 0;
            if (l < nc)
                for (int i = 0; i < N; i++) cnt += lab[i] == l;
            const uint64_t nonempty = ballot(l < nc && cnt > 0);
            double nv[4];
            int nk[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int p = l + W * q;
                nk[q] = -1;
                if (p < nc * E) {
                    const int c = p / E, k = p - c * E;
                    double sm = 0.0;
                    int n = 0;
                    for (int i = 0; i < N; i++)
                        if (lab[i] == c) {
                            sm = sm + obs[i * ES + k];
                            n++;
                        }
                    if (n > 0) {
                        nv[q] = sm / (double)n;
                        nk[q] = popc(nonempty & ((1ull << c) - 1)) * ES + k;
                    }
                }
            }
            wsync();
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (nk[q] >= 0) book[nk[q]] = nv[q];
            nc = popc(nonempty);
            if (!(fabs(prev0 - prev1) > 1e-5) || it + 1 >= KMEANS_MAXIT) break;
        }
        wsync();
        if (prev1 < best_d) {
            best_d = prev1;
            best_n = nc;
            for (int o = l; o < nc * ES; o += W) best[o] = book[o];
        }
    }
    wsync();
    if (best_n == 0) return row ? __builtin_nan("") : 0.0;  // no finite distortion: the reference raises
    if (l < best_n) csq[l] = sqsum(best + l * ES, E);
    wsync();
    int li = 0;
    double low = __builtin_inf();
    if (row)
        for (int c = 0; c < best_n; c++) {
            const double d = vq_d2(obs + l * ES, best + c * ES, E, xs, csq[c]);
            if (d < low) {
                low = d;
                li = c;
            }
        }
    if (row) lab[l] = li;
    wsync();
    if (l < best_n) {
        int n = 0;
        for (int i = 0; i < N; i++) n += lab[i] == l;
        cntv[l] = n;
    }
    wsync();
    return nc_from_sizes(row ? (double)cntv[li] : 0.0, row);
}

// clusterfeck: leader clustering of the filled reports with the token weights (0 -> 1e-5),
// mode = heaviest cluster; a mode farther than 1.07 from the weighted outcomes re-clusters
// once at 3x the cut and the closer mode wins; nc = normalize(1 - dist(own cluster, mode) /
// (max + 1e-8)).  Rows are visited in order (wave-uniform); lane x = cluster x.
struct Feck {
    double* sum;   // [N][ES] sum(vec * repVec, axis=0), running in member order
    double* crep;  // [N] running member weight
    int* first;    // [N] founding row (a singleton's meanVec)
    int* count;    // [N]
    int* of;       // [N] cluster of each row, -1 = none
    double* dx;    // [N] per-cluster distance to the mode
    const double* F;
    int ES, E;
    __device__ double mean(int x, int k) const {
        return count[x] == 1 ? F[first[x] * ES + k] : sum[x * ES + k] / crep[x];
    }
};

// one cluster() pass (:194-230); returns the mode (:162-165) and, through dm, the row
// distances of process() (:177-183) for that mode, and the mode's distance to outc
__device__ __noinline__ void feck_pass(Feck& f, const double* wv, int N, double thr, const double* outc, double& dmode,
                                       double& dm) {
    const int l = lane_id(), E = f.E, ES = f.ES;
    const bool col = l < E;
    int ncl = 0;
    for (int i = 0; i < N; i++) {
        const double* Fi = f.F + i * ES;
        const bool valid = l < ncl;
        double d = 0.0;
        if (valid)
            d = sqrt(lane_pw_sum([&](int k) { const double t = Fi[k] - f.mean(l, k); return t * t; }, E));
        const bool cand = valid && d < 0x1p255;
        const double dmin = -wave_max(cand ? -d : -__builtin_inf());
        const uint64_t at = ballot(cand && d == dmin);
        const double wi = wv[i];
        if (at && dmin < thr) {
            const int bx = __builtin_ctzll(at);
            if (col) f.sum[bx * ES + l] = f.sum[bx * ES + l] + Fi[l] * wi;
            wsync();
            if (l == 0) {
                f.crep[bx] = f.crep[bx] + wi;
                f.count[bx] += 1;
                f.of[i] = bx;
            }
        } else if (!ballot(col && __builtin_isnan(Fi[l]))) {
            const int x = ncl++;
            if (col) f.sum[x * ES + l] = Fi[l] * wi;
            if (l == 0) {
                f.first[x] = i;
                f.count[x] = 1;
                f.crep[x] = wi;
                f.of[i] = x;
            }
        } else if (l == 0) {
            f.of[i] = -1;
        }
        wsync();
    }
    const bool valid = l < ncl;
    const double r = valid ? f.crep[l] : 0.0;
    const double top = wave_max(valid ? r : -__builtin_inf());
    const uint64_t tm = ballot(valid && r == top && r > 0.0);
    const int mode = tm ? __builtin_ctzll(tm) : 0;
    dmode = sqrt(lane_pw_sum([&](int k) { const double t = f.mean(mode, k) - outc[k]; return t * t; }, E));
    if (valid) f.dx[l] = sqrt(lane_pw_sum([&](int k) { const double t = f.mean(mode, k) - f.mean(l, k); return t * t; }, E));
    wsync();
    dm = 0.0;
    if (l < N) {
        const int o = f.of[l];
        dm = o >= 0 ? f.dx[o] : 0.0;
    }
    wsync();
}

__device__ __noinline__ double feck_nc(const BatchArgs& a, const double* F, int ES, int N, int E, double rep,
                                       double* X) {
    const int l = lane_id();
    const bool row = l < N, col = l < E;
    const int nr = smem_rows(N), ne = smem_evs(E);
    Feck f;
    f.F = F;
    f.ES = ES;
    f.E = E;
    f.sum = X;
    f.crep = X + N * ES;
    f.first = reinterpret_cast<int*>(f.crep + nr);
    f.count = reinterpret_cast<int*>(f.crep + 2 * nr);
    f.of = reinterpret_cast<int*>(f.crep + 3 * nr);
    f.dx = f.crep + 4 * nr;
    double* wv = f.crep + 5 * nr;
    double* outc = wv + nr;  // [E]
    const double tok = trunc(rep * 1e6);
    const double w = row ? (tok == 0.0 ? 0.00001 : tok) : 0.0;  // :202-204
    if (row) wv[l] = w;
    double thr = a.cluster_threshold;
    if (!(thr > 0.0)) {
        thr = log10((double)E) / 1.77;
        if (thr == 0.0) thr = 0.3;
    }
    // outcomes = np.ma.average(features, axis=0, weights=rep) (:167)
    const double scl = wave_pw_sum(w, row);
    if (E == 1) {
        const double num = wave_pw_sum(row ? F[l * ES] * w : 0.0, row);
        if (l == 0) outc[0] = num / scl;
    }
    wsync();
    if (E > 1 && col) {
        double num = F[l] * wv[0];
        for (int i = 1; i < N; i++) num = num + F[i * ES + l] * wv[i];
        outc[l] = num / scl;
    }
    wsync();
    (void)ne;
    double d1, dm;
    feck_pass(f, wv, N, thr, outc, d1, dm);
    if (d1 > 1.07) {  // :174-176
        double d2, dm2;
        feck_pass(f, wv, N, thr * 3, outc, d2, dm2);
        if (d2 < d1) dm = dm2;
    }
    const double mx = wave_max(row ? dm : -__builtin_inf());
    const double rv = 1.0 - dm / (mx + 0.00000001);
    double u = row ? fabs(rv) : 0.0;
    double Su = wave_pw_sum(u, row);
    if (Su == 0) {
        u += 1.0;
        Su = wave_pw_sum(u, row);
    }
    return row ? u / Su : 0.0;
}

}  // namespace

// The compiled shapes' row pitch: E (1) or E | 1 (0).  The odd pitch spreads a row-phase column
// read over the banks, but 50 x 20 rounds at the even one fit nine LDS units instead of ten -- 14
// rounds a CU instead of 12 with the 128-VGPR budget below (C3: 1.53 -> 1.46 ms, 42.5 -> 44.6 M
// rounds/s; the even pitch under the three-wave budget, 12 a CU, ran 1.534-1.546 ms against the odd
// pitch's 1.530-1.540: its bank conflicts cost little).  (Build parameters for A/B runs.)
#ifndef PCX_BATCHED_ES_EVEN
#define PCX_BATCHED_ES_EVEN 1
#endif
__host__ __device__ constexpr int compiled_es(int E) { return PCX_BATCHED_ES_EVEN ? E : (E | 1); }
#ifndef PCX_BATCHED_WAVES  // waves per SIMD the compiled packed shapes' VGPR budget is sized for (4: 128 VGPRs)
#define PCX_BATCHED_WAVES 4
#endif

// NT/ET > 0: the round shape is a compile-time constant (the Monte Carlo shapes the
// launcher specialises, e.g. the 50 x 20 of config C3): every loop bound is known, so
// the sequential column/row loops unroll and their LDS reads issue ahead of the
// dependent adds.  NT = ET = 0: any N <= 64, E <= 32 at run time.  Same arithmetic.
template <int NT, int ET, bool CLUS, bool PK>
__global__ void __launch_bounds__(64, (NT > 0 && PK) ? PCX_BATCHED_WAVES : 3) batched_round_kernel(BatchArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int N = NT > 0 ? NT : a.N, E = ET > 0 ? ET : a.E, ES = ET > 0 ? compiled_es(ET) : a.ES;
    const int l = lane_id();
    const int64_t b = blockIdx.x;
    constexpr int NRM = NT > 0 ? NT : 64;  // median scratch rows
    Smem S = carve(smem, N, E, ES, NRM, PK);
    const bool row = l < N, col = l < E;
    const int64_t bo = a.bounds_shared ? 0 : b * E;
    const bool has_bounds = a.scaled != nullptr;

    long long mprof[3] = {0, 0, 0};  // diagnostic: median sort / walk cycles (PCX_STAMPS)
    STAMP(0);
    // ---- load the round -------------------------------------------------
    const double* Rg = a.reports + b * (int64_t)N * E;
    bool scj = false;
    double loj = 0.0, hij = 0.0;
    if (col && has_bounds) {
        scj = a.scaled[bo + l] != 0;
        loj = a.lo[bo + l];
        hij = a.hi[bo + l];
    }
    double raw = row && a.reputation ? a.reputation[b * N + l] : 0.0;
    if constexpr (NT > 0 && ET > 0 && (NT * ET) % 2 == 0) {
        // every 16-byte load of the round in flight at once, then the LDS scatter
        constexpr int TOT2 = NT * ET / 2, NV = (TOT2 + W - 1) / W;
        double2 v[NV];
#pragma unroll
        for (int q = 0; q < NV; q++)
            if (l + W * q < TOT2) v[q] = reinterpret_cast<const double2*>(Rg)[l + W * q];
#pragma unroll
        for (int q = 0; q < NV; q++) {
            const int idx = 2 * (l + W * q);
            if (idx < NT * ET) {
                const int i0 = idx / ET, j0 = idx - i0 * ET;
                const int i1 = (idx + 1) / ET, j1 = idx + 1 - i1 * ET;
                S.F[i0 * ES + j0] = v[q].x;
                S.F[i1 * ES + j1] = v[q].y;
            }
        }
    } else {
        for (int idx = l; idx < N * E; idx += W) {
            const int i = idx / E, j = idx - i * E;
            S.F[i * ES + j] = Rg[idx];
        }
    }
    const uint64_t scaled_mask = ballot(col && scj);

    // ---- a1: reputation (__init__.py:138-146) -----------------------------
    double rep;
    if (a.reputation) {
        const double tot = wave_pw_sum(raw, row);
        rep = raw / tot;
    } else {
        rep = 1.0 / (double)N;
    }
    const double tok = trunc(rep * 1e6);
    if (row) S.rep[l] = rep;
    const double denom = tree_sum(row ? tok : 0.0) - 1.0;  // exact integer sum
    wsync();

    STAMP(1);
    // ---- a2: rescale (:266-269) + NA masks (:278) -------------------------
    // (the next column's value is loaded before this column's stores: a load after a store to
    // the same LDS array would otherwise wait for it)
    double xnext = row ? S.F[l * ES] : 0.0;
    // per-lane counts, 7 bits each: row l's zeros (bits 0-7) and NaNs (8-15), column l's zeros (16-23)
    uint32_t nacnt = 0;
    for (int j = 0; j < E; j++) {
        const bool sc = (scaled_mask >> j) & 1;
        const double lo = bcast(loj, j), hi = bcast(hij, j);
        double x = xnext;
        if (j + 1 < E) xnext = row ? S.F[l * ES + j + 1] : 0.0;
        if (row) {
            if (sc) {
                x = (x - lo) / (hi - lo);
                if (a.int_dtype) x = trunc(x);
                S.F[l * ES + j] = x;
            }
        }
        const uint64_t nm = ballot(row && __builtin_isnan(x));
        const uint64_t zm = ballot(row && x == 0.0);
        nacnt += (uint32_t)((zm >> l) & 1) + ((uint32_t)((nm >> l) & 1) << 8) + (l == j ? (uint32_t)popc(zm) << 16 : 0u);
        if (l == 0) S.miss[j] = nm | zm;
    }
    wsync();
    // result["original"] (the rescaled reports), from LDS in row-major order: every store
    // instruction writes 64 consecutive doubles (whole lines), not one column's 50 strided ones
    if (a.original) round_to_global(a.original + b * (int64_t)N * E, S.F, N, E, ES, NT, ET);

    STAMP(2);
    // ---- a3: interpolation guesses (:284-313), column phase ----------------
    uint64_t miss_j = 0;
    if (col) miss_j = S.miss[l];
    constexpr int RKW = (ET > 0 ? ET + 3 : EMAX) / 4;  // interpolation-median ranks, a byte per column
    uint32_t rkq[RKW];
#pragma unroll
    for (int k = 0; k < RKW; k++) rkq[k] = 0;
    uint32_t rk_valid = 0;
    {
        // tot: the SPEC's sequential sum of the present reputations (a missing row adds
        // +0.0, which leaves a sum that starts at +0.0 unchanged).  A binary column's
        // guess only matters through catch(): the sum of (rep/tot)*F is formed cheaply as
        // (sum rep*F)/tot, and the SPEC's exact sequential sum is replayed only for a
        // column whose cheap value lies within 1e-12 * sum|rep*F|/tot of a catch threshold
        // (the two differ by at most ~2*(N+2) ulp of that magnitude), so the caught value
        // is the SPEC's bit for bit.  Scaled columns only need tot here (the median).
        constexpr int NR = NT > 0 ? NT : 64;
        double tot = 0.0, sp = 0.0, sa = 0.0;
#pragma unroll 10
        for (int i = 0; i < NR; i++) {
            if (i < N) {
                const bool miss = (miss_j >> i) & 1;
                const double re = miss ? 0.0 : S.rep[i];
                const double f = miss ? 0.0 : S.F[i * ES + (col ? l : 0)];
                tot = tot + re;
                sp = fma(re, f, sp);
                sa = fma(fabs(re), fabs(f), sa);
            }
        }
        const double t_lo = 1.5 - a.catch_tol, t_hi = 1.5 + a.catch_tol;  // catch_() thresholds
        const double accf = sp / tot, margin = 1e-12 * (sa / tot);
        const bool binary_fill = col && miss_j && !scj;
        const bool fast = tot > 0.0 && __builtin_isfinite(accf) && __builtin_isfinite(margin) &&
                          fabs(accf - t_lo) > margin && fabs(accf - t_hi) > margin;
        double acc = accf;
        if (ballot(binary_fill && !fast)) {
            double ex = 0.0;  // SPEC: sum of (rep/tot)*F over the present rows, in row order
#pragma unroll
            for (int i = 0; i < NR; i++) {
                if (i < N) {
                    const double t = (S.rep[i] / tot) * S.F[i * ES + (col ? l : 0)];
                    ex = ((miss_j >> i) & 1) ? ex : ex + t;
                }
            }
            if (!fast) acc = ex;
        }
        if (binary_fill) {
            double g = catch_(acc, a.catch_tol);
            if (a.int_dtype) g = trunc(g);
            S.guess[l] = g;
        }
        if (col && miss_j) S.tot[l] = tot;  // the present-reputation total, for the median phase
    }
    wsync();
    STAMP(13);
    // scaled columns with missing reports: weighted median of the present values
    {
        uint64_t todo = ballot(col && scj && miss_j != 0);
        // the (x, w) pairs of interpolation median j: present reports, rep / tot (:292-303);
        // Wsum = weightedstats' sum(weights), sequential in row order (absent rows add +0.0,
        // which leaves a sum from +0.0 unchanged)
        auto pair_of = [&](int j, double& x, double& w, bool& present, double& Wsum) {
            const uint64_t mj = S.miss[j];
            present = row && !((mj >> l) & 1);
            const double tot = S.tot[j];
            x = row ? S.F[l * ES + j] : 0.0;
            w = present ? S.rep[l] / tot : 0.0;
            Wsum = 0.0;  // (formed inside the median only where a decision needs it: wlazy)
        };
        auto finish = [&](int j, double g) {
            if (a.int_dtype) g = trunc(g);
            if (l == 0) S.guess[j] = g;
        };
        // one median at a time: the scratch lives in M, dead until the covariance.  Each lane's
        // rank among the present keys is kept (one byte per column) for the outcome median of the
        // same column, whose keys are these plus the fill's (a8 below: no second rank loop)
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            double x0, w0, W0;
            bool p0;
            pair_of(j, x0, w0, p0, W0);
            int rk = -1;
            finish(j, wave_wmedian_rank<(NT > 0 ? NT : 64)>(x0, w0, p0, W0, N, S.M, a.stamps ? mprof : nullptr,
                                                            false, 0, &rk, true));
            if (ballot(rk >= 0)) {  // the rank loop ran (no dominant weight, no NaN)
                rk_valid |= 1u << j;
                const int sh = 8 * (j & 3);
                rkq[j >> 2] = (rkq[j >> 2] & ~(0xffu << sh)) | ((uint32_t)(rk & 0xff) << sh);
            }
            wsync();
        }
    }
    wsync();
    STAMP(14);
    // fill (row phase; the next column's masks and fill loaded ahead of this column's store)
    if (row) {
        uint64_t mn = S.miss[0];
        double gn = S.guess[0];
        for (int j = 0; j < E; j++) {
            const uint64_t mj = mn;
            const double g = gn;
            if (j + 1 < E) {
                mn = S.miss[j + 1];
                gn = S.guess[j + 1];
            }
            if ((mj >> l) & 1) S.F[l * ES + j] = g;
        }
    }
    wsync();
    if (a.filled) round_to_global(a.filled + b * (int64_t)N * E, S.F, N, E, ES, NT, ET);

    STAMP(3);
    // ---- old = rep . F (np.dot) -------------------------------------------
    double oldj = col ? ob_vecmat(S.rep, S.F + l, ES, N, E, l) : 0.0;  // np.dot(rep, F) (:490)

    double sc_i = 0.0, nc_i = 0.0, ld_j = 0.0;
    int branch = 5, flags = 0, iters = 0, comps = -1;
    const int alg = a.algorithm;
    const bool clus = CLUS && alg >= 5;  // k-means / hierarchical / clusterfeck call wpca too (:393, :408, :422)
    if (alg == 0 || alg == 2 || alg == 3 || clus) {  // wpca (:315-339): PCA, big-five, fixed-variance
        // ---- a5: weighted mean, np.ma.average (:317-319) -------------------
        const double den = wave_pw_sum(rep, row);
        double muj = 0.0;
        if (E == 1) {
            const double p = row ? S.F[l * ES] * rep : 0.0;
            const double acc = wave_pw_sum(p, row);
            muj = acc / den;
        } else if (col) {
            double acc = S.F[l] * S.rep[0];
            for (int i = 1; i < N; i++) acc = acc + S.F[i * ES + l] * S.rep[i];
            muj = acc / den;
        }
        if constexpr (!PK) {  // (the clusterings and big-five read it from LDS)
            wsync();
            if (col) S.mu[l] = muj;
            wsync();
        }

        STAMP(4);
        // ---- a6: token-weighted covariance (:326), lower triangle ----------
        // fp64 MFMA, lower tiles of the 2 x 2 grid: entry (j, k), j >= k, accumulates
        // fma((F_ij - mu_j) * tok_i, F_ik - mu_k, acc) over i ascending -- the SPEC's
        // chain bit for bit (rows past N and events past E are exact zero padding)
        bool nonzero = false, finite = true;
        {
            constexpr int NR = NT > 0 ? NT : 64;
            const int ml = l & 15, kq = l >> 4;
            const bool two = E > 16;
            const double m0 = __shfl(muj, ml), m1 = __shfl(muj, 16 + ml);  // column ml's / 16 + ml's mean
            const double mu0 = ml < E ? m0 : 0.0, mu1 = 16 + ml < E ? m1 : 0.0;
            d4v c00 = {0, 0, 0, 0}, c10 = {0, 0, 0, 0}, c11 = {0, 0, 0, 0};
#pragma unroll
            for (int i0 = 0; i0 < NR; i0 += 4) {
                if (i0 < N) {
                    const int i = i0 + kq;
                    const bool ok = i < N;
                    const double tk = ok ? trunc(S.rep[i] * 1e6) : 0.0;  // the integer tokens (a1)
                    const bool v0 = ok && ml < E, v1 = ok && 16 + ml < E;
                    const double d0 = v0 ? S.F[i * ES + ml] - mu0 : 0.0;
                    const double d1 = v1 ? S.F[i * ES + 16 + ml] - mu1 : 0.0;
                    const double a0 = v0 ? d0 * tk : 0.0, a1 = v1 ? d1 * tk : 0.0;
                    c00 = mfma_f64(a0, d0, c00);
                    if (two) {
                        c10 = mfma_f64(a1, d0, c10);
                        c11 = mfma_f64(a1, d1, c11);
                    }
                }
            }
            auto put = [&](int j, int k, double acc) {  // j >= k
                const double c = acc / denom;
                S.C[sym_at<PK>(j, k, ES)] = c;
                S.M[sym_at<PK>(j, k, ES)] = c;
                if (!PK) {
                    S.C[k * ES + j] = c;
                    S.M[k * ES + j] = c;
                }
                nonzero |= c != 0.0;
                finite &= __builtin_isfinite(c) != 0;
            };
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int j0 = kq + 4 * r, j1 = 16 + kq + 4 * r, k0 = ml, k1 = 16 + ml;
                if (j0 < E && k0 <= j0) put(j0, k0, c00[r]);
                if (j1 < E && k0 < E) put(j1, k0, c10[r]);
                if (j1 < E && k1 <= j1) put(j1, k1, c11[r]);
            }
        }
        const bool any_nz = ballot(nonzero) != 0;
        const bool all_fin = ballot(!finite) == 0;
        wsync();

        STAMP(5);
        // ---- a7: leading eigenvector by power iteration (:330-336) -------
        double xv = 0.0;
        if (!all_fin) {
            xv = col ? 1.0 : 0.0;
            flags |= 2;
        } else if (!any_nz) {
            xv = l == 0 ? 1.0 : 0.0;
            flags |= 1;
        } else {
            // start: the column with the largest diagonal entry (first max; C is finite here)
            const double dg = col ? S.C[sym_at<PK>(l, l, ES)] : -__builtin_inf();
            const int kd = __builtin_ctzll(ballot(col && dg == wave_max(dg)));
            double x0 = col ? S.C[sym_at<PK>(l, kd, ES)] : 0.0;
            const double n0 = sqrt(tree_sum(x0 * x0));
            xv = col ? x0 / n0 : 0.0;
            int sqn = 0;
            for (; sqn < PI_PRESQUARE; sqn++) square_scaled<PK>(S.M, ES, E);
            int it = 0, since = 0;
            for (;;) {
                const double y = matvec_unit<PK>(S.M, ES, xv, E);
                const double d = wave_max(col ? fabs(y - xv) : 0.0);
                xv = y;
                it++;
                since++;
                if (d <= PI_TOL) break;
                if (it >= PI_MAXIT) {
                    flags |= 4;
                    break;
                }
                if (since >= PI_SQUARE_EVERY && sqn < PI_MAX_SQUARINGS) {
                    square_scaled<PK>(S.M, ES, E);
                    sqn++;
                    since = 0;
                }
            }
            for (int p = 0; p < PI_POLISH; p++) xv = matvec_unit<PK>(S.C, ES, xv, E);
            // SPEC sign: first nonzero component negative; a unit vector e_k is +e_k
            const uint64_t nzm = ballot(col && xv != 0.0);
            if (nzm) {
                const double xf = bcast(xv, __builtin_ctzll(nzm));
                const bool neg = popc(nzm) == 1 ? xf < 0.0 : xf > 0.0;
                if (neg) xv = -xv;
            }
            iters = it + PI_POLISH + sqn;
        }
        // loading = v / sqrt(sum(v**2)) with numpy's pairwise sum (:336)
        const double nv = sqrt(wave_pw_sum(xv * xv, col));
        ld_j = col ? xv / nv : 0.0;
        wsync();
        if (clus) {
            // the loading only: scores stay zeros (:357)
        } else if (alg == 0) {
            // scores s = wcd . loading (:337), row phase (column j's mean and loading from lane j)
            const int r = row ? l : 0;
            double acc = 0.0;
            for (int j = 0; j < E; j++) acc = fma(S.F[r * ES + j] - lane_value(muj, j), lane_value(ld_j, j), acc);
            if (row) sc_i = acc;
        } else if (flags & 2) {
            sc_i = __builtin_nan("");  // the reference's second svd raises (:375, :431)
        } else if constexpr (!PK) {  // (the packed layout is never launched for these)
            // ---- big-five (:373-390) / fixed-variance (:429-451): net score =
            // sum_c Sigma_c * (wcd . loading_c); Sigma, loadings from Jacobi (SPEC)
            const double trace = wave_pw_sum(col ? S.C[l * ES + l] : 0.0, col);  // np.trace
            wsync();
            for (int o = l; o < E * E; o += W) {
                const int j = o / E, k = o - j * E;
                S.M[j * ES + k] = S.C[j * ES + k];
            }
            wsync();
            jacobi_eig_wave(S.M, S.C, ES, E, S.x, S.ld);  // A in M; V overwrites C; x, ld are dead
            const double sig = col ? fabs(S.M[l * ES + l]) : 0.0;
            if (col) S.nv1[l] = sig;
            wsync();
            if (col) {  // order: descending Sigma, ties by index
                int rk = 0;
                for (int k = 0; k < E; k++) rk += (S.nv1[k] > sig) | ((S.nv1[k] == sig) & (k < l));
                S.nv2[rk] = (double)l;
            }
            wsync();
            const int kmax = alg == 2 ? a.max_components : E;
            double net = 0.0, ve = 0.0;
            int used = kmax;
            for (int c = 0; c < kmax; c++) {
                const int idx = (int)S.nv2[c];
                const double sg = S.nv1[idx];
                const double fl = S.C[idx] < 0.0 ? -1.0 : 1.0;  // loading *= -1 if loading[0] < 0
                if (row) {
                    double d = 0.0;
                    for (int j = 0; j < E; j++) d = fma(S.F[l * ES + j] - S.mu[j], fl * S.C[j * ES + idx], d);
                    net = net + sg * d;
                }
                if (alg == 3) {  // cumsum(Sigma / trace) >= threshold -> stop (:432, :448)
                    ve = ve + sg / trace;
                    if (ve >= a.variance_threshold) {
                        used = c + 1;
                        break;
                    }
                }
            }
            comps = alg == 3 ? used : -1;
            sc_i = net;
            wsync();
        }
    } else if (alg == 4) {  // cokurtosis: caller-supplied scores (:455-457)
        sc_i = row ? a.aux_scores[b * N + l] : 0.0;
    }
    STAMP(6);
    if constexpr (CLUS) {
        if (clus) {
            double* X = smem + smem_doubles(N, E, ES, NRM, PK);
            if (alg == 6)
                nc_i = hier_nc(S.F, S.mu, ES, N, E, a.hierarchy_threshold, reinterpret_cast<uint64_t*>(X));
            else if (alg == 5)
                nc_i = kmeans_nc(a, b, S.F, S.mu, ES, N, E, X);
            else
                nc_i = feck_nc(a, S.F, ES, N, E, rep, X);
            wsync();
        }
    }
    if (alg != 1 && !clus) {
        // ---- a8/a9: nonconformity_rank (:487-500) / nonconformity (:475-485); the
        // non-PCA algorithms call nonconformity directly (:389, :450, :456)
        const bool any_nan = ballot(row && __builtin_isnan(sc_i)) != 0;
        double mn = wave_max(row ? -sc_i : -__builtin_inf());
        mn = -mn;
        double mx = wave_max(row ? sc_i : -__builtin_inf());
        if (any_nan) {
            mn = __builtin_nan("");
            mx = __builtin_nan("");
        }
        const double set1 = sc_i + fabs(mn);
        const double set2 = sc_i - mx;
        double a1 = fabs(set1), a2 = fabs(set2);
        double S1 = wave_pw_sum(a1, row);
        if (S1 == 0) {
            a1 += 1.0;
            S1 = wave_pw_sum(a1, row);
        }
        double S2 = wave_pw_sum(a2, row);
        if (S2 == 0) {
            a2 += 1.0;
            S2 = wave_pw_sum(a2, row);
        }
        if (row) {
            S.n1[l] = a1 / S1;
            S.n2[l] = a2 / S2;
        }
        if (col) S.old[l] = oldj;
        wsync();
        double d1 = 0.0, d2 = 0.0;
        if (col) {
            d1 = ob_vecmat(S.n1, S.F + l, ES, N, E, l);  // np.dot(normalize(set1), F) (:492)
            d2 = ob_vecmat(S.n2, S.F + l, ES, N, E, l);
            const double t = 0.01 * oldj;
            S.nv1[l] = d1 + t;
            S.nv2[l] = d2 + t;
        }
        wsync();
        double ref = 0.0;  // non-PCA: straight to the continuous rule
        if (alg == 0) {
            const double r0 = rank_avg(S.old, E);
            const double r1 = rank_avg(S.nv1, E);
            const double r2 = rank_avg(S.nv2, E);
            const double e1 = fabs(r1 - r0), e2 = fabs(r2 - r0);
            ref = wave_pw_sum(e1, col) - wave_pw_sum(e2, col);
        }
        bool pick1;
        if (ref == 0) {
            const double q1 = d1 - oldj, q2 = d2 - oldj;
            const double ref2 = wave_pw_sum(q1 * q1, col) - wave_pw_sum(q2 * q2, col);
            pick1 = ref2 <= 0;
            branch = pick1 ? 3 : 4;
        } else {
            pick1 = ref < 0;
            branch = pick1 ? 1 : 2;
        }
        nc_i = pick1 ? set1 : set2;
    }

    STAMP(7);
    // ---- a10: reputation update (:460-472) --------------------------------
    const double meanrep = wave_pw_sum(rep, row) / (double)N;
    double u = fabs(nc_i * (rep / meanrep));
    double Su = wave_pw_sum(u, row);
    // PCA: a NaN total leaves the reference's this_rep / smooth_rep fully MASKED (SPEC
    // rep_masked: participation_columns, reporter_bonus and author_bonus are numpy.ma's data)
    const bool rep_masked = alg == 0 && __builtin_isnan(Su);
    if (Su == 0) {
        u += 1.0;
        Su = wave_pw_sum(u, row);
    }
    const double this_i = u / Su;
    const double smooth_i = a.alpha * this_i + (1.0 - a.alpha) * rep;
    wsync();
    if (row) S.smooth[l] = smooth_i;
    wsync();

    STAMP(8);
    // ---- a12/a13: outcomes (:510-538) -------------------------------------
    double rawj = col ? ob_vecmat(S.smooth, S.F + l, ES, N, E, l) : 0.0;  // np.dot(smooth_rep, F) (:510)
    STAMP(15);
    if (scaled_mask) {
        const double Wsm = [&] {  // builtin sequential sum of smooth_rep (weightedstats)
            double w = 0.0;
            if (l == 0)
                for (int i = 0; i < N; i++) w += S.smooth[i];
            return bcast(w, 0);
        }();
        uint64_t todo = scaled_mask;
        while (todo) {  // scratch in M, dead after the scores
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const double x0 = row ? S.F[l * ES + j] : 0.0;
            // the filled column's keys are the interpolation median's (present rows) plus the
            // fill's (missing rows, all equal): a present row's count of smaller keys is its
            // recorded one plus the missing rows when the fill's key is below its own, a missing
            // row's is the present keys below the fill's -- the same counts the loop would make
            const bool reuse = (rk_valid >> j) & 1;
            int rk = 0;
            if (reuse) {
                const uint64_t mj = S.miss[j];
                const bool ms = (mj >> l) & 1;
                const uint32_t key = key_hi32(x0);
                const uint32_t kg = (uint32_t)__builtin_amdgcn_readlane((int)key, __builtin_ctzll(mj));
                const int below = popc(ballot(row && !ms && key < kg));
                const int own = (int)((rkq[j >> 2] >> (8 * (j & 3))) & 0xffu);
                rk = ms ? below : own + (kg < key ? popc(mj) : 0);
            }
            const double m = wave_wmedian_rank<(NT > 0 ? NT : 64)>(x0, smooth_i, row, Wsm, N, S.M,
                                                                   a.stamps ? mprof : nullptr, reuse, rk);
            if (l == j) rawj = m;
            wsync();
        }
    }
    STAMP(16);
    double adjj = 0.0, finj = 0.0;
    if (col) {
        if (scj) {
            adjj = rawj;
            finj = adjj * (hij - loj);
            finj = finj + loj;
        } else {
            adjj = catch_(rawj, a.catch_tol);
            finj = adjj;
        }
        S.adj[l] = adjj;
    }
    wsync();

    STAMP(9);
    // ---- a14: certainty (:540-546): pairwise sum of the matching smooth_rep --
    // every column at once, one lane per column: the hit masks first (F is read for the
    // last time), then each row lane scatters its smooth_rep into the compacted hit list of
    // every column it matches (into F, dead from here on), then lane j runs numpy's pairwise
    // add.reduce (n <= 128: eight strided accumulators, fixed tree, sequential tail) on
    // its column's list
    double certj = 0.0;
    {
        uint64_t* hitm = reinterpret_cast<uint64_t*>(S.M);  // [E]; M is dead after the medians
        double fn = row ? S.F[l * ES] : 0.0, an = S.adj[0];  // (next column's loads ahead of this column's store)
        for (int j = 0; j < E; j++) {
            const double f = fn, av = an;
            if (j + 1 < E) {
                fn = row ? S.F[l * ES + j + 1] : 0.0;
                an = S.adj[j + 1];
            }
            const uint64_t hm = ballot(row && f == av);
            if (l == 0) hitm[j] = hm;
        }
        wsync();
        const int NS = cert_stride(N, ES);  // odd stride: lane-per-column reads spread over the banks
        double* comp = S.F;    // [E][NS]
        for (int j = 0; j < E; j++) {
            const uint64_t hm = hitm[j];
            if ((hm >> l) & 1) comp[j * NS + mbcnt64(hm)] = smooth_i;
        }
        wsync();
        if (col) {
            constexpr int TMAX = (NT > 0 ? NT : 64) / 8;
            const uint64_t hm = hitm[l];
            const int n = popc(hm), T = n >> 3;
            const double* c = comp + l * NS;
            double res = 0.0;
            if (T) {
                double r[8];
#pragma unroll
                for (int k = 0; k < 8; k++) r[k] = c[k];
#pragma unroll
                for (int t = 1; t < TMAX; t++)
                    if (t < T) {
#pragma unroll
                        for (int k = 0; k < 8; k++) r[k] = r[k] + c[8 * t + k];
                    }
                res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
            }
            for (int q = 8 * T; q < n; q++) res = res + c[q];  // the tail (everything when n < 8)
            certj = n ? res : (a.algorithm == 0 ? __builtin_nan("") : 0.0);
        }
    }
    // normalize(certainty), mean(certainty)
    double ac = fabs(certj);
    double Sc = wave_pw_sum(ac, col);
    if (Sc == 0) {
        ac += 1.0;
        Sc = wave_pw_sum(ac, col);
    }
    const double reward = ac / Sc;
    const double avg_cert = wave_pw_sum(certj, col) / (double)E;

    STAMP(10);
    // ---- a15: participation and bonuses (:549-581) -------------------------
    double pcj = 0.0, nzj = 0.0;
    // every smooth_rep finite: a row with na = 0 adds p = x * 0 = +-0 and pe = +-0, which leave
    // (s, c) bit for bit as they were (neither is ever -0.0), so only the missing rows are visited
    const bool smooth_finite = !ballot(row && !__builtin_isfinite(smooth_i));
    if (col) {
        const uint64_t nam = S.miss[l];
        // dot2(smooth, na) with na in {0,1}
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
        if (smooth_finite) {
            for (uint64_t mm = nam; mm; mm &= mm - 1) step(S.smooth[__builtin_ctzll(mm)], 1.0);
        } else {
            for (int i = 0; i < N; i++) step(S.smooth[i], ((nam >> i) & 1) ? 1.0 : 0.0);
        }
        pcj = 1.0 - (s + c);
        nzj = (double)((nacnt >> 16) & 0xffu);
    }
    double narow = 0.0;
    int nnan = 0;
    if (row) {
        narow = (double)(nacnt & 0xffu);
        nnan = (int)((nacnt >> 8) & 0xffu);
    }
    const bool rowmasked = row && nnan == E;
    const double pr = 1.0 - narow / (double)E;
    const double pna = 1.0 - wave_pw_sum(pcj, col) / (double)E;
    double ar = rowmasked ? 0.0 : fabs(pr);
    double Sr = wave_pw_sum(ar, row);
    if (Sr == 0) {
        ar = rowmasked ? 0.0 : fabs(pr) + 1.0;
        Sr = wave_pw_sum(ar, row);
    }
    const double rel = rowmasked ? fabs(pr) : ar / Sr;
    double apc = fabs(pcj);
    double Spc = wave_pw_sum(apc, col);
    if (Spc == 0) {
        apc += 1.0;
        Spc = wave_pw_sum(apc, col);
    }
    const double relc = apc / Spc;

    STAMP(11);
    // ---- write the round ---------------------------------------------------
    if (row) {
        const int64_t o = b * N + l;
        if (a.old_rep) a.old_rep[o] = rep;
        if (a.this_rep) a.this_rep[o] = this_i;
        if (a.smooth_rep) a.smooth_rep[o] = smooth_i;
        if (a.scores) a.scores[o] = sc_i;
        if (a.na_row) a.na_row[o] = narow;
        if (a.participation_rows) a.participation_rows[o] = pr;
        if (a.relative_part) a.relative_part[o] = rel;
        if (a.reporter_bonus) a.reporter_bonus[o] = (rowmasked || rep_masked) ? rel : rel * pna + smooth_i * (1.0 - pna);
    }
    if (col) {
        const int64_t o = b * E + l;
        if (a.adj_first_loadings) a.adj_first_loadings[o] = ld_j;
        if (a.outcomes_raw) a.outcomes_raw[o] = rawj;
        if (a.outcomes_adjusted) a.outcomes_adjusted[o] = adjj;
        if (a.outcomes_final) a.outcomes_final[o] = finj;
        if (a.certainty) a.certainty[o] = certj;
        if (a.consensus_reward) a.consensus_reward[o] = reward;
        if (a.nas_filled) a.nas_filled[o] = nzj;
        if (a.participation_columns) a.participation_columns[o] = rep_masked ? 1.0 : pcj;
        if (a.author_bonus) a.author_bonus[o] = rep_masked ? 1.0 : relc * pna + reward * (1.0 - pna);
    }
    if (l == 0) {
        if (a.participation) a.participation[b] = 1.0 - pna;
        if (a.avg_certainty) a.avg_certainty[b] = avg_cert;
        if (a.branch) a.branch[b] = branch;
        if (a.flags) a.flags[b] = flags;
        if (a.pi_iters) a.pi_iters[b] = iters;
        if (a.components) a.components[b] = comps;
    }
    STAMP(12);
    if (a.stamps && threadIdx.x == 0) {
        a.stamps[b * 32 + 20] = mprof[0];
        a.stamps[b * 32 + 21] = mprof[1];
    }
}

// the launch's instantiation: <50, 20> for the C3 shape, else the dynamic one; packed
// C / M unless the algorithm needs the Jacobi eigenpairs (big-five, fixed-variance) or
// is a clustering one
static bool shape_50x20(int N, int E, int ES) { return N == 50 && E == 20 && ES == 21; }
static bool packed_alg(int alg) { return alg == 0 || alg == 1 || alg == 4; }

size_t batched_lds_bytes(int N, int E, int alg) {
    const bool c50 = shape_50x20(N, E, E | 1) && alg < 5;  // the <50, 20> instantiation
    const int ES = c50 ? compiled_es(E) : E | 1;
    const int NR = c50 ? 50 : 64;
    return smem_doubles(N, E, ES, NR, packed_alg(alg)) * sizeof(double);
}

hipError_t launch_batched(const BatchArgs& a, hipStream_t stream) {
    // PCX_BATCHED_LDS_PAD (diagnostic): extra dynamic LDS bytes per round, to measure
    // throughput against resident rounds per CU (tools/occupancy_batched.py)
    static const size_t pad = [] {
        const char* e = getenv("PCX_BATCHED_LDS_PAD");
        return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)0;
    }();
    size_t lds = batched_lds_bytes(a.N, a.E, a.algorithm) + pad;
    if (a.B <= 0) return hipSuccess;
    const dim3 grid((unsigned)a.B), block(64);
    const bool pk = packed_alg(a.algorithm);
    if (a.algorithm >= 5) {  // clustering algorithms: their own instantiation and LDS region
        lds += sizeof(double) * (size_t)cluster_lds_doubles(a.N, a.E, a.ES);
        static bool attr = [] {
            return hipFuncSetAttribute(reinterpret_cast<const void*>(&batched_round_kernel<0, 0, true, false>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
        }();
        (void)attr;
        hipLaunchKernelGGL((batched_round_kernel<0, 0, true, false>), grid, block, lds, stream, a);
    } else if (shape_50x20(a.N, a.E, a.ES)) {
        if (pk)
            hipLaunchKernelGGL((batched_round_kernel<50, 20, false, true>), grid, block, lds, stream, a);
        else
            hipLaunchKernelGGL((batched_round_kernel<50, 20, false, false>), grid, block, lds, stream, a);
    } else if (pk) {
        hipLaunchKernelGGL((batched_round_kernel<0, 0, false, true>), grid, block, lds, stream, a);
    } else {
        hipLaunchKernelGGL((batched_round_kernel<0, 0, false, false>), grid, block, lds, stream, a);
    }
    return hipGetLastError();
}

}  // namespace pcx
