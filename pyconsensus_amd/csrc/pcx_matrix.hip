// pcx_matrix.hip -- the single-matrix consensus path on MI355X (gfx950).
//
// One N x E report matrix (row-major fp64, NaN = missing), optionally sharded by
// reporter rows over several GPUs.  The stages of pcx_mat_stage() (include/pcx.h)
// restate pyconsensus Oracle.consensus(), algorithm="PCA"
// (pyconsensus/__init__.py:102-611):
//
//   * every pass over the matrix recomputes the element transform on the fly
//     (rescale of scaled events :266-269, NA test :278, fill :310-312, centring
//     :322) instead of materialising rescaled / filled / centred copies;
//   * column sums (np.dot(v, F) and the interpolation sums) are compensated
//     (double-double) so they are within an ulp of exact -- the reference's own
//     order is OpenBLAS-internal or a sequential Python loop;
//   * the covariance wcd^T diag(tokens) wcd (:326) runs on fp64 MFMA
//     (v_mfma_f64_16x16x4_f64) with LDS-staged 128x128 tiles, split-K over rows;
//   * the leading eigenvector (svd, :330) comes from power iteration;
//   * weighted medians (weightedstats, :303, :520) are exact weighted selections
//     over an order-preserving integer key of the values, with weights summed as
//     exact fixed-point limbs (order-independent, identical on any GPU count).
//
// Per-rank partial results are written into slot [rank] of [world][...] buffers;
// the host all-reduces (SUM) them between stages and the next stage combines the
// ranks in rank order, so results do not depend on the communication algorithm.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <initializer_list>
#include <cmath>
#include <map>
#include <mutex>
#include <numeric>
#include <vector>

#include "../../include/pcx.h"
#include "pcx_device.h"
#include "pcx_gemm_i8.h"
#include "pcx_internal.h"
#include "pcx_seqsum.h"

namespace pcx {
namespace {

constexpr int CS = 16;           // dd slots per column in cstat
constexpr int SS = 16;           // dd slots in scal
constexpr int NB = SEL_NB;       // selection buckets
// rows per load batch of the weight-mode column passes, and the minimum waves per SIMD their
// registers are held to (build parameters for A/B runs).  Measured at C5 (round 6, the phase-2
// first pass): 8 rows, 107 VGPRs, 3.85-3.98 ms; 12 rows (139 VGPRs, 3 waves) 7.44 ms; 16 rows
// (171 VGPRs, 2 waves) 7.77 ms, or held to 4 waves (58 VGPRs spilled) 7.65 ms.
#ifndef PCX_SEL_WUNROLL
#define PCX_SEL_WUNROLL 8
#endif
constexpr int SEL_WUNROLL = PCX_SEL_WUNROLL;
#ifndef PCX_SEL_WWAVES
#define PCX_SEL_WWAVES 1
#endif
constexpr int SEL_HC = 2;  // copies of each k_sel_hist bucket (4: 12.3 vs 9.0 ms at C5; 1: 9.37 vs 8.66 ms, round 5)
constexpr int SELS = 40;         // sel_state words per scaled event
constexpr int BT = 256;          // threads per block for row/column passes
constexpr int CM = 8;            // doubles per column in mpart / cmax

enum ev_slot { EV_GUESS = 0, EV_MU, EV_OLD, EV_LD, EV_D1, EV_D2, EV_RAW, EV_ADJ, EV_FIN, EV_CERT, EV_PC,
               EV_MINX, EV_MAXX, EV_MISS, EV_NZERO, EV_SPARE, EV_LDP, EV_K, EV_MUP };  // (pcx_runner.cpp: EV_SLOTS)
enum row_slot { RV_S = 0, RV_U, RV_THIS, RV_SMOOTH, RV_N1, RV_N2 };
enum scal_slot { SC_TOK = 0, SC_REP, SC_A1, SC_A1P, SC_A2, SC_A2P, SC_U, SC_UP, SC_AR, SC_ARP, SC_BIGTOK, SC_MAXTOK };
enum info_slot { IN_BRANCH = 0, IN_PI_ITERS, IN_FLAGS, IN_SEL_ACTIVE, IN_SEL_ARGMAX, IN_PICK1, IN_HARD, IN_SEL_WACTIVE,
                 IN_COV_GENERAL, IN_COV_MIXED, IN_COV_TOK1, IN_SEL_WLIMB, IN_COV_GUARD, IN_COV_GUARD_COLS,
                 IN_COV_GUARD_BOUND };  // (word 15: M_POWER's squaring scratch)
static_assert((int)IN_COV_GUARD == (int)INFO_COV_GUARD && (int)IN_COV_GUARD_COLS == (int)INFO_COV_GUARD_COLS &&
                  (int)IN_COV_GUARD_BOUND == (int)INFO_COV_GUARD_BOUND,
              "info slots");

// ------------------------------------------------------------------ element transform
struct ColParam {
    bool scaled;
    double lo, range, guess, mu;
    double rr;  // RN(1 / range); NaN when range lies outside [2^-100, 2^100] (quotients then divide)
};

// d / b correctly rounded from y = RN(1 / b) (Markstein: q0 = RN(d y) is faithful, the residual
// d - b q0 is exact in one fma, and RN(q0 + r y) = RN(d / b)), in 4 fp64 ops where the IEEE
// division sequence (div_scale x2, rcp, 5 fma, div_fmas, div_fixup) takes 11 with a quarter-rate
// rcp.  The theorem assumes no underflow or overflow: with |b| in [2^-100, 2^100] (else y is
// NaN) and |q0| in [2^-860, 2^1000], |d| >= 2^-960 keeps the residual exact and q finite.  Other
// cells -- zeros among them, whose sign the fast path can get wrong (-0 / b) -- divide (a branch,
// skipped when no lane needs it).  NaN d passes: the fast path returns NaN as the division does.
// tests/test_fastdiv.py checks the sequence and its guard against the division bit for bit.
__device__ __forceinline__ double div_rn(double d, double b, double y) {
    const double q0 = d * y;
    const double r = __builtin_fma(-q0, b, d);
    double q = __builtin_fma(r, y, q0);
    const bool slow = __builtin_isnan(y) | (fabs(q0) < 0x1p-860) | (fabs(q0) > 0x1p1000);
    if (__builtin_expect(slow, 0)) q = d / b;
    return q;
}

__device__ __forceinline__ double range_rcp(double range) {
    const double a = fabs(range);
    return (a >= 0x1p-100 && a <= 0x1p100) ? 1.0 / range : __builtin_nan("");
}

__device__ __forceinline__ double rescale(double r, const ColParam& p, int int_dtype) {
    if (!p.scaled) return r;
    double x = div_rn(r - p.lo, p.range, p.rr);
    if (int_dtype) x = trunc(x);
    return x;
}

__device__ __forceinline__ bool missing(double x) { return __builtin_isnan(x) || x == 0.0; }

__device__ __forceinline__ ColParam col_param(const pcx_mat& m, int c, bool with_fill) {
    ColParam p;
    p.scaled = m.scaled && m.scaled[c] && !m.rescaled;  // (in place already: the identity)
    p.lo = p.scaled ? m.lo[c] : 0.0;
    p.range = p.scaled ? (m.hi[c] - m.lo[c]) : 1.0;
    p.guess = with_fill ? m.ev[EV_GUESS * m.n_events + c] : 0.0;
    p.mu = with_fill ? m.ev[EV_MU * m.n_events + c] : 0.0;
    p.rr = p.scaled ? range_rcp(p.range) : 1.0;
    return p;
}

// filled value F_ic (:310-312)
__device__ __forceinline__ double filled(double r, const ColParam& p, int int_dtype) {
    const double x = rescale(r, p, int_dtype);
    return missing(x) ? p.guess : x;
}

// ------------------------------------------------------------------ the reference's own order
// For one rank with N*E < 9216 the reference's np.dot runs single-threaded OpenBLAS dgemv and
// its np.sum numpy's pairwise sum; m.ob_order replays both (oracle/pcx_oracle_batched.c
// ob_vecmat / pw_sum, fitted bit for bit on the goldens' host), so rank ties that rounding
// makes or breaks (e.g. np.dot(rep, F) of two events with equal counts under uniform weights,
// :489-490) fall as in the reference.  One thread runs each whole sum (N*E < 9216: short).

// numpy pairwise_sum: blocks of <= 128 with 8 accumulators, halves rounded to multiples of 8
template <class G>
__device__ double pw_leaf(G g, int64_t off, int64_t n) {
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; i++) r += g(off + i);
        return r;
    }
    double r[8];
    for (int k = 0; k < 8; k++) r[k] = g(off + k);
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int k = 0; k < 8; k++) r[k] += g(off + i + k);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += g(off + i);
    return res;
}

template <class G>
__device__ double pw_sum_dev(G g, int64_t n) {  // the recursion of pw_sum, as an explicit stack
    int64_t off_[32], n_[32];
    double left_[32];
    int state_[32];  // 0 = fresh, 1 = left half pending, 2 = right half pending
    int sp = 0;
    off_[0] = 0;
    n_[0] = n;
    state_[0] = 0;
    for (;;) {
        double ret;
        if (n_[sp] > 128) {  // split: evaluate the left half first
            int64_t n2 = n_[sp] / 2;
            n2 -= n2 % 8;
            state_[sp] = 1;
            off_[sp + 1] = off_[sp];
            n_[sp + 1] = n2;
            state_[sp + 1] = 0;
            sp++;
            continue;
        }
        ret = pw_leaf(g, off_[sp], n_[sp]);
        for (;;) {  // hand ret to the parent frames
            if (sp == 0) return ret;
            sp--;
            if (state_[sp] == 1) {
                int64_t n2 = n_[sp] / 2;
                n2 -= n2 % 8;
                left_[sp] = ret;
                state_[sp] = 2;
                off_[sp + 1] = off_[sp] + n2;
                n_[sp + 1] = n_[sp] - n2;
                state_[sp + 1] = 0;
                sp++;
                break;
            }
            ret = left_[sp] + ret;
        }
    }
}

// numpy's ddot (E == 1): 4 x 8-lane fma accumulators per 32 terms, folded to 4 x 4 lanes,
// 16 per step, lanes (0 + 2) + (1 + 3), then a sequential fma tail
template <class V, class X>
__device__ double ob_ddot(V v, X x, int64_t n) {
    double acc8[4][8], acc4[4][4];
    for (int r = 0; r < 4; r++)
        for (int l = 0; l < 8; l++) acc8[r][l] = 0.0;
    const int64_t n32 = n & ~(int64_t)31, n16 = n & ~(int64_t)15;
    for (int64_t i = 0; i < n32; i += 32)
        for (int k = 0; k < 32; k++) acc8[k / 8][k % 8] = fma(v(i + k), x(i + k), acc8[k / 8][k % 8]);
    for (int r = 0; r < 4; r++)
        for (int l = 0; l < 4; l++) acc4[r][l] = acc8[r][l] + acc8[r][l + 4];
    for (int64_t i = n32; i < n16; i += 16)
        for (int k = 0; k < 16; k++) acc4[k / 4][k % 4] = fma(v(i + k), x(i + k), acc4[k / 4][k % 4]);
    double A[4];
    for (int l = 0; l < 4; l++) A[l] = ((acc4[0][l] + acc4[1][l]) + acc4[2][l]) + acc4[3][l];
    double d = (A[0] + A[2]) + (A[1] + A[3]);
    for (int64_t i = n16; i < n; i++) d = fma(v(i), x(i), d);
    return d;
}

// np.dot(v, F)[j] as cblas_dgemv(RowMajor, Trans) = column-major dgemv_n on the E x N matrix:
// events j < E & ~3 in the 4-row vector kernel (reporters in blocks of 4: the second product
// rounded, fma with the first, third, fourth; y = y + block; tails of 2 and 1), the last E % 4
// events a sequential fma chain (E = 2, 3: unrolled pairs), E = 1 numpy's ddot
template <class V, class X>
__device__ double ob_vecmat(V v, X F, int64_t N, int64_t E, int64_t j) {
    if (E == 1) return ob_ddot(v, F, N);
    if (j < (E & ~(int64_t)3)) {
        double y = 0.0;
        int64_t n = 0;
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
    int64_t i = 0;
    if (E == 2 || E == 3)
        for (; i + 4 <= N; i += 4) {
            t = t + fma(F(i), v(i), F(i + 1) * v(i + 1));
            t = t + fma(F(i + 2), v(i + 2), F(i + 3) * v(i + 3));
        }
    for (; i < N; i++) t = fma(F(i), v(i), t);
    return t;
}

// np.dot(w, F)[c] of the filled column c, weights w[i] (ob_order)
__device__ __forceinline__ double ob_col_dot(const pcx_mat& m, const double* w, int c) {
    const ColParam p = col_param(m, c, true);
    const int64_t E = m.n_events;
    return ob_vecmat([&](int64_t i) { return w[i]; },
                     [&](int64_t i) { return filled(m.reports[i * E + c], p, m.int_dtype); }, m.n_rows, E, c);
}

// ------------------------------------------------------------------ block reductions
template <int NT>
__device__ dd block_sum_dd(dd v, dd* lds) {
    v = wave_sum_dd(v);
    const int w = threadIdx.x / WAVE, l = threadIdx.x % WAVE;
    __syncthreads();
    if (l == 0) lds[w] = v;
    __syncthreads();
    dd r{0.0, 0.0};
    if (threadIdx.x == 0)
        for (int i = 0; i < NT / WAVE; i++) r = dd_add(r, lds[i]);
    __syncthreads();
    return r;  // valid on thread 0
}

__device__ __forceinline__ dd ld_dd(const double* p) { return {p[0], p[1]}; }
__device__ __forceinline__ void st_dd(double* p, dd v) {
    p[0] = v.hi;
    p[1] = v.lo;
}

// sum over ranks (rank order) of a [world][stride] dd buffer at offset
__device__ __forceinline__ dd rank_sum(const double* buf, int world, int64_t stride, int64_t off) {
    dd r{0.0, 0.0};
    for (int w = 0; w < world; w++) r = dd_add(r, ld_dd(buf + w * stride + off));
    return r;
}

// ------------------------------------------------------------------ limbs (exact sums)
struct L3 {
    uint64_t a, b, c;  // value = a*2^-35 + b*2^-78 + c*2^-121
};

__device__ __forceinline__ L3 l3_norm(L3 x) {  // carry so that b, c < 2^43
    const uint64_t M = (1ull << 43) - 1;
    x.b += x.c >> 43;
    x.c &= M;
    x.a += x.b >> 43;
    x.b &= M;
    return x;
}
__device__ __forceinline__ L3 l3_add(L3 x, L3 y) { return l3_norm({x.a + y.a, x.b + y.b, x.c + y.c}); }
__device__ __forceinline__ L3 l3_twice(L3 x) { return l3_norm({x.a * 2, x.b * 2, x.c * 2}); }
__device__ __forceinline__ int l3_cmp(L3 x, L3 y) {  // both normalised
    if (x.a != y.a) return x.a < y.a ? -1 : 1;
    if (x.b != y.b) return x.b < y.b ? -1 : 1;
    if (x.c != y.c) return x.c < y.c ? -1 : 1;
    return 0;
}
__device__ __forceinline__ L3 l3_of(double w) {
    const limbs3 t = to_limbs(w);
    return {t.l0, t.l1, t.l2};
}
__device__ __forceinline__ double l3_to_double(L3 x) {
    return ldexp((double)x.a, -35) + (ldexp((double)x.b, -78) + ldexp((double)x.c, -121));
}

// ================================================================== PCX_M_REPUTATION
__global__ void __launch_bounds__(1024) k_rep_total(pcx_mat m) {
    __shared__ dd lds[16];
    if (m.ob_order) {  // np.sum's own pairwise order
        if (threadIdx.x == 0) m.pvec[0] = pw_sum_dev([&](int64_t i) { return m.rep_raw[i]; }, m.n_total);
        return;
    }
    acc2 a;
    for (int64_t i = threadIdx.x; i < m.n_total; i += blockDim.x) a.add(m.rep_raw[i]);
    dd v = block_sum_dd<1024>(a.get(), lds);
    if (threadIdx.x == 0) {
        m.pvec[0] = dd_to_double(v);  // total reputation (np.sum, :144)
    }
}

__global__ void __launch_bounds__(BT) k_rep_local(pcx_mat m) {
    __shared__ dd lds[8];
    acc2 at, ar;
    double big = 0.0;  // tokens outside [0, 63]: the int8 covariance path needs tok * z <= 126
    double tmax = 0.0;  // the largest token (scales the mixed block's digits of tok w)
    const double tot = m.rep_raw ? m.pvec[0] : 0.0;
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const double r = m.rep_raw ? m.rep_raw[m.row_offset + i] / tot : 1.0 / (double)m.n_total;
        const double t = trunc(r * 1e6);
        m.rep[i] = r;
        m.tok[i] = t;
        at.add(t);
        ar.add(r);
        big += (t >= 0.0 && t <= 63.0) ? 0.0 : 1.0;
        tmax = fmax(tmax, t);
    }
    dd st = block_sum_dd<BT>(at.get(), lds);
    dd sr = block_sum_dd<BT>(ar.get(), lds);
    dd sb = block_sum_dd<BT>(dd{big, 0.0}, lds);
    __shared__ double tm[BT / WAVE];
    for (int o = WAVE / 2; o >= 1; o >>= 1) tmax = fmax(tmax, __shfl_xor(tmax, o, WAVE));
    if (threadIdx.x % WAVE == 0) tm[threadIdx.x / WAVE] = tmax;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < BT / WAVE; k++) tmax = fmax(tmax, tm[k]);
        st_dd(m.spart + blockIdx.x * 8 + 0, st);
        st_dd(m.spart + blockIdx.x * 8 + 2, sr);
        st_dd(m.spart + blockIdx.x * 8 + 4, sb);
        st_dd(m.spart + blockIdx.x * 8 + 6, dd{tmax, 0.0});
    }
}

// the largest block value of spart slot `src` (hi parts) -> scal[rank][slot] (one block)
__global__ void __launch_bounds__(BT) k_spart_max(pcx_mat m, int nblk, int slot, int src) {
    __shared__ double red[BT];
    double v = 0.0;
    for (int b = threadIdx.x; b < nblk; b += BT) v = fmax(v, m.spart[b * 8 + 2 * src]);
    red[threadIdx.x] = v;
    __syncthreads();
    for (int st = BT / 2; st >= 1; st >>= 1) {
        if (threadIdx.x < st) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + st]);
        __syncthreads();
    }
    if (threadIdx.x == 0) st_dd(m.scal + ((int64_t)m.rank * SS + slot) * 2, dd{red[0], 0.0});
}

// reduce spart[nblk][4 dd] slots src0 .. src0+k into scal[rank][slot0 .. slot0+k): one
// block per slot, a fixed strided assignment of the row-pass blocks to threads and a fixed
// dd tree (deterministic)
__global__ void __launch_bounds__(BT) k_spart_finish(pcx_mat m, int nblk, int k, int slot0, int src0 = 0) {
    __shared__ dd lds[BT / WAVE];
    const int j = blockIdx.x;
    if (j >= k) return;
    dd r{0.0, 0.0};
    for (int b = threadIdx.x; b < nblk; b += BT) r = dd_add(r, ld_dd(m.spart + b * 8 + 2 * (src0 + j)));
    r = block_sum_dd<BT>(r, lds);
    if (threadIdx.x == 0) st_dd(m.scal + ((int64_t)m.rank * SS + slot0 + j) * 2, r);
}

// ================================================================== column passes
// grid (ceil(E/BT), G): thread = one event column, loop over a chunk of rows.
// align > 1 rounds the chunk up to a multiple of align rows (whole 128-byte lines for
// the column-major T writes of k_colstats); trailing blocks may get an empty range.
// [r0, r1) of this block's row chunk; align: chunk starts a multiple of it -- except an empty
// trailing chunk, which is [n_rows, n_rows) (callers stepping in aligned groups test r0 < r1)
__device__ __forceinline__ void row_range(const pcx_mat& m, int64_t& r0, int64_t& r1, int64_t align = 1) {
    int64_t per = (m.n_rows + gridDim.y - 1) / gridDim.y;
    per = (per + align - 1) / align * align;
    r0 = (int64_t)blockIdx.y * per;
    r0 = r0 < m.n_rows ? r0 : m.n_rows;
    r1 = r0 + per < m.n_rows ? r0 + per : m.n_rows;
}

// compensated sum of v[r0 .. r1), identical in every lane of the wave (lanes stride the
// rows, then a fixed butterfly); every lane of the wave must call it
__device__ __forceinline__ dd chunk_sum_dd(const double* v, int64_t r0, int64_t r1) {
    acc2 a;
    for (int64_t i = r0 + (threadIdx.x & (WAVE - 1)); i < r1; i += WAVE) a.add(v[i]);
    return wave_sum_dd(a.get());
}

// Row loop of the column passes: U rows' loads are issued before any of them is
// consumed (the per-row work carries a dependency through the running sums, so
// without this each thread keeps one 8-byte load in flight -- ~2 TB/s at C5).
constexpr int ROW_UNROLL = 8;

template <int U, class LOAD, class PROC>
__device__ __forceinline__ void rows_unrolled(int64_t r0, int64_t r1, LOAD load, PROC proc) {
    int64_t i = r0;
    for (; i + U <= r1; i += U) {
        decltype(load(i)) v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = load(i + u);
#pragma unroll
        for (int u = 0; u < U; u++) proc(i + u, v[u]);
    }
    for (; i < r1; i++) proc(i, load(i));
}

// Software-pipelined row loop of the column passes: the next U rows' loads are issued before
// the current U rows are processed, so every wave keeps loads in flight through its compute
// (with rows_unrolled a wave alternates a load burst and a compute burst, and at the few waves
// per CU these passes run the bursts leave HBM idle).
#ifndef PCX_PIPE_U
#define PCX_PIPE_U 8
#endif
constexpr int PIPE_U = PCX_PIPE_U;

template <int U, class LOAD, class PROC>
__device__ __forceinline__ void rows_pipelined(int64_t r0, int64_t r1, LOAD load, PROC proc) {
    int64_t i = r0;
    if (r1 - r0 >= U) {
        decltype(load(i)) cur[U];
#pragma unroll
        for (int u = 0; u < U; u++) cur[u] = load(i + u);
        for (; i + 2 * U <= r1; i += U) {
            decltype(load(i)) nxt[U];
#pragma unroll
            for (int u = 0; u < U; u++) nxt[u] = load(i + U + u);
#pragma unroll
            for (int u = 0; u < U; u++) proc(i + u, cur[u]);
#pragma unroll
            for (int u = 0; u < U; u++) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < U; u++) proc(i + u, cur[u]);
        i += U;
    }
    for (; i < r1; i++) proc(i, load(i));
}

// the same over a strided row set i = first, first + stride, ... < n
template <int U, class LOAD, class PROC>
__device__ __forceinline__ void rows_strided(int64_t first, int64_t stride, int64_t n, LOAD load, PROC proc) {
    int64_t i = first;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        decltype(load(i)) v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = load(i + u * stride);
#pragma unroll
        for (int u = 0; u < U; u++) proc(i + u * stride, v[u]);
    }
    for (; i < n; i += stride) proc(i, load(i));
}

struct XW {
    double x, w;
};

// min / max of two non-NaN doubles (fmin / fmax canonicalise both operands first: three more
// fp64 VALU ops per element in k_colstats)
__device__ __forceinline__ double min_nn(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double max_nn(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// ---------------------------------------------------------------- covariance operands
// z in {0, 1, 2} of 16 rows packed into one uint32 (the B operand of k_gemm_i8): row r at bit
// 8 (r % 4) + 2 (r / 4); zpack_bit(r) is the bit of value 1
__device__ __forceinline__ uint32_t zpack_bit(int r) { return 1u << (8 * (r & 3) + 2 * (r >> 2)); }

// PCX_M_COLSTATS: present count, sum rep, sum rep*x, zero count, max rep (first row),
// min/max present value; writes the scaled columns (column-major) into T.  A lane owns a column
// and walks the rows, so its T column is one contiguous run; the lanes' values go through a
// per-wave LDS tile of 16 rows, and the wave writes them out as 8 whole 128-byte segments per
// store instruction (lanes 8 k .. 8 k + 7 one column's 16 rows), where a lane-per-column store
// touched 64 lines with 16 bytes each (C5: 9.1 -> 8.3 ms; 6.9 with no T at all).  The division
// by the range as a reciprocal plus one exact correction (div_rn), int_dtype as a template
// parameter, scalar row addresses and the mantissa-bit off-grid test: 47 -> 26 VALU per element,
// 8.3 -> 7.4 ms (5.57 TB/s).  Rejected: T in 16-row blocks [row / 16][scaled column][16], so a
// wave's stores form one contiguous run (8.3 ms either way).
constexpr int CS_TLD = 18;  // doubles per column in the transpose tile (16 rows + pad: 16-byte aligned pairs)
template <bool EQW, bool INT>  // EQW: reputation=None (every weight 1/N); INT: m.int_dtype
__global__ void __launch_bounds__(BT) k_colstats(pcx_mat m) {
    __shared__ __attribute__((aligned(16))) double tile[BT / WAVE][WAVE * CS_TLD];
    const int E = (int)m.n_events;
    // the wave's first column (wave-uniform: a scalar register, so row addresses are scalar too)
    const int c0 = __builtin_amdgcn_readfirstlane(blockIdx.x * BT + (threadIdx.x & ~(WAVE - 1)));
    if (c0 >= E) return;
    const int lane = threadIdx.x & (WAVE - 1);
    const bool live = c0 + lane < E;
    const int c = live ? c0 + lane : E - 1;  // dead lanes shadow the last column (nothing stored)
    const int cl = c - c0;                    // the lane's column within the wave's run
    const ColParam p = col_param(m, c, false);
    double* const lt = tile[threadIdx.x / WAVE];
    // the flush's columns: lane l writes rows 2 (l & 7), +1 of wave column 8 k + (l >> 3), k < 8
    int tsi[8];  // their T columns (-1: not scaled)
    bool any_t = false;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int cw = c0 + 8 * k + (lane >> 3);
        tsi[k] = (m.scaled_index && cw < E) ? m.scaled_index[cw] : -1;
        any_t |= tsi[k] >= 0;
    }
    any_t = __any(any_t);  // wave-uniform
    int64_t r0, r1;
    row_range(m, r0, r1, 16);  // 16-row groups: whole 128-byte T segments
    // rows [g0, g0 + nr) of the tile to T (wave-uniform call; every lane takes part); with an
    // even row count every segment (an even offset from T's 256-byte aligned base) takes a 16-byte store
    const bool t_al = (m.n_rows & 1) == 0;
    auto flush = [&](int64_t g0, int nr) {
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        const int pr = 2 * (lane & 7);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (tsi[k] < 0) continue;
            const double* src = lt + (8 * k + (lane >> 3)) * CS_TLD + pr;
            double* dst = m.T + (int64_t)tsi[k] * m.n_rows + g0 + pr;
            if (t_al && pr + 1 < nr) {
                *reinterpret_cast<double2*>(dst) = *reinterpret_cast<const double2*>(src);
            } else {
                if (pr < nr) dst[0] = src[0];
                if (pr + 1 < nr) dst[1] = src[1];
            }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
    };
    acc2 sr, srx, sx;
    constexpr bool eqw = EQW;
    // counts in 32-bit integers and the first present row as an offset (fewer fp64 VALU ops per
    // element: the pass was VALU-bound before the division became a reciprocal)
    uint32_t icnt = 0, inz = 0;
    uint32_t fro = 0xffffffffu;  // EQW: the first present row's offset from r0 (a running min)
    double mx = -1.0, arg = -1.0, mn_x = __builtin_inf(), mx_x = -__builtin_inf();
    // a present value outside {1, 1.5, 2} (M_COV_PLAN): inside [1, 2] (from mn_x / mx_x at the
    // end) the grid values are those whose mantissa has no bit below its top one -- an OR of
    // those bits replaces three compares per element
    uint32_t mant_hi = 0, mant_lo = 0;
    // EQW: every weight is 1 / N (k_rep_local), so the largest one is the first present row's:
    // no weight loads, and the argmax is that row's index, converted once at the end
    int64_t first_row = -1;
    rows_pipelined<PIPE_U>(
        r0, r1,
        [&](int64_t i) {  // (the row's wave-uniform base: a scalar address plus the lane offset)
            const __amdgpu_buffer_rsrc_t row = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<double*>(m.reports + i * E + c0), 0, WAVE * 8, 0x00020000);
            const double x = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(row, cl * 8, 0, 0));
            return XW{x, eqw ? 0.0 : m.rep[i]};
        },
        [&](int64_t i, XW v) {
            const double x = rescale(v.x, p, INT ? 1 : 0);
            const bool isn = __builtin_isnan(x);
            const bool z = x == 0.0;
            if (any_t) {
                lt[lane * CS_TLD + (i & 15)] = (isn || z) ? __builtin_nan("") : x;
                if ((i & 15) == 15) flush(i - 15, 16);
            }
            inz += z ? 1u : 0u;
            if (isn || z) return;
            icnt++;
            if constexpr (eqw) {  // reputation=None: every weight is 1/N -- sum x alone, scale once at the end
                sx.add(x);
                fro = min(fro, (uint32_t)(i - r0));
            } else {
                const double r = v.w;
                sr.add(r);
                srx.add_prod(r, x);
                if (r > mx) {
                    mx = r;
                    arg = (double)(m.row_offset + i);
                }
            }
            mn_x = min_nn(mn_x, x);
            mx_x = max_nn(mx_x, x);
            const uint64_t xb = __double_as_longlong(x);
            mant_hi |= (uint32_t)(xb >> 32) & 0x7ffffu;  // (mantissa bits 32..50; 51 is 1.5's)
            mant_lo |= (uint32_t)xb;
        });
    if (any_t && r1 > r0 && (r1 & 15)) flush(r1 & ~(int64_t)15, (int)(r1 & 15));  // the last, partial group
    if (!live) return;
    const double cnt = (double)icnt, nz = (double)inz;
    // (read for unscaled events only; no present value: not off the grid)
    const bool offgrid = !p.scaled && icnt > 0 && !(mn_x >= 1.0 && mx_x <= 2.0 && mant_hi == 0 && mant_lo == 0);
    if (eqw && fro != 0xffffffffu) first_row = r0 + fro;
    if (eqw && first_row >= 0) {
        mx = 1.0 / (double)m.n_total;  // = m.rep[i] (k_rep_local)
        arg = (double)(m.row_offset + first_row);
    }
    double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
    st_dd(pp + 0, {cnt, 0.0});
    if constexpr (eqw) {  // sum r = cnt r exactly, sum r x = (sum x) r to dd accuracy
        const double r = 1.0 / (double)m.n_total;  // = m.rep[i] (k_rep_local)
        st_dd(pp + 2, two_prod_dd(cnt, r));
        st_dd(pp + 4, dd_mul_d(sx.get(), r));
    } else {
        st_dd(pp + 2, sr.get());
        st_dd(pp + 4, srx.get());
    }
    st_dd(pp + 6, {nz, 0.0});
    double* mp = m.mpart + ((int64_t)blockIdx.y * E + c) * CM;
    mp[0] = mx;
    mp[1] = arg;
    mp[2] = mn_x;
    mp[3] = mx_x;
    mp[4] = offgrid ? 1.0 : 0.0;
}

// reduce part[G][E][k] over G (in order) into cstat[rank][E][base + k]; optional max partials
// one wave per column: lane l sums the row-chunk partials g = l, l + 64, ... of each dd slot,
// then a fixed butterfly over the lanes (deterministic); the column extremes likewise, the
// max-reputation argmax keeping the first row chunk on ties (the sequential order's choice)
constexpr int CF_MAXK = 8;
__global__ void __launch_bounds__(BT) k_col_finish(pcx_mat m, int G, int k, int base, int with_max) {
    const int c = blockIdx.x * (BT / WAVE) + threadIdx.x / WAVE;
    const int lane = threadIdx.x % WAVE;
    const int E = (int)m.n_events;
    if (c >= E) return;  // wave-uniform
    dd r[CF_MAXK];
#pragma unroll
    for (int j = 0; j < CF_MAXK; j++) r[j] = dd{0.0, 0.0};
    for (int g = lane; g < G; g += WAVE) {
        const double* pp = m.part + ((int64_t)g * E + c) * 16;
#pragma unroll
        for (int j = 0; j < CF_MAXK; j++)
            if (j < k) r[j] = dd_add(r[j], ld_dd(pp + 2 * j));
    }
#pragma unroll
    for (int j = 0; j < CF_MAXK; j++)
        if (j < k) {
            const dd t = wave_sum_dd(r[j]);
            if (lane == 0) st_dd(m.cstat + (((int64_t)m.rank * E + c) * CS + base + j) * 2, t);
        }
    if (with_max) {
        double mx = -1.0, arg = -1.0, mn_x = __builtin_inf(), mx_x = -__builtin_inf(), og = 0.0;
        int gi = G;  // chunk of the current maximum
        for (int g = lane; g < G; g += WAVE) {
            const double* mp = m.mpart + ((int64_t)g * E + c) * CM;
            if (mp[0] > mx) {
                mx = mp[0];
                arg = mp[1];
                gi = g;
            }
            mn_x = fmin(mn_x, mp[2]);
            mx_x = fmax(mx_x, mp[3]);
            og = fmax(og, mp[4]);
        }
        for (int d = WAVE / 2; d >= 1; d >>= 1) {
            const double omx = __shfl_xor(mx, d, WAVE), oarg = __shfl_xor(arg, d, WAVE);
            const int ogi = __shfl_xor(gi, d, WAVE);
            if (omx > mx || (omx == mx && ogi < gi)) {
                mx = omx;
                arg = oarg;
                gi = ogi;
            }
            mn_x = fmin(mn_x, __shfl_xor(mn_x, d, WAVE));
            mx_x = fmax(mx_x, __shfl_xor(mx_x, d, WAVE));
            og = fmax(og, __shfl_xor(og, d, WAVE));
        }
        if (lane == 0) {
            double* o = m.cmax + ((int64_t)m.rank * E + c) * CM;
            o[0] = mx;
            o[1] = arg;
            o[2] = mn_x;
            o[3] = mx_x;
            o[4] = og;
        }
    }
}

__device__ __forceinline__ dd cst(const pcx_mat& m, int c, int slot) {
    return rank_sum(m.cstat, m.world, m.n_events * CS * 2, ((int64_t)c * CS + slot) * 2);
}
__device__ __forceinline__ dd scl(const pcx_mat& m, int slot) {
    return rank_sum(m.scal, m.world, SS * 2, (int64_t)slot * 2);
}

// PCX_M_GUESS: interpolation fills of binary events; mark scaled events that need a median
__global__ void __launch_bounds__(BT) k_guess(pcx_mat m) {
    const int c = blockIdx.x * BT + threadIdx.x;
    const int E = (int)m.n_events;
    if (c >= E) return;
    const dd cnt = cst(m, c, 0);
    const dd S_r = cst(m, c, 1);
    const dd S_rx = cst(m, c, 2);
    const double present = dd_to_double(cnt);
    const double miss = (double)m.n_total - present;
    double mn_x = __builtin_inf(), mx_x = -__builtin_inf();
    for (int w = 0; w < m.world; w++) {
        mn_x = fmin(mn_x, m.cmax[((int64_t)w * E + c) * CM + 2]);
        mx_x = fmax(mx_x, m.cmax[((int64_t)w * E + c) * CM + 3]);
    }
    m.ev[EV_MINX * E + c] = mn_x;
    m.ev[EV_MAXX * E + c] = mx_x;
    m.ev[EV_MISS * E + c] = miss;
    m.ev[EV_NZERO * E + c] = dd_to_double(cst(m, c, 3));
    const bool sc = m.scaled && m.scaled[c];
    double g = 0.0;
    m.hard[c] = HARD_NONE;
    if (!sc && !m.no_fill) {
        // sequential weighted mean of the present reports, then catch (:304-309)
        const double mean = present > 0 ? dd_div(S_rx, S_r) : 0.0;
        g = catch_value(mean, m.catch_tolerance);
        if (m.int_dtype) g = trunc(g);
        // within the sequential sum's rounding of a catch threshold: replay the reference's
        // order (k_hard_*); the bound is (n terms of |w x|, plus the w / total roundings)
        if (miss > 0 && present > 0) {
            const double B = (4.0 * present + 64.0) * 0x1p-53 * (fabs(mean) + 1.0);
            if (fabs(mean - (1.5 - m.catch_tolerance)) <= B || fabs(mean - (1.5 + m.catch_tolerance)) <= B)
                m.hard[c] = HARD_MEAN;
        }
    }
    m.ev[EV_GUESS * E + c] = g;  // scaled events: phase-1 median (selection)
}

// PCX_M_MEAN: mu = rep . F / sum(rep) (np.ma.average, :317-319); old = rep . F (:490)
__global__ void __launch_bounds__(BT) k_mean(pcx_mat m) {
    const int c = blockIdx.x * BT + threadIdx.x;
    const int E = (int)m.n_events;
    if (c >= E) return;
    const dd S_r = cst(m, c, 1);
    const dd S_rx = cst(m, c, 2);
    const dd R_tot = scl(m, SC_REP);
    const double g = m.ev[EV_GUESS * E + c];
    const dd miss_w = dd_sub(R_tot, S_r);  // reputation of the filled cells
    const dd num = m.ev[EV_MISS * E + c] > 0 ? dd_add(S_rx, dd_mul_d(miss_w, g)) : S_rx;
    m.ev[EV_OLD * E + c] = m.ob_order ? ob_col_dot(m, m.rep, c) : dd_to_double(num);  // np.dot(rep, F) (:489)
    m.ev[EV_MU * E + c] = dd_div(num, R_tot);
}

// ================================================================== covariance (fp64 MFMA)
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int CT = 128;          // C tile edge
constexpr int KB = 16;           // rows staged per step
constexpr int LDP = CT + 16;     // padded LDS row (bank-conflict-free b64 fragment reads)

__device__ __forceinline__ void tri_index(int t, int& I, int& J) {
    int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while ((i + 1) * (i + 2) / 2 <= t) i++;
    while (i * (i + 1) / 2 > t) i--;
    I = i;
    J = t - i * (i + 1) / 2;
}

// 128x128 tile of A_I^T B_J accumulated over rows [rb, re) on fp64 MFMA
// (v_mfma_f64_16x16x4_f64): 4 waves in 2x2, each 64x64 = 4x4 MFMA blocks; 16 rows
// are staged per step through LDS (rows padded to LDP doubles so the b64 fragment
// reads are bank-conflict free) and the next 16 are prefetched into registers
// while the MFMAs run.  LOADER fills va (A side) / vb (B side) for 8 columns.
template <class LOADER>
__device__ void mfma_tile(LOADER& ld, int I, int J, int64_t rb, int64_t re, d4 (&acc)[4][4]) {
    __shared__ __attribute__((aligned(16))) double As[KB][LDP];
    __shared__ __attribute__((aligned(16))) double Bs[KB][LDP];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    const int sr = tid >> 4;        // staged row 0..15
    const int scg = (tid & 15) * 8; // staged column group
    double va[8], vb[8];
    if (rb < re) ld.load(rb + sr, re, I, J, scg, va, vb);
    for (int64_t i0 = rb; i0 < re; i0 += KB) {
        __syncthreads();
        for (int k = 0; k < 8; k++) {
            As[sr][scg + k] = va[k];
            Bs[sr][scg + k] = vb[k];
        }
        __syncthreads();
        if (i0 + KB < re) ld.load(i0 + KB + sr, re, I, J, scg, va, vb);  // prefetch under the MFMAs
#pragma unroll
        for (int kk = 0; kk < KB / 4; kk++) {
            const int kr = kk * 4 + (lane >> 4);
            double af[4], bf[4];
#pragma unroll
            for (int a = 0; a < 4; a++) af[a] = As[kr][wr * 64 + a * 16 + (lane & 15)];
#pragma unroll
            for (int b = 0; b < 4; b++) bf[b] = Bs[kr][wc * 64 + b * 16 + (lane & 15)];
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int b = 0; b < 4; b++)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
    }
}

// D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * r
__device__ __forceinline__ void store_tile(double* out, int64_t ld, int64_t E, int I, int J, const d4 (&acc)[4][4]) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++)
            for (int r = 0; r < 4; r++) {
                const int64_t p = (int64_t)I * CT + wr * 64 + a * 16 + (lane >> 4) + 4 * r;
                const int64_t q = (int64_t)J * CT + wc * 64 + b * 16 + (lane & 15);
                if (p < E && q < E) out[p * ld + q] = acc[a][b][r];
            }
}

__device__ __forceinline__ uint32_t zpack_get(uint32_t P, int r) { return (P >> (8 * (r & 3) + 2 * (r >> 2))) & 3u; }
__device__ __forceinline__ uint32_t* zb_packed(const pcx_mat& m) { return reinterpret_cast<uint32_t*>(m.zB); }

// PCX_M_COV_PLAN: the wcd column order.  A "grid" event is binary with every filled value
// in {1, 1.5, 2} (present reports on the grid -- k_colstats -- and a fill, if any, on it),
// while every token lies in [0, 63] (so tok * z fits int8).  General events take the
// first wcd positions, grid events the rest, each group in event order; the covariance
// tiles made only of grid positions run on int8 MFMA over z = 2 (F - 1) in {0, 1, 2}:
//   sum_i tok_i (F_ij - mu_j)(F_ik - mu_k) = c_j c_k T + (c_j Z_k + c_k Z_j) / 2 + P_jk / 4
// with c = 1 - mu, T = sum tok, Z_j = sum tok z_ij, P_jk = sum tok z_ij z_ik (exact integers).
__device__ __forceinline__ bool grid_event(const pcx_mat& m, int c, bool big) {
    const int64_t E = m.n_events;
    if (big || (m.scaled && m.scaled[c])) return false;
    for (int w = 0; w < m.world; w++)
        if (m.cmax[((int64_t)w * E + c) * CM + 4] != 0.0) return false;
    const double g = m.ev[EV_GUESS * E + c];
    return m.ev[EV_MISS * E + c] == 0.0 || g == 1.0 || g == 1.5 || g == 2.0;
}

__global__ void __launch_bounds__(1024) k_cov_plan(pcx_mat m) {
    __shared__ int wg[16], wb[16];
    __shared__ int base[2];
    const int E = (int)m.n_events;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const bool big = dd_to_double(scl(m, SC_BIGTOK)) > 0.0;
    int ng = 0;
    for (int c = tid; c < E; c += 1024) ng += grid_event(m, c, big) ? 0 : 1;
    for (int s = 32; s >= 1; s >>= 1) ng += __shfl_xor(ng, s, WAVE);
    if (lane == 0) wg[wv] = ng;
    __syncthreads();
    if (tid == 0) {
        int G = 0;
        for (int w = 0; w < 16; w++) G += wg[w];
        base[0] = 0;
        base[1] = G;
        m.info[IN_COV_GENERAL] = G;
    }
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int c0 = 0; c0 < E; c0 += 1024) {
        const int c = c0 + tid;
        const bool valid = c < E;
        const bool gr = valid && grid_event(m, c, big);
        const uint64_t bg = __ballot(valid && !gr), bb = __ballot(gr);
        if (lane == 0) {
            wg[wv] = __popcll(bg);
            wb[wv] = __popcll(bb);
        }
        __syncthreads();
        int pg = base[0], pb = base[1];
        for (int w = 0; w < wv; w++) {
            pg += wg[w];
            pb += wb[w];
        }
        if (valid) {
            const int pos = gr ? pb + __popcll(bb & lt) : pg + __popcll(bg & lt);
            m.cov_perm[pos] = c;
            m.cov_pos[c] = pos;
        }
        __syncthreads();
        if (tid == 0) {
            for (int w = 0; w < 16; w++) {
                base[0] += wg[w];
                base[1] += wb[w];
            }
        }
        __syncthreads();
    }
    for (int64_t p = E + tid; p < m.wcd_ld; p += 1024) m.cov_perm[p] = -1;
    // mixed pairs (a general position q < 128 jb with a grid one) on int8 slices of w: the
    // fixed-point exponent of each general position from the bound of |F - mu| over its
    // present values (all ranks) and its fill; any non-finite bound keeps them on fp64
    __syncthreads();
    const int G = base[0];
    const int gb = (G + CT - 1) / CT * CT;
    int bad = 0;
    double maxtok = 0.0;  // the largest token over all ranks (scal slot SC_MAXTOK, an integer)
    for (int w = 0; w < m.world; w++) maxtok = fmax(maxtok, m.scal[((int64_t)w * SS + SC_MAXTOK) * 2]);
    if (!big && gb > 0 && gb < E) {
        for (int q = tid; q < gb; q += 1024) {
            const int c = m.cov_perm[q];
            const double mu = m.ev[EV_MU * E + c];
            double bnd = 0.0;
            if (m.ev[EV_MISS * E + c] < (double)m.n_total) {  // some present report
                double mn = __builtin_inf(), mx = -__builtin_inf();
                for (int w = 0; w < m.world; w++) {
                    mn = fmin(mn, m.cmax[((int64_t)w * E + c) * CM + 2]);
                    mx = fmax(mx, m.cmax[((int64_t)w * E + c) * CM + 3]);
                }
                bnd = fmax(fabs(mx - mu), fabs(mn - mu));
            }
            if (m.ev[EV_MISS * E + c] > 0.0) bnd = fmax(bnd, fabs(m.ev[EV_GUESS * E + c] - mu));
            if (!__builtin_isfinite(bnd) || __builtin_isnan(mu)) bad = 1;
            // the general x general product's digits of w itself: |w| 2^-f <= 1/2 likewise
            if (m.escale) m.escale[q] = bnd > 0.0 && __builtin_isfinite(bnd) ? ldexp(1.0, -(ilogb(bnd) + 2)) : 1.0;
            // the digits are of tok w: |tok w| <= maxtok bnd < 2^(ilogb + 1), so |tok w| 2^-e <= 1/2
            // with e = ilogb + 2 (first digit |d| <= 64)
            bnd *= maxtok;
            m.dscale[q] = bnd > 0.0 && __builtin_isfinite(bnd) ? ldexp(1.0, -(ilogb(bnd) + 2)) : 1.0;
        }
    }
    bad = __syncthreads_or(bad);
    if (tid == 0) {
        m.info[IN_COV_MIXED] = (!big && gb > 0 && gb < E && !bad) ? 1 : 0;
        // every token of this rank is maxtok = 2^k (the largest anywhere): tok w 2^-e = w 2^-f
        // exactly (dscale = 2^-k escale above) and both digit strings coincide, so the general x
        // general product takes zD for both operands (reputation=None: int(1/N 1e6) = 1 for
        // N <= 1e6; 8 for a 125k-row consensus)
        // (compared exactly: the token sum is an exact double-double of integers, maxtok n_rows an
        // exact two-product -- in doubles, a sum above 2^53 a few units short would compare equal)
        const dd tsum = ld_dd(m.scal + ((int64_t)m.rank * SS + SC_TOK) * 2);
        const bool pow2 = maxtok >= 1.0 && maxtok < 0x1p52 && maxtok == ldexp(1.0, ilogb(maxtok));
        const double pp = maxtok * (double)m.n_rows, pe = fma(maxtok, (double)m.n_rows, -pp);
        m.info[IN_COV_TOK1] = (pow2 && (tsum.hi - pp) + (tsum.lo - pe) == 0.0) ? 1 : 0;
    }
}

// PCX_M_WCD: wcd = F - mu (:317-322) materialised once, [wcd_rows][wcd_ld] in the
// M_COV_PLAN column order with zero padding, plus the tokens zero-padded past n_rows, and
// for the pure-grid positions (>= 128 cov_jb) the int8 operands tok * z (zA) and z (zB) in
// 16-row interleaved column-major blocks [row / 16][position][16] -- one 16-byte MFMA
// fragment per (position, 16 rows) -- and Z_j = sum tok z_ij (zsum, exact).  The
// consensus entry's "original" / "filled" matrices are written here too (no M_MATRICES
// pass over the reports).
constexpr int WCD_COLS = 2 * BT;  // columns per block (2 per thread)
// 4096 blocks, halved until each has at least WCD_MIN_ROWS rows: a C5 shard (125k rows) on ~1k
// blocks of ~1k rows ran k_wcd 3.49 -> 3.30 ms against 4096 of 256 (1M rows: 4096 either way)
#ifndef PCX_WCD_MIN_ROWS  // (a build parameter for A/B runs, tools/ab_variant.sh)
#define PCX_WCD_MIN_ROWS 768
#endif
#ifndef PCX_WCD_MIN_WG
#define PCX_WCD_MIN_WG 1024
#endif
constexpr int64_t WCD_MIN_ROWS = PCX_WCD_MIN_ROWS;

// Blocks own a contiguous row range (a multiple of 64 rows) of a 512-event block; each
// wave also counts the NaN / zero rescaled reports of its 128 events per row (ballots),
// the block folds its four waves in LDS and writes the counts of 64 rows at a time to
// rowpart[column block] (k_scores adds the column blocks up: rowstat for na_row /
// participation, :549-567).
__global__ void __launch_bounds__(BT) k_wcd(pcx_mat m) {
    __shared__ uint32_t cnt[4][64][2];
    const int E = (int)m.n_events;
    const int64_t ld = m.wcd_ld;
    const int c0 = blockIdx.y * WCD_COLS + 2 * threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t gb = (int64_t)m.cov_jb * CT;
    const bool even_e = (E & 1) == 0;  // 16-byte aligned event pairs in the N x E outputs
    ColParam p[2];
    bool ok[2], zc[2];
    int64_t pos[2];
    for (int k = 0; k < 2; k++) {
        const int c = c0 + k;
        ok[k] = c < E;
        p[k] = ok[k] ? col_param(m, c, true) : ColParam{false, 0.0, 1.0, 0.0, 0.0, 1.0};
        pos[k] = ok[k] ? m.cov_pos[c] : (c < ld ? c : -1);  // padding positions keep their index
        zc[k] = ok[k] && pos[k] >= gb;
    }
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; blockIdx.y == 0 && i < m.wcd_rows + 64;
         i += (int64_t)gridDim.x * BT)
        m.tokp[i] = i < m.n_rows ? m.tok[i] : 0.0;
    const int64_t per = ((m.wcd_rows + gridDim.x - 1) / gridDim.x + 63) / 64 * 64;
    int64_t r0 = blockIdx.x * per;
    r0 = r0 < m.wcd_rows ? r0 : m.wcd_rows;
    const int64_t r1 = r0 + per < m.wcd_rows ? r0 + per : m.wcd_rows;
    uint32_t* part = m.rowpart + (int64_t)blockIdx.y * m.wcd_rows * 2;
    int64_t zs[2] = {0, 0};
    for (int64_t g0 = r0; g0 < r1; g0 += 64) {
        const int gn = r1 - g0 < 64 ? (int)(r1 - g0) : 64;  // a multiple of 16 (wcd_rows % 16 == 0)
        for (int q0 = 0; q0 < gn; q0 += 16) {
            uint32_t za[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}}, zb[2] = {0, 0}, nb[2] = {0, 0};
#pragma unroll
            for (int h = 0; h < 4; h++) {
                double rv[4][2];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int64_t i = g0 + q0 + 4 * h + u;
                    const bool live = i < m.n_rows;
                    const double* r = m.reports + (live ? i : 0) * E + c0;
                    rv[u][0] = (live && ok[0]) ? r[0] : 0.0;
                    rv[u][1] = (live && ok[1]) ? r[1] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int64_t i = g0 + q0 + 4 * h + u;
                    const bool live = i < m.n_rows;
                    const int tk = (live && (zc[0] || zc[1])) ? (int)m.tok[i] : 0;
                    double w[2] = {0.0, 0.0}, xo[2] = {0.0, 0.0}, fo[2] = {0.0, 0.0};
                    int nn = 0, nz = 0;
#pragma unroll
                    for (int k = 0; k < 2; k++) {
                        if (live && ok[k]) {
                            const double x = rescale(rv[u][k], p[k], m.int_dtype);
                            nn += __builtin_isnan(x) ? 1 : 0;
                            nz += x == 0.0 ? 1 : 0;
                            const double f = missing(x) ? p[k].guess : x;
                            w[k] = f - p[k].mu;
                            // (a NaN report keeps its own bits in `original`, as numpy's (r - lo) /
                            // range does: div_rn's fma(-q0, ..) would return it negated)
                            xo[k] = __builtin_isnan(x) ? rv[u][k] : x;
                            fo[k] = f;
                            if (m.compact) nb[k] |= missing(x) ? 1u << (4 * h + u) : 0u;
                            if (zc[k]) {
                                const int z = (int)((f - 1.0) * 2.0);
                                za[k][h] |= (uint32_t)(uint8_t)(int8_t)(tk * z) << (8 * u);
                                zb[k] |= (uint32_t)z * zpack_bit(4 * h + u);
                                zs[k] += tk * z;
                            }
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 2; k++) {
                        // compact: the general positions' filled values Fg (padding rows: mu, F - mu = 0)
                        // for M_GEMV2 / M_OUTCOMES; the grid positions live in zA / zB only
                        if (m.compact && pos[k] >= 0 && pos[k] < gb)
                            m.Fg[i * gb + pos[k]] = (live && ok[k]) ? fo[k] : p[k].mu;
                        // wcd = F - mu of the general positions (all of them without the int8 mixed
                        // block) for k_syrk / k_scores_grid / k_digits (centring the compact Fg on
                        // the fly instead writes 8 GB less at C5, but k_syrk then runs 26 ms, not 18)
                        // (with cov_gg8 nothing reads wcd: k_digits and k_scores_grid take Fg - mu,
                        // the same subtraction bit for bit -- 8 GB fewer bytes written at C5)
                        if (pos[k] >= 0 && (!m.cov_mixed || pos[k] < gb) && !m.cov_gg8) m.wcd[i * ld + pos[k]] = w[k];
                    }
                    // in place (result["original"] aliases the reports, as the reference's own does,
                    // __init__.py:121, 266-269, 584): only the scaled columns change -- the rescaled
                    // value over the report this thread just read
                    if (live && m.orig_inplace) {
                        double* rw = const_cast<double*>(m.reports) + i * E + c0;
#pragma unroll
                        for (int k = 0; k < 2; k++)
                            if (ok[k] && p[k].scaled) rw[k] = xo[k];
                    }
                    // result["original"] / result["filled"] (:266-313), event order
                    if (live && (m.original || m.filled)) {
                        const int64_t o = i * E + c0;
                        if (even_e && ok[1]) {
                            if (m.original) *(double2*)(m.original + o) = double2{xo[0], xo[1]};
                            if (m.filled) *(double2*)(m.filled + o) = double2{fo[0], fo[1]};
                        } else {
#pragma unroll
                            for (int k = 0; k < 2; k++)
                                if (ok[k]) {
                                    if (m.original) m.original[o + k] = xo[k];
                                    if (m.filled) m.filled[o + k] = fo[k];
                                }
                        }
                    }
                    const uint64_t b0 = __ballot(nn >= 1), b1 = __ballot(nn == 2);
                    const uint64_t z0 = __ballot(nz >= 1), z1 = __ballot(nz == 2);
                    if (lane == 0) {
                        cnt[wv][q0 + 4 * h + u][0] = __popcll(b0) + __popcll(b1);
                        cnt[wv][q0 + 4 * h + u][1] = __popcll(z0) + __popcll(z1);
                    }
                }
            }
            const int64_t grp = (g0 + q0) >> 4;
            if (m.compact) {
#pragma unroll
                for (int k = 0; k < 2; k++)
                    if (ok[k]) m.nam[grp * ld + pos[k]] = (uint16_t)nb[k];
            }
#pragma unroll
            for (int k = 0; k < 2; k++)
                if (zc[k]) {
                    const int64_t o = grp * m.zq + (pos[k] - gb);
                    *(uint4*)(m.zA + o * 16) = uint4{za[k][0], za[k][1], za[k][2], za[k][3]};
                    zb_packed(m)[o] = zb[k];
                }
        }
        __syncthreads();
        if (threadIdx.x < gn) {
            const int t = threadIdx.x;
            const uint32_t a = cnt[0][t][0] + cnt[1][t][0] + cnt[2][t][0] + cnt[3][t][0];
            const uint32_t z = cnt[0][t][1] + cnt[1][t][1] + cnt[2][t][1] + cnt[3][t][1];
            *(uint2*)(part + (g0 + t) * 2) = uint2{a, z};
        }
        __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < 2; k++)
        if (zc[k] && zs[k] != 0) atomicAdd((unsigned long long*)&m.zsum[c0 + k], (unsigned long long)zs[k]);
}

// PCX_M_COV step 2: partial C = wcd^T diag(tok) wcd (:326) over one row slice, one
// 128x128 lower-triangle tile per workgroup on fp64 MFMA.  Rows arrive by
// global_load_lds_dwordx4 (one 1 KB tile row per wave instruction) into a two-stage
// LDS ring of 8-row stages; one raw barrier per stage, counted vmcnt (the only
// vector-memory ops in the loop are these DMAs).  39 KB LDS and <= 168 VGPRs
// (launch bounds) = 3 workgroups (3 waves per SIMD) per CU: one wave alone issues an
// f64 MFMA only every ~128 cycles, several interleave to the 64-cycle rate.  Variant
// sweep (BK, ring depth, waves per SIMD, 8-wave tiles): tools/covbench, profiles/r1.
// The A operand is rounded as tok*w before the MFMA (np.ma.multiply(wcd.T, tokens)).
constexpr int SY_BK = 8;                        // rows per stage
constexpr int SY_NBUF = 2;                      // LDS ring depth
constexpr int SY_LDP = CT + 16;                 // padded LDS row: conflict-free b64 fragment reads

template <bool DIAG>
struct SyRing {
    static constexpr int A_OFF = 0;
    static constexpr int B_OFF = SY_BK * SY_LDP;
    static constexpr int T_OFF = (DIAG ? 1 : 2) * SY_BK * SY_LDP;
    static constexpr int STRIDE = T_OFF + 4 * 32;             // doubles per buffer
    static constexpr int LPW = (DIAG ? SY_BK / 4 : SY_BK / 2) + 1;  // DMAs per wave per stage
};
constexpr size_t SY_LDS_BYTES = (size_t)SY_NBUF * SyRing<false>::STRIDE * sizeof(double);


template <bool DIAG>
__device__ __forceinline__ void syrk_tile(const double* W, const double* tok, int64_t ld, int I, int J, int64_t s0,
                                          int64_t ns, double* lds, d4 (&acc)[4][4]) {
    using R = SyRing<DIAG>;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const double* colA = W + I * CT + 2 * lane;
    const double* colB = W + J * CT + 2 * lane;
    auto issue = [&](int64_t s, int b) {
        double* buf = lds + b * R::STRIDE;
        const int64_t row0 = (s0 + s) * SY_BK;
#pragma unroll
        for (int k = 0; k < SY_BK / 4; k++) {
            const int r = wv + 4 * k;
            __builtin_amdgcn_global_load_lds((const void*)(colA + (row0 + r) * ld),
                                             (lds_ptr_t)(buf + R::A_OFF + r * SY_LDP), 16, 0, 0);
        }
        if (!DIAG) {
#pragma unroll
            for (int k = 0; k < SY_BK / 4; k++) {
                const int r = wv + 4 * k;
                __builtin_amdgcn_global_load_lds((const void*)(colB + (row0 + r) * ld),
                                                 (lds_ptr_t)(buf + R::B_OFF + r * SY_LDP), 16, 0, 0);
            }
        }
        // 64 dwords = tokens of rows row0 .. row0+31 (tokp is padded) into this wave's slot
        __builtin_amdgcn_global_load_lds((const void*)((const char*)(tok + row0) + 4 * lane),
                                         (lds_ptr_t)(buf + R::T_OFF + wv * 32), 4, 0, 0);
    };
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < SY_NBUF - 1; s++)
        if (s < ns) issue(s, s);
    for (int64_t t = 0; t < ns; t++) {
        if (t + SY_NBUF - 2 < ns)
            wait_vmcnt<R::LPW * (SY_NBUF - 2)>();
        else
            wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t + SY_NBUF - 1 < ns) issue(t + SY_NBUF - 1, (int)((t + SY_NBUF - 1) % SY_NBUF));
        const double* buf = lds + (int)(t % SY_NBUF) * R::STRIDE;
        const double* As = buf + R::A_OFF;
        const double* Bs = DIAG ? As : buf + R::B_OFF;
        const double* Ts = buf + R::T_OFF + wv * 32;
#pragma unroll
        for (int kk = 0; kk < SY_BK / 4; kk++) {
            const int kr = kk * 4 + (lane >> 4);
            const double tk = Ts[kr];
            double af[4], bf[4];
#pragma unroll
            for (int a = 0; a < 4; a++) af[a] = As[kr * SY_LDP + wr * 64 + a * 16 + (lane & 15)] * tk;
#pragma unroll
            for (int b = 0; b < 4; b++) bf[b] = Bs[kr * SY_LDP + wc * 64 + b * 16 + (lane & 15)];
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int b = 0; b < 4; b++)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        asm volatile("" ::: "memory");
    }
}


// one work item = (tile (I,J) of the trapezoid J < cov_jb of the lower triangle, row
// slice ks) -> cslab[ks] (lower part, wcd positions); the pure-grid tiles are k_syrk_i8's
__global__ void __launch_bounds__(256, 3) k_syrk(pcx_mat m) {
    extern __shared__ __attribute__((aligned(16))) double sy_lds[];
    const int E = (int)m.n_events;
    const int ntiles = m.cov_fp_tiles, nks = m.fp_ks;
    const int nb = (int)(m.wcd_ld / CT);
    const int item = xcd_remap(blockIdx.x, gridDim.x);
    const int ks = item / ntiles;
    int J = 0, I = item % ntiles;
    if (m.cov_mixed) {
        tri_index(I, I, J);  // the Jb x Jb triangle of general tiles
    } else {
        while (I >= nb - J) {  // column J of the trapezoid holds tiles I = J .. nb-1
            I -= nb - J;
            J++;
        }
        I += J;
    }
    const int64_t nst = m.wcd_rows / SY_BK;
    const int64_t per = (nst + nks - 1) / nks;
    const int64_t s0 = ks * per < nst ? ks * per : nst;
    const int64_t s1 = s0 + per < nst ? s0 + per : nst;
    d4 acc[4][4];
    if (I == J)
        syrk_tile<true>(m.wcd, m.tokp, m.wcd_ld, I, J, s0, s1 - s0, sy_lds, acc);
    else
        syrk_tile<false>(m.wcd, m.tokp, m.wcd_ld, I, J, s0, s1 - s0, sy_lds, acc);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int64_t ld = m.fp_ld, pmax = ld < E ? ld : E;
    double* out = m.cslab + (int64_t)ks * ld * ld;
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++)
            for (int r = 0; r < 4; r++) {
                const int64_t p = (int64_t)I * CT + wr * 64 + a * 16 + (lane >> 4) + 4 * r;
                const int64_t q = (int64_t)J * CT + wc * 64 + b * 16 + (lane & 15);
                if (p < pmax && q <= p) out[p * ld + q] = acc[a][b][r];
            }
}

// tok * w of the general positions q < gb (the exact product, as a double-double) as PCX_NDIG
// balanced base-254 digits of (tok w) 2^-e (|tok w 2^-e| <= 1/2): the nearest integer X to
// (tok w 2^-e) 254^NDIG, written in base 254 with digits |d| <= 127, the widest balanced digit
// int8 holds.  The residue is <= 0.52 254^-NDIG of 2^e (6: 2^-48.8 of the column's bound on
// |tok w|, 3.8e-15 relative).  (Round 4 extracted the digits greedily from the top in
// double-double arithmetic, 77 fp64 ops per element against 46 here: M_COV_I8 20.0 -> 19.6 ms.)  Each chunk of rows (blockIdx.y) also adds the
// sum of every digit over its rows to dtok (int64 atomics: exact, order-free): S_q = sum tok w_q
// from the same digits (k_cov_tokrow), so neither int8 product carries a token column.
constexpr double DIG_SCALE = [] {  // 254^NDIG (exact: 6 digits need 48 bits)
    double c = 1.0;
    for (int k = 0; k < PCX_NDIG; k++) c *= PCX_DBASE;
    return c;
}();
// With cov_gg8 the same pass writes PCX_NDIG digits of w 2^-f (escale) to zE, the other operand of
// the general x general product (w 2^-f is exact; X = rint(w 2^-f 254^NDIG) from the product and
// its fma error, as for tok w).  Four lanes share a position's 16-row group, a quarter (4 rows, one
// byte per row: one dword per digit) each, so a wave stores 16 positions x 16 bytes = 256
// contiguous bytes per digit and a lane holds two dwords per digit (a lane per position holding
// all 16 rows -- the round-4 layout -- took 182 VGPRs with both operands: two waves per SIMD,
// 7.0 ms at C5 against 2.7 ms for the tok w digits alone).
__device__ __forceinline__ void balanced_digits(double X, uint32_t (&d)[PCX_NDIG], int u, int32_t* dsum) {
#pragma unroll
    for (int k = PCX_NDIG - 1; k >= 0; k--) {
        double di = X;
        if (k > 0) {
            const double qd = rint(X * (1.0 / PCX_DBASE));
            di = fma(-qd, PCX_DBASE, X);
            X = qd;
        }
        d[k] |= (uint32_t)(uint8_t)(int8_t)(int)di << (8 * u);
        if (dsum) dsum[k] += (int)di;
    }
}

// The covariance guard's sums (k_cov_guard), per general position over this rank's rows, taken by
// the digit passes beside the digits: with t = (tok w 2^-e) 254^NDIG the exact scaled value and X =
// rint(t) its digits' value, the residue delta = X - t (|delta| <= 0.52), summed as sum delta tok and
// sum delta^2 (and for the digits of w, eta = Xe - te: sum tok eta, sum tok eta^2), plus the L1 norm
// of the digits 1 .. NDIG - 1 and, once per rank, sum tok^2.  Each thread sums its rows in fp64
// (error << 2^-24 for the <= 4096 rows of a chunk) and adds the fixed-point value at 2^-24 (the
// squares rounded up) to int64 slots: exact and order-free, so the guard's decision is the same on
// every run.  (A per-row 1 / tok for sum delta^2 / tok cost k_digits1 35 VGPRs: 4 -> 3 waves per
// SIMD, 3.5 -> 4.4 ms at C5; the bound takes tok >= 1 instead, below.)
constexpr double G_FIX = 0x1p24;
// sum |d| over the packed digits 1 .. NDIG - 1 (two's complement bytes; as offset binary b ^ 0x80 =
// d + 128, |d| = |(b ^ 0x80) - 128|: one v_sad_u8 per four digits)
template <int W>
__device__ __forceinline__ int32_t digit_l1(const uint32_t (&d)[PCX_NDIG][W], int32_t acc) {
#pragma unroll
    for (int k = 1; k < PCX_NDIG; k++)
#pragma unroll
        for (int j = 0; j < W; j++) acc = (int32_t)__builtin_amdgcn_sad_u8(d[k][j] ^ 0x80808080u, 0x80808080u, (uint32_t)acc);
    return acc;
}
__device__ __forceinline__ int32_t digit_l1(const uint32_t (&d)[PCX_NDIG], int32_t acc) {
#pragma unroll
    for (int k = 1; k < PCX_NDIG; k++) acc = (int32_t)__builtin_amdgcn_sad_u8(d[k] ^ 0x80808080u, 0x80808080u, (uint32_t)acc);
    return acc;
}
__device__ __forceinline__ void guard_add(int64_t* slot, double v, bool up) {
    const double f = v * G_FIX;
    const long long x = up ? (long long)ceil(f * (1.0 + 0x1p-40)) : (long long)rint(f);
    if (x) atomicAdd((unsigned long long*)slot, (unsigned long long)x);
}

constexpr int DG_POS = BT / 4;  // positions per k_digits workgroup
__global__ void __launch_bounds__(BT) k_digits(pcx_mat m) {
    const int gb = m.cov_jb * CT;
    const int h = threadIdx.x & 3;  // rows 4h .. 4h + 3 of each 16-row group
    const int q = blockIdx.x * DG_POS + (threadIdx.x >> 2);
    const bool live = q < gb;
    const int qq = live ? q : 0;
    const double sc = m.dscale[qq];
    const bool fg = m.cov_gg8 != 0;            // no wcd written: w = Fg - mu (k_wcd's own op)
    const bool gg = fg && m.zE != m.zD;       // the digits of w too (the same ones when every token is 1)
    const double esc = gg ? m.escale[qq] : 1.0;
    const double mu = fg ? m.ev[EV_MU * m.n_events + m.cov_perm[qq]] : 0.0;
    const int64_t ng = m.wcd_rows / 16;
    const int64_t per = (ng + gridDim.y - 1) / gridDim.y;
    const int64_t g0 = blockIdx.y * per, g1 = g0 + per < ng ? g0 + per : ng;
    const int64_t ldd = zd_ld(gb);
    int32_t dsum[PCX_NDIG];  // |d| <= 127: int32-exact for any chunk under 16M rows
#pragma unroll
    for (int k = 0; k < PCX_NDIG; k++) dsum[k] = 0;
    int32_t l1d = 0, l1e = 0;                         // the guard's sums (guard_add)
    double sd = 0.0, sd2 = 0.0, se = 0.0, se2 = 0.0, tok2 = 0.0;
    for (int64_t grp = g0; live && grp < g1; grp++) {
        uint32_t d[PCX_NDIG], e[PCX_NDIG];
#pragma unroll
        for (int k = 0; k < PCX_NDIG; k++) d[k] = e[k] = 0;
        double wr[4], tk[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int64_t i = grp * 16 + 4 * h + u;
            wr[u] = fg ? m.Fg[i * gb + q] - mu : m.wcd[i * m.wcd_ld + q];
            tk[u] = m.tokp[i];  // 0 past n_rows
        }
#pragma unroll 2
        for (int u = 0; u < 4; u++) {  // (two rows at a time: the guard's sums beside four rows' digit
                                       // chains took 139 VGPRs, three waves per SIMD)
            const double w = wr[u] * sc;  // exact (power of two)
            double hi = w * tk[u], lo = fma(w, tk[u], -hi);  // tok w exactly
            // X = rint((tok w 2^-e) 254^NDIG) (|X| <= 254^NDIG / 2 < 2^48, within 0.52 of the
            // exact value), then its balanced base-254 digits from the least significant up:
            // q = rint(X / 254) -- X / 254 is a multiple of 1/254 and X * (1/254) lies within 2^-14 of
            // it, so the rounding is exact but for the 1/2 tie, where either neighbour leaves
            // |d| = 127 -- and d = X - 254 q exactly
            const double pv = hi * DIG_SCALE, pe = fma(hi, DIG_SCALE, -pv), pl = fma(lo, DIG_SCALE, pe);
            const double X = rint(pv + pl);
            balanced_digits(X, d, u, dsum);
            const double dl = (X - pv) - pl;  // X - t (X - pv exact)
            sd = fma(dl, tk[u], sd);
            sd2 = fma(dl, dl, sd2);
            tok2 = fma(tk[u], tk[u], tok2);
            if (gg) {
                const double v = wr[u] * esc, uv = v * DIG_SCALE, ue = fma(v, DIG_SCALE, -uv);
                const double Xe = rint(uv + ue);
                balanced_digits(Xe, e, u, nullptr);
                const double el = (Xe - uv) - ue;
                se = fma(tk[u], el, se);
                se2 = fma(tk[u] * el, el, se2);
            }
        }
        const int64_t o = (grp * ldd + q) * 16 + 4 * h;
        l1d = digit_l1(d, l1d);
        if (gg) l1e = digit_l1(e, l1e);
#pragma unroll
        for (int k = 0; k < PCX_NDIG; k++) *(uint32_t*)(m.zD + o + (int64_t)k * gb * 16) = d[k];
        if (gg) {
#pragma unroll
            for (int k = 0; k < PCX_NDIG; k++) *(uint32_t*)(m.zE + o + (int64_t)k * gb * 16) = e[k];
        }
    }
#pragma unroll
    for (int k = 0; k < PCX_NDIG; k++) {  // the position's four quarters summed, one atomic
        int32_t t = dsum[k];
        t += __shfl_xor(t, 1, WAVE);
        t += __shfl_xor(t, 2, WAVE);
        if (live && h == 0 && t) atomicAdd((unsigned long long*)&m.dtok[(int64_t)k * gb + q], (unsigned long long)(int64_t)t);
    }
    // the guard's sums: the four quarters' fp64 sums added, then one fixed-point atomic each
    auto q4 = [](double v) {
        v += __shfl_xor(v, 1, WAVE);
        return v + __shfl_xor(v, 2, WAVE);
    };
    l1d += __shfl_xor(l1d, 1, WAVE);
    l1d += __shfl_xor(l1d, 2, WAVE);
    l1e += __shfl_xor(l1e, 1, WAVE);
    l1e += __shfl_xor(l1e, 2, WAVE);
    sd = q4(sd);
    sd2 = q4(sd2);
    se = q4(se);
    se2 = q4(se2);
    tok2 = q4(tok2);
    if (live && h == 0 && m.gacc) {
        int64_t* ga = m.gacc + q;
        if (l1d) atomicAdd((unsigned long long*)&ga[G_L1D * gb], (unsigned long long)(int64_t)l1d);
        guard_add(&ga[G_SD * gb], sd, false);
        guard_add(&ga[G_SD2 * gb], sd2, true);
        if (gg) {
            if (l1e) atomicAdd((unsigned long long*)&ga[G_L1E * gb], (unsigned long long)(int64_t)l1e);
            guard_add(&ga[G_SE * gb], se, false);
            guard_add(&ga[G_SE2 * gb], se2, true);
        }
    }
    if (live && h == 0 && q == 0 && m.gacc && tok2 > 0.0)  // sum tok^2 (exact: integers below 2^53)
        atomicAdd((unsigned long long*)&m.gacc[G_NSTAT * gb], (unsigned long long)(int64_t)tok2);
}

// The tok w digits alone (no zE to write: no general x general product on int8, or every token 1):
// one lane per position holding a whole 16-row group (16-byte stores; 2.66 ms at C5 against 3.8
// ms for the four-lane layout above, whose point is the register room for both strings).
__global__ void __launch_bounds__(BT) k_digits1(pcx_mat m) {
    const int gb = m.cov_jb * CT;
    const int q = blockIdx.x * BT + threadIdx.x;
    if (q >= gb) return;
    const double sc = m.dscale[q];
    const bool fg = m.cov_gg8 != 0;  // no wcd written: w = Fg - mu (k_wcd's own op)
    const double mu = fg ? m.ev[EV_MU * m.n_events + m.cov_perm[q]] : 0.0;
    const int64_t ng = m.wcd_rows / 16;
    const int64_t per = (ng + gridDim.y - 1) / gridDim.y;
    const int64_t g0 = blockIdx.y * per, g1 = g0 + per < ng ? g0 + per : ng;
    const int64_t ldd = zd_ld(gb);
    int32_t dsum[PCX_NDIG];  // |d| <= 127: int32-exact for any chunk under 16M rows
#pragma unroll
    for (int k = 0; k < PCX_NDIG; k++) dsum[k] = 0;
    int32_t l1 = 0;  // the guard's sums (guard_add)
    double sd = 0.0, sd2 = 0.0, tok2 = 0.0;
    for (int64_t grp = g0; grp < g1; grp++) {
        uint32_t d[PCX_NDIG][4];
#pragma unroll
        for (int k = 0; k < PCX_NDIG; k++) d[k][0] = d[k][1] = d[k][2] = d[k][3] = 0;
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int64_t i = grp * 16 + r;
            const double w = (fg ? m.Fg[i * gb + q] - mu : m.wcd[i * m.wcd_ld + q]) * sc;  // exact (power of two)
            const double tk = m.tokp[i];                                                    // 0 past n_rows
            double hi = w * tk, lo = fma(w, tk, -hi);  // tok w exactly
            const double pv = hi * DIG_SCALE, pe = fma(hi, DIG_SCALE, -pv), pl = fma(lo, DIG_SCALE, pe);
            double X = rint(pv + pl);
            const double dl = (X - pv) - pl;  // X - t (X - pv exact)
            sd = fma(dl, tk, sd);
            sd2 = fma(dl, dl, sd2);
            tok2 = fma(tk, tk, tok2);
#pragma unroll
            for (int k = PCX_NDIG - 1; k >= 0; k--) {  // (k_digits: the same digits)
                double di = X;
                if (k > 0) {
                    const double qd = rint(X * (1.0 / PCX_DBASE));
                    di = fma(-qd, PCX_DBASE, X);
                    X = qd;
                }
                d[k][r >> 2] |= (uint32_t)(uint8_t)(int8_t)(int)di << (8 * (r & 3));
                dsum[k] += (int)di;
            }
        }
#pragma unroll
        for (int k = 0; k < PCX_NDIG; k++)
            *(uint4*)(m.zD + ((grp * ldd) + (int64_t)k * gb + q) * 16) = uint4{d[k][0], d[k][1], d[k][2], d[k][3]};
        l1 = digit_l1(d, l1);
    }
#pragma unroll
    for (int k = 0; k < PCX_NDIG; k++)
        if (dsum[k]) atomicAdd((unsigned long long*)&m.dtok[(int64_t)k * gb + q], (unsigned long long)(int64_t)dsum[k]);
    if (m.gacc) {  // (one digit string: the guard derives the w digits' sums, k_cov_guard)
        int64_t* ga = m.gacc + q;
        if (l1) atomicAdd((unsigned long long*)&ga[G_L1D * gb], (unsigned long long)(int64_t)l1);
        guard_add(&ga[G_SD * gb], sd, false);
        guard_add(&ga[G_SD2 * gb], sd2, true);
        if (q == 0 && tok2 > 0.0)  // sum tok^2 (exact: integers below 2^53)
            atomicAdd((unsigned long long*)&m.gacc[G_NSTAT * gb], (unsigned long long)(int64_t)tok2);
    }
}

// plain loader for the Gram product of a symmetric E x E matrix (power-iteration squaring)
struct GramLoader {
    const double* A;
    int E;
    __device__ void load(int64_t i, int64_t re, int I, int J, int scg, double* va, double* vb) const {
        for (int k = 0; k < 8; k++) {
            const int qa = I * CT + scg + k, qb = J * CT + scg + k;
            va[k] = (i < re && qa < E) ? A[i * E + qa] : 0.0;
            vb[k] = (i < re && qb < E) ? A[i * E + qb] : 0.0;
        }
    }
};

// the power iteration's mode from the covariance flags of M_COV_REDUCE / M_COV_FINISH, read on the
// device so that M_POWER needs no host read before it launches: 0 iterate, 1 non-finite
// covariance (LAPACK raises, H = ones, :331-333), 2 zero covariance (svd(0): U = I)
__device__ __forceinline__ int pi_mode_of(int64_t flags) { return (flags & 2) ? 1 : (!(flags & 8) ? 2 : 0); }

// out = A^T A = A A (A symmetric), lower tiles mirrored; atomically tracks max |out| bits
// (nothing unless the power iteration runs: `flags` = &info[IN_FLAGS])
__global__ void __launch_bounds__(256) k_gram(const double* A, int E, double* out, unsigned long long* maxbits,
                                              const int64_t* flags) {
    if (pi_mode_of(*flags) != 0) return;
    int I, J;
    tri_index(blockIdx.x, I, J);
    GramLoader ld{A, E};
    d4 acc[4][4];
    mfma_tile(ld, I, J, 0, E, acc);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    double mx = 0.0;
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++)
            for (int r = 0; r < 4; r++) {
                const int p = I * CT + wr * 64 + a * 16 + (lane >> 4) + 4 * r;
                const int q = J * CT + wc * 64 + b * 16 + (lane & 15);
                if (p < E && q < E && q <= p) {
                    const double v = acc[a][b][r];
                    out[(int64_t)p * E + q] = v;
                    out[(int64_t)q * E + p] = v;
                    mx = fmax(mx, fabs(v));
                }
            }
    mx = wave_max_d(mx);
    if (lane == 0) atomicMax(maxbits, (unsigned long long)__double_as_longlong(mx));
}

// The same product split over the K (row) range for large E: tile t of the lower triangle, slice z
// of the rows -> slab[z] (a tile's own entries), then k_gram_reduce sums the slices in slice order.
// At E = 1000 the single-pass k_gram is 36 workgroups on 256 CUs (0.24 ms per squaring, three
// squarings per consensus); split 8 ways it fills the chip.
__global__ void __launch_bounds__(256) k_gram_part(const double* A, int E, double* slab, int ks,
                                                   const int64_t* flags) {
    if (pi_mode_of(*flags) != 0) return;
    const int t = blockIdx.x / ks, z = blockIdx.x % ks;
    int I, J;
    tri_index(t, I, J);
    const int64_t per = ((E + ks - 1) / ks + KB - 1) / KB * KB;
    const int64_t rb = (int64_t)z * per, re = rb + per < E ? rb + per : E;
    GramLoader ld{A, E};
    d4 acc[4][4];
    mfma_tile(ld, I, J, rb < E ? rb : E, re, acc);
    store_tile(slab + (int64_t)z * E * E, E, E, I, J, acc);
}

// 32 x 32 tiles of the lower triangle: the slices summed in order (coalesced over q), the tile
// mirrored through LDS so the upper half's stores are coalesced too
constexpr int GR_T = 32;
__global__ void __launch_bounds__(256) k_gram_reduce(const double* slab, int ks, int E, double* out,
                                                     unsigned long long* maxbits, const int64_t* flags) {
    if (pi_mode_of(*flags) != 0) return;
    __shared__ double t[GR_T][GR_T + 1];
    int I, J;
    tri_index(blockIdx.x, I, J);
    const int tx = threadIdx.x % GR_T, ty = threadIdx.x / GR_T;  // 32 x 8
    const int64_t n2 = (int64_t)E * E;
    double mx = 0.0;
    for (int r = ty; r < GR_T; r += 256 / GR_T) {
        const int64_t p = (int64_t)I * GR_T + r, q = (int64_t)J * GR_T + tx;
        double v = 0.0;
        if (p < E && q <= p) {
            const int64_t o = p * E + q;
            v = slab[o];
            for (int z = 1; z < ks; z++) v += slab[(int64_t)z * n2 + o];
            out[o] = v;
            mx = fmax(mx, fabs(v));
        }
        t[r][tx] = v;
    }
    __syncthreads();
    for (int r = ty; r < GR_T; r += 256 / GR_T) {  // out[q][p] = out[p][q], coalesced over p
        const int64_t q = (int64_t)J * GR_T + r, p = (int64_t)I * GR_T + tx;
        if (p < E && q < p) out[q * E + p] = t[tx][r];
    }
    mx = wave_max_d(mx);
    if ((threadIdx.x & 63) == 0) atomicMax(maxbits, (unsigned long long)__double_as_longlong(mx));
}

__global__ void __launch_bounds__(BT) k_scale(double* M, int64_t n, const unsigned long long* maxbits,
                                              const int64_t* flags) {
    if (pi_mode_of(*flags) != 0) return;
    const double mx = __longlong_as_double(*maxbits);
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < n; i += (int64_t)gridDim.x * BT)
        M[i] = mx > 0.0 ? M[i] / mx : M[i];
}

__device__ __forceinline__ dd two_prod(double a, double b) {
    const double p = a * b;
    return fast_two_sum(p, fma(a, b, -p));
}

// PCX_M_COV_REDUCE: C = sum of slabs over the lower triangle of wcd positions, in event
// order (cov_perm) and mirrored (unnormalised).  Pure-grid entries hold the exact integer
// P_jk: C_jk = c_j c_k T + (c_j Z_k + c_k Z_j) / 2 + P_jk / 4 with this rank's T, Z, P
// (c = 1 - mu is exact for mu in [1, 2]), evaluated in double-double.
// exact int64 sum of one int32 entry over k-slice slabs (four chains: four loads in flight)
__device__ __forceinline__ int64_t slab_sum(const int32_t* P, int64_t slab, int ks) {
    int64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    int k = 0;
    for (; k + 4 <= ks; k += 4) {
        a0 += P[(int64_t)k * slab];
        a1 += P[(int64_t)(k + 1) * slab];
        a2 += P[(int64_t)(k + 2) * slab];
        a3 += P[(int64_t)(k + 3) * slab];
    }
    for (; k < ks; k++) a0 += P[(int64_t)k * slab];
    return (a0 + a1) + (a2 + a3);
}

// a / 254 in double-double: q1 = hi / 254, the remainder hi - 254 q1 is exact (fma)
__device__ __forceinline__ dd dd_div_base(dd a) {
    const double q1 = a.hi / PCX_DBASE;
    const double r = fma(-q1, PCX_DBASE, a.hi) + a.lo;
    return fast_two_sum(q1, r / PCX_DBASE);
}

// sum tok z_row w_q of the mixed block from its PCX_NDIG digit products: Horner in double-double
// over 1/254 (sum_k P_k 254^-(k+1)), times 2^e
__device__ __forceinline__ dd mixed_comb(const pcx_mat& m, int64_t row, int64_t q) {
    const int64_t gb = (int64_t)m.cov_jb * CT, ldm = PCX_NDIG * gb;
    const int32_t* P = m.Pmx + row * ldm + q;
    const int64_t slab = m.zq * ldm;
    dd a{(double)slab_sum(P + (PCX_NDIG - 1) * gb, slab, m.ks_mx), 0.0};
    for (int d = PCX_NDIG - 2; d >= 0; d--) a = dd_add(dd_div_base(a), dd{(double)slab_sum(P + d * gb, slab, m.ks_mx), 0.0});
    return dd_mul_d(dd_div_base(a), ldexp(1.0, -ilogb(m.dscale[q])));  // 2^e
}

// sum tok w_p w_q (q <= p < gb) from the general x general digit products (256-position tiles over
// each digit's gb positions: p's tile ta = p / 256): the pairs of each
// weight 254^-(s + 2) summed exactly in int64 (over the pairs i + j = s and the k-slices), Horner
// over 1/254 in double-double from the smallest weight up, times 2^(e_p + f_q).  Dropping the pairs
// i + j >= NDIG leaves < 5.2 254^-NDIG of the two bounds' product per row, beside the digits' own
// residue (2 x 0.52 x 254^-NDIG x 1/2): ~2e-14 of |tok w_p| |w_q|'s bound, exact sums otherwise
// (fp64 tiles: a rounding per multiply-add).
__device__ double gg_comb(const pcx_mat& m, int64_t p, int64_t q) {
    const int SMAX = m.gg_smax;  // PCX_NDIG - 1, or 2 PCX_NDIG - 2 once the guard asked for every pair
    const int nt = (m.cov_jb * CT + GT - 1) / GT;
    const int ta = (int)(p / GT), tb = (int)(q / GT), tl = ta * (ta + 1) / 2 + tb;
    const int64_t within = (p % GT) * GT + (q % GT), within_t = (q % GT) * GT + (p % GT);
    const bool sym = m.zE == m.zD;
    const int64_t kstride = gemm_i8x_slab(1, 0, 0, 0, nt) * (GT * GT);  // one k-slice's slabs
    dd a{0.0, 0.0};
    for (int sd = SMAX; sd >= 0; sd--) {
        int64_t t = 0;
        for (int i = 0; i <= sd && i < PCX_NDIG; i++) {
            const int j = sd - i;
            if (j >= PCX_NDIG) continue;  // (i + j = sd: every pair of this weight)
            // (one digit string: a diagonal tile's pair i > j is (j, i) transposed, never computed)
            if (sym && ta == tb && i > j)
                t += slab_sum(m.Pgx + gemm_i8x_slab(0, j, i, tl, nt) * (GT * GT) + within_t, kstride, m.ks_gx);
            else
                t += slab_sum(m.Pgx + gemm_i8x_slab(0, i, j, tl, nt) * (GT * GT) + within, kstride, m.ks_gx);
        }
        a = dd_add(sd == SMAX ? a : dd_div_base(a), dd{(double)t, 0.0});
    }
    a = dd_div_base(dd_div_base(a));  // the (s + 2): 254^-2 more
    // 2^(e_p + f_q) applied to the rounded value: the product of the two scales alone can overflow
    return ldexp(dd_to_double(a), -ilogb(m.dscale[p]) - ilogb(m.escale[q]));
}

// S_q = sum tok w_q of every general position (shared by all grid rows): k_digits' digit sums
// (exact), recombined like mixed_comb
__global__ void __launch_bounds__(BT) k_cov_tokrow(pcx_mat m, double* S) {
    const int64_t q = blockIdx.x * (int64_t)BT + threadIdx.x;
    const int64_t gb = (int64_t)m.cov_jb * CT;
    if (q >= gb) return;
    dd a{(double)m.dtok[(PCX_NDIG - 1) * gb + q], 0.0};
    for (int d = PCX_NDIG - 2; d >= 0; d--) a = dd_add(dd_div_base(a), dd{(double)m.dtok[d * gb + q], 0.0});
    st_dd(S + 2 * q, dd_mul_d(dd_div_base(a), ldexp(1.0, -ilogb(m.dscale[q]))));  // 2^e
}

// entry (p, q), q <= p, of the position-space lower triangle of this rank's unnormalised C
// (S: the token row's S_q in dd, k_cov_tokrow)
__device__ __forceinline__ double cov_entry(const pcx_mat& m, const double* S, int64_t p, int64_t q) {
    const int64_t E = m.n_events;
    const int64_t gb = (int64_t)m.cov_jb * CT;
    const int64_t cp = m.cov_perm[p], cq = m.cov_perm[q];
    if (m.cov_gg8 && p < gb) return gg_comb(m, p, q);  // general x general on int8 digits
    if (q < gb && (!m.cov_mixed || p < gb)) {  // fp64 tiles: the slabs of k_syrk
        const int64_t ld = m.fp_ld, sl = ld * ld;
        const double* cs = m.cslab + p * ld + q;
        double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;  // four chains: four loads in flight
        int k = 0;
        for (; k + 4 <= m.fp_ks; k += 4) {
            a0 += cs[(int64_t)k * sl];
            a1 += cs[(int64_t)(k + 1) * sl];
            a2 += cs[(int64_t)(k + 2) * sl];
            a3 += cs[(int64_t)(k + 3) * sl];
        }
        for (; k < m.fp_ks; k++) a0 += cs[(int64_t)k * sl];
        return (a0 + a1) + (a2 + a3);
    }
    if (q >= gb) {  // grid x grid: P from the int8 products
        const double P = (double)slab_sum(m.Pgg + (p - gb) * m.zq + (q - gb), m.zq * m.zq, m.ks_gg);
        // (T, mu, Z: per-position loads beside the slab chain)
        const double T = dd_to_double(ld_dd(m.scal + ((int64_t)m.rank * SS + SC_TOK) * 2));
        const double ap = 1.0 - m.ev[EV_MU * E + cp], aq = 1.0 - m.ev[EV_MU * E + cq];
        const double Zp = 0.5 * (double)m.zsum[cp], Zq = 0.5 * (double)m.zsum[cq];
        dd r = dd_mul_d(two_prod(ap, aq), T);
        r = dd_add(r, dd_add(two_prod(ap, Zq), two_prod(aq, Zp)));
        r = dd_add(r, dd{0.25 * P, 0.0});
        return dd_to_double(r);
    }
    if (p >= gb && m.cov_mixed) {
        // general q x grid p: sum tok w_q (c_p + z_p / 2) = c_p S_q + Q_pq / 2, with S_q (the
        // token column) and Q_pq = sum tok z_p w_q from the digit products, Horner in dd
        const dd Sq = ld_dd(S + 2 * q), Q = mixed_comb(m, p - gb, q);
        const double ap = 1.0 - m.ev[EV_MU * E + cp];
        return dd_to_double(dd_add(dd_mul_d(Sq, ap), dd_mul_d(Q, 0.5)));
    }
    return 0.0;
}

// PCX_M_COV_REDUCE: C in event order, both triangles, from this rank's slabs in one pass: one
// 32 x 32 tile of the position-space lower triangle per workgroup, written as C[cov_perm[p]]
// [cov_perm[q]] row by row and mirrored through LDS (positions rise with the event index inside
// the general and the grid group, so both stores are row segments).  One rank: divided by
// (sum tokens - 1) on the way (:326, else M_COV_FINISH after the exchange), and the power
// iteration's finite / non-zero flags are collected here (k_pi_check's job).
constexpr int CV_T = 32;
__global__ void __launch_bounds__(CV_T * 8) k_cov_assemble(pcx_mat m, const double* S, int finish) {
    const int64_t E = m.n_events;
    int I, J;
    tri_index(blockIdx.x, I, J);
    __shared__ double t[CV_T][CV_T + 1];
    const int tx = threadIdx.x % CV_T, ty = threadIdx.x / CV_T;
    const double denom = finish ? dd_to_double(scl(m, SC_TOK)) - 1.0 : 1.0;
    int nonfinite = 0, nonzero = 0;
    for (int r = ty; r < CV_T; r += 8) {
        const int64_t p = (int64_t)I * CV_T + r, q = (int64_t)J * CV_T + tx;
        double v = 0.0;
        if (p < E && q <= p) {
            v = cov_entry(m, S, p, q);
            if (finish) v = v / denom;
            m.C[(int64_t)m.cov_perm[p] * E + m.cov_perm[q]] = v;
            nonfinite |= !__builtin_isfinite(v);
            nonzero |= v != 0.0;
        }
        t[r][tx] = v;
    }
    __syncthreads();
    for (int r = ty; r < CV_T; r += 8) {  // (q, p) = (J*T + r, I*T + tx), q < p
        const int64_t q = (int64_t)J * CV_T + r, p = (int64_t)I * CV_T + tx;
        if (p < E && q < p) m.C[(int64_t)m.cov_perm[q] * E + m.cov_perm[p]] = t[tx][r];
    }
    if (finish) {
        nonfinite = __syncthreads_or(nonfinite);
        nonzero = __syncthreads_or(nonzero);
        if (threadIdx.x == 0 && (nonfinite || nonzero))
            atomicOr((unsigned long long*)&m.info[IN_FLAGS], (nonfinite ? 2ull : 0ull) | (nonzero ? 8ull : 0ull));
    }
}

// PCX_M_COV_FINISH: divide by (sum tokens - 1) (:326)
__global__ void __launch_bounds__(BT) k_cov_finish(pcx_mat m) {
    const int64_t E = m.n_events;
    const int64_t idx = blockIdx.x * (int64_t)BT + threadIdx.x;
    if (idx >= E * E) return;
    const double denom = dd_to_double(scl(m, SC_TOK)) - 1.0;
    m.C[idx] = m.C[idx] / denom;
}

// ------------------------------------------------------------------ the int8 covariance's guard
// The emulation's result for an entry with a general position differs from the covariance of the
// fp64 centred matrix (C~_pq = sum tok w_p w_q, w = fl(F - mu), :322-326) by, per row, the digit
// strings' residues and the dropped digit pairs.  With D = (tok w_p + delta) / S_p and E = (w_q +
// eta) / T_q the digit values (S = 2^e, T = 2^f; |delta| <= 0.52 254^-NDIG S per row):
//   (a) sum delta w_q: sum tok w_q ~ 0 (mu is the token-weighted mean), so for any c, sum delta w_q =
//       sum (delta - c tok) w_q + c sum tok w_q, and Cauchy-Schwarz (over the rows with tok >= 1; a row
//       with tok 0 has delta 0) gives |sum (delta - c tok) w_q| <= sqrt(sum (delta - c tok)^2 / tok)
//       sqrt(C~_qq) <= sqrt(sum (delta - c tok)^2) sqrt(C~_qq); with the best c = sum delta tok /
//       sum tok^2: |(a)| <= sqrt(V_p) sqrt(C~_qq) + |c| |sum tok w_q|, V_p = sum delta^2 -
//       (sum delta tok)^2 / sum tok^2 -- a constant residue (a column whose rows mostly share one
//       value, equal tokens) cancels here;
//   (b) sum tok w_p eta: likewise with V'_q = sum tok eta^2 - (sum tok eta)^2 / T;
//   (c) sum delta eta <= sqrt(sum delta^2) sqrt(sum tok eta^2);
//   (d) the dropped pairs i + j > smax: per row sum_{i >= 1} |d_i| 254^-(i+1) |tail of E past digit
//       smax - i| <= 0.502 254^-(smax+2) S T L1(d) (and the same with L1(e)), so over the rows
//       <= 0.502 254^-(smax+2) S_p T_q sqrt(L1d_p L1e_q) -- linear in the rows: this is the term a
//       column of equal values with a few outliers makes large (their digits sit far below the scale
//       the outliers set);
//   the mean's rounding: |sum tok w_q| <= min(T (|mu_q| 2^-50 + max|w_q| 2^-52), sqrt(T C~_qq)).
// Relative to sqrt(C_pp C_qq) each term is a product of per-position factors, so the bound R is a sum
// of products of their maxima.  (the general x grid block has (a) and the mean term only: z is exact.)
// R <= 2^-40 passes; otherwise the pairs i + j > smax are computed too (no (d): every digit product
// exact) when that alone brings R under 2^-40, else the general pairs go to fp64 (k_syrk).
constexpr double GUARD_EPS = 0x1p-40;

// gacc (int64, this rank) -> gsum (doubles) for the exchange; L1 exact, the others at 2^-24
__global__ void __launch_bounds__(BT) k_guard_stats(pcx_mat m) {
    const int64_t gb = (int64_t)m.cov_jb * CT, n = G_NSTAT * gb + 1;  // (+ sum tok^2)
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < n; i += (int64_t)gridDim.x * BT) {
        const double v = (double)m.gacc[i];
        m.gsum[i] = (i < 2 * gb || i == G_NSTAT * gb) ? v : v * (1.0 / G_FIX);
    }
}

__device__ __forceinline__ double blk_max_d(double v, double* lds) {
    v = wave_max_d(v);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) lds[wv] = v;
    __syncthreads();
    double r = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); k++) r = fmax(r, lds[k]);
    return r;
}

// one workgroup: R over every general position (and the grid positions' mean factor) from the
// final C (normalised: times sum tok - 1), gsum (all ranks) and the digit scales
__global__ void __launch_bounds__(1024) k_cov_guard(pcx_mat m) {
    __shared__ double lds[16];
    __shared__ int cnt;
    const int64_t E = m.n_events, gb = (int64_t)m.cov_jb * CT;
    const double T = dd_to_double(scl(m, SC_TOK)), denom = T - 1.0;
    const bool gg = m.cov_gg8 != 0, one = m.zE == m.zD;  // one digit string: every token maxtok = 2^k
    double maxtok = 0.0;
    for (int w = 0; w < m.world; w++) maxtok = fmax(maxtok, m.scal[((int64_t)w * SS + SC_MAXTOK) * 2]);
    // (the k_digits row chunks: each adds at most one 2^-24 unit of rounding per sum and rank)
    const double ferr = (double)m.world * 4096.0 / G_FIX;
    const double tok2 = m.gsum[G_NSTAT * gb];  // sum tok^2 over all rows and ranks (exact)
    const double b6 = 1.0 / DIG_SCALE;  // 254^-NDIG
    if (threadIdx.x == 0) cnt = 0;
    double rd = 0.0, re = 0.0, gd = 0.0, ge = 0.0, kd = 0.0, ke = 0.0, ad = 0.0, ae = 0.0, bg = 0.0, bq = 0.0;
    bool bad = !(denom != 0.0 && __builtin_isfinite(denom) && T > 0.0 && tok2 > 0.0);
    for (int64_t q = threadIdx.x; !bad && q < E; q += blockDim.x) {
        const int c = m.cov_perm[q];
        const double Cqq = m.C[(int64_t)c * E + c] * denom * (1.0 - 0x1p-40);
        const double mu = m.ev[EV_MU * E + c];
        if (q >= gb) {  // grid position: |F - mu| <= 1; a constant column's entries are exact zeros
            if (Cqq > 0.0) bq = fmax(bq, fmin(T * (fabs(mu) * 0x1p-50 + 0x1p-52) / sqrt(Cqq), sqrt(T)));
            continue;
        }
        const double S = 1.0 / m.dscale[q], Tq = gg ? 1.0 / m.escale[q] : 0.0;
        const double* g = m.gsum + q;
        // (one digit string: eta = delta in its units, every token maxtok: sum tok eta = sum delta tok,
        // sum tok eta^2 = maxtok sum delta^2)
        const double l1d = g[G_L1D * gb], sd = g[G_SD * gb], sd2 = g[G_SD2 * gb];
        const double l1e = one ? l1d : g[G_L1E * gb], se = one ? sd : g[G_SE * gb], se2 = one ? maxtok * sd2 : g[G_SE2 * gb];
        const double sdl = fmax(0.0, fabs(sd) - ferr), sel = fmax(0.0, fabs(se) - ferr);
        const double Vd = fmax(0.0, sd2 + ferr - sdl * sdl / tok2);
        const double Ve = fmax(0.0, se2 + ferr * (one ? maxtok : 1.0) - sel * sel / T);
        if (!(Cqq > 0.0) || !__builtin_isfinite(Cqq)) {
            // no spread: exact only when nothing was rounded or dropped
            if (l1d != 0.0 || sd2 != 0.0 || (gg && (l1e != 0.0 || se2 != 0.0)) || !__builtin_isfinite(Cqq)) bad = true;
            continue;
        }
        const double rC = 1.0 / sqrt(Cqq);
        const double rdq = b6 * S * sqrt(Vd) * rC, adq = b6 * S * (fabs(sd) + ferr) / tok2 * rC;
        double own = rdq;
        rd = fmax(rd, rdq);
        ad = fmax(ad, adq);
        const double bgq = fmin(T * (fabs(mu) * 0x1p-50 + (gg ? 0.5 * Tq : 0.5 * S) * 0x1p-52) * rC, sqrt(T));
        bg = fmax(bg, bgq);
        own += adq * bgq;
        if (gg) {
            const double req = b6 * Tq * sqrt(Ve) * rC, aeq = b6 * Tq * (fabs(se) + ferr) / T * rC;
            const double gdq = S * sqrt(l1d) * rC, geq = Tq * sqrt(l1e) * rC;
            const double kdq = S * sqrt(sd2 + ferr) * rC, keq = Tq * sqrt(se2 + ferr * (one ? maxtok : 1.0)) * rC;
            re = fmax(re, req);
            ae = fmax(ae, aeq);
            gd = fmax(gd, gdq);
            ge = fmax(ge, geq);
            kd = fmax(kd, kdq);
            ke = fmax(ke, keq);
            own += req + aeq * bgq + b6 * b6 * kdq * keq;
            if (m.gg_smax < 2 * PCX_NDIG - 2) own += 0.502 * pow(PCX_DBASE, -(double)(m.gg_smax + 2)) * gdq * geq;
        }
        if (!(own <= GUARD_EPS)) atomicAdd(&cnt, 1);
    }
    bad = __syncthreads_or(bad);
    rd = blk_max_d(rd, lds);
    re = blk_max_d(re, lds);
    gd = blk_max_d(gd, lds);
    ge = blk_max_d(ge, lds);
    kd = blk_max_d(kd, lds);
    ke = blk_max_d(ke, lds);
    ad = blk_max_d(ad, lds);
    ae = blk_max_d(ae, lds);
    bg = blk_max_d(bg, lds);
    bq = blk_max_d(bq, lds);
    if (threadIdx.x == 0) {
        // (a) + mean term over general and grid q; (b), (c), (d) over general pairs
        double R = rd + ad * fmax(bg, bq);
        double Rd = 0.0;
        if (gg) {
            R += re + ae * bg + b6 * b6 * kd * ke;
            if (m.gg_smax < 2 * PCX_NDIG - 2) Rd = 0.502 * pow(PCX_DBASE, -(double)(m.gg_smax + 2)) * gd * ge;
        }
        int mode = COV_GUARD_PASS;
        if (bad || !(R + Rd <= GUARD_EPS)) mode = (!bad && gg && Rd > 0.0 && R <= GUARD_EPS) ? COV_GUARD_PAIRS : COV_GUARD_FP64;
        const double bound = bad ? __builtin_inf() : R + Rd;
        m.info[IN_COV_GUARD] = mode;
        m.info[IN_COV_GUARD_COLS] = bad ? (int64_t)gb : cnt;
        m.info[IN_COV_GUARD_BOUND] = (int64_t)__double_as_longlong(bound);
    }
}

// PCX_M_WCD_REBUILD (the guard's fp64 fallback): wcd = F - mu wherever the fp64 tiles of the whole
// trapezoid (general x every position) read what k_wcd did not write -- the general positions from
// the compact Fg when cov_gg8 ran (k_wcd wrote no wcd), the grid positions from their 2-bit codes
// (F = 1 + z / 2 exactly, so F - mu is k_wcd's own subtraction); rows past n_rows 0
__global__ void __launch_bounds__(BT) k_wcd_rebuild(pcx_mat m, int general) {
    const int64_t E = m.n_events, gb = (int64_t)m.cov_jb * CT, ld = m.wcd_ld;
    const int64_t p = blockIdx.y * (int64_t)BT + threadIdx.x;
    if (p >= E || (!general && p < gb)) return;
    const double mu = m.ev[EV_MU * E + m.cov_perm[p]];
    const int64_t ng = m.wcd_rows / 16;
    for (int64_t g = blockIdx.x; g < ng; g += gridDim.x) {
        if (p < gb) {
#pragma unroll 4
            for (int r = 0; r < 16; r++) {
                const int64_t i = g * 16 + r;
                m.wcd[i * ld + p] = i < m.n_rows ? m.Fg[i * gb + p] - mu : 0.0;
            }
        } else {
            const uint32_t P = zb_packed(m)[g * m.zq + (p - gb)];
#pragma unroll 4
            for (int r = 0; r < 16; r++) {
                const int64_t i = g * 16 + r;
                m.wcd[i * ld + p] = i < m.n_rows ? (1.0 + 0.5 * (double)zpack_get(P, r)) - mu : 0.0;
            }
        }
    }
}

// ================================================================== power iteration
// pvec layout: [0..E) x, [E+64 .. 2E+64) y, scalars at pvec[3*(E+64) + k]
__device__ __forceinline__ double* pv_x(const pcx_mat& m) { return m.pvec; }
__device__ __forceinline__ double* pv_y(const pcx_mat& m) { return m.pvec + (m.n_events + 64); }
__device__ __forceinline__ double* pv_s(const pcx_mat& m) { return m.pvec + 3 * (m.n_events + 64); }

__global__ void __launch_bounds__(BT) k_pi_check(pcx_mat m) {
    const int64_t E = m.n_events;
    int nonfinite = 0, nonzero = 0;
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < E * E; i += (int64_t)gridDim.x * BT) {
        const double c = m.C[i];
        nonfinite |= !__builtin_isfinite(c);
        nonzero |= c != 0.0;
    }
    nonfinite = __syncthreads_or(nonfinite);
    nonzero = __syncthreads_or(nonzero);
    if (threadIdx.x == 0 && (nonfinite || nonzero))
        atomicOr((unsigned long long*)&m.info[IN_FLAGS], (nonfinite ? 2ull : 0ull) | (nonzero ? 8ull : 0ull));
}

// start vector: column of C with the largest diagonal entry (first), normalised
__global__ void __launch_bounds__(1024) k_pi_start(pcx_mat m) {
    __shared__ double sv[1024];
    __shared__ int si[1024];
    __shared__ dd lds[16];
    const int E = (int)m.n_events;
    if (pi_mode_of(m.info[IN_FLAGS]) != 0) {  // no iteration: the host's first poll sees "converged"
        if (threadIdx.x == 0) {
            pv_s(m)[0] = 0.0;
            pv_s(m)[1] = 1.0;
            pv_s(m)[2] = 0.0;
        }
        return;
    }
    double best = -__builtin_inf();
    int bi = 0;
    for (int j = threadIdx.x; j < E; j += 1024) {
        const double d = m.C[(int64_t)j * E + j];
        if (d > best) {
            best = d;
            bi = j;
        }
    }
    sv[threadIdx.x] = best;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int s = 512; s >= 1; s >>= 1) {
        if (threadIdx.x < s) {
            const double o = sv[threadIdx.x + s];
            const int oi = si[threadIdx.x + s];
            if (o > sv[threadIdx.x] || (o == sv[threadIdx.x] && oi < si[threadIdx.x])) {
                sv[threadIdx.x] = o;
                si[threadIdx.x] = oi;
            }
        }
        __syncthreads();
    }
    const int kd = si[0];
    acc2 a;
    for (int j = threadIdx.x; j < E; j += 1024) {
        const double x = m.C[(int64_t)j * E + kd];
        a.add(x * x);
    }
    const dd n2 = block_sum_dd<1024>(a.get(), lds);
    __shared__ double nrm;
    if (threadIdx.x == 0) nrm = sqrt(dd_to_double(n2));
    __syncthreads();
    for (int j = threadIdx.x; j < E; j += 1024) pv_x(m)[j] = m.C[(int64_t)j * E + kd] / nrm;
    if (threadIdx.x == 0) {  // delta, converged, steps (k_pi_norm)
        pv_s(m)[0] = 1.0;
        pv_s(m)[1] = 0.0;
        pv_s(m)[2] = 0.0;
    }
}

// pv_s slots of the power iteration: [0] delta = max |x_new - x_old| of the last step, [1] 1 once
// delta <= PI_TOL (later steps of the same batch return at once), [2] steps run
constexpr double PI_TOL_M = 1e-14;

// y = M x, one wavefront per row; nothing once the iteration has converged (honor_done)
__global__ void __launch_bounds__(BT) k_pi_gemv(pcx_mat m, const double* M, int honor_done) {
    const int E = (int)m.n_events;
    const int row = blockIdx.x * (BT / WAVE) + threadIdx.x / WAVE;
    const int lane = threadIdx.x % WAVE;
    if (row >= E || (honor_done && pv_s(m)[1] != 0.0) || pi_mode_of(m.info[IN_FLAGS]) != 0) return;
    const double* Cr = M + (int64_t)row * E;
    const double* x = pv_x(m);
    double acc = 0.0;
    for (int q = lane; q < E; q += WAVE) acc = fma(Cr[q], x[q], acc);
    acc = wave_sum_d(acc);
    if (lane == 0) pv_y(m)[row] = acc;
}

// The same for E > 1024 (the early-exit path, no golden pinned to its sum order) with E even:
// 16-byte loads, four independent chains per lane (the row loop had one dependent fma chain per
// lane: ~2.7 TB/s over the 134 MB of a 4096-event C)
__global__ void __launch_bounds__(BT) k_pi_gemv4(pcx_mat m, const double* M, int honor_done) {
    const int E = (int)m.n_events;
    const int row = blockIdx.x * (BT / WAVE) + threadIdx.x / WAVE;
    const int lane = threadIdx.x % WAVE;
    if (row >= E || (honor_done && pv_s(m)[1] != 0.0) || pi_mode_of(m.info[IN_FLAGS]) != 0) return;
    const double2* Cr = reinterpret_cast<const double2*>(M + (int64_t)row * E);
    const double2* x = reinterpret_cast<const double2*>(pv_x(m));
    const int h = E / 2;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int q = lane;
    for (; q + 3 * WAVE < h; q += 4 * WAVE) {
        const double2 c0 = Cr[q], c1 = Cr[q + WAVE], c2 = Cr[q + 2 * WAVE], c3 = Cr[q + 3 * WAVE];
        const double2 x0 = x[q], x1 = x[q + WAVE], x2 = x[q + 2 * WAVE], x3 = x[q + 3 * WAVE];
        a0 = fma(c0.y, x0.y, fma(c0.x, x0.x, a0));
        a1 = fma(c1.y, x1.y, fma(c1.x, x1.x, a1));
        a2 = fma(c2.y, x2.y, fma(c2.x, x2.x, a2));
        a3 = fma(c3.y, x3.y, fma(c3.x, x3.x, a3));
    }
    for (; q < h; q += WAVE) {
        const double2 c0 = Cr[q], x0 = x[q];
        a0 = fma(c0.y, x0.y, fma(c0.x, x0.x, a0));
    }
    const double acc = wave_sum_d((a0 + a1) + (a2 + a3));
    if (lane == 0) pv_y(m)[row] = acc;
}

// x <- y / |y|; delta = max |x_new - x_old|  (pv_s[0] = delta, [1] converged, [2] steps)
__global__ void __launch_bounds__(1024) k_pi_norm(pcx_mat m, int honor_done) {
    __shared__ dd lds[16];
    __shared__ double red[1024];
    __shared__ double nrm;
    const int E = (int)m.n_events;
    if (honor_done && pv_s(m)[1] != 0.0) return;  // (uniform: every thread reads the same flag)
    if (pi_mode_of(m.info[IN_FLAGS]) != 0) return;
    acc2 a;
    for (int j = threadIdx.x; j < E; j += 1024) {
        const double y = pv_y(m)[j];
        a.add(y * y);
    }
    const dd n2 = block_sum_dd<1024>(a.get(), lds);
    if (threadIdx.x == 0) nrm = sqrt(dd_to_double(n2));
    __syncthreads();
    double d = 0.0;
    for (int j = threadIdx.x; j < E; j += 1024) {
        const double xn = pv_y(m)[j] / nrm;
        d = fmax(d, fabs(xn - pv_x(m)[j]));
        pv_x(m)[j] = xn;
    }
    red[threadIdx.x] = d;
    __syncthreads();
    for (int s = 512; s >= 1; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        pv_s(m)[0] = red[0];
        pv_s(m)[2] += 1.0;
        if (honor_done && red[0] <= PI_TOL_M) pv_s(m)[1] = 1.0;
    }
}

// loading (:336): sign rule of the batched SPEC, then v / sqrt(sum v^2)
// (also the step count and flags of the result: info[IN_PI_ITERS], info[IN_FLAGS] = svd-fail 2 /
// zero-covariance 1 / the host's iteration-cap bit 4 -- no host write, no sync after M_POWER)
__global__ void __launch_bounds__(1024) k_pi_finish(pcx_mat m, int64_t iters, int64_t maxit_flag) {
    __shared__ dd lds[16];
    __shared__ int first_nz, nnz, mode_s;
    __shared__ double scale;
    const int E = (int)m.n_events;
    double* x = pv_x(m);
    if (threadIdx.x == 0) {
        first_nz = E;
        nnz = 0;
        mode_s = pi_mode_of(m.info[IN_FLAGS]);
    }
    __syncthreads();
    const int mode = mode_s;
    if (threadIdx.x == 0) {  // (every thread has its mode: info[IN_FLAGS] may be rewritten)
        m.info[IN_PI_ITERS] = mode == 0 ? iters : 0;
        m.info[IN_FLAGS] = mode == 1 ? 2 : (mode == 2 ? 1 : maxit_flag);
    }
    for (int j = threadIdx.x; j < E; j += 1024) {
        double v = mode == 1 ? 1.0 : (mode == 2 ? (j == 0 ? 1.0 : 0.0) : x[j]);
        x[j] = v;
        if (v != 0.0) {
            atomicMin(&first_nz, j);
            atomicAdd(&nnz, 1);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 1.0;
        if (mode == 0 && first_nz < E) {
            const double xf = x[first_nz];
            const bool neg = nnz == 1 ? xf < 0.0 : xf > 0.0;
            s = neg ? -1.0 : 1.0;
        }
        scale = s;
    }
    __syncthreads();
    acc2 a;
    for (int j = threadIdx.x; j < E; j += 1024) {
        const double v = x[j] * scale;
        x[j] = v;
        a.add(v * v);
    }
    const dd n2 = block_sum_dd<1024>(a.get(), lds);
    __shared__ double nv;
    if (threadIdx.x == 0) nv = sqrt(dd_to_double(n2));
    __syncthreads();
    for (int j = threadIdx.x; j < E; j += 1024) m.ev[EV_LD * E + j] = x[j] / nv;
}

// ================================================================== row passes
// PCX_M_SCORES: s_i = sum_j wcd_ij * loading_j (:337), one wavefront per row;
// per-row NaN / zero counts; min/max keys of the scores.
// PCX_M_SCORES (PCA): scores = wcd . loading (:337) from the materialised wcd (the
// same f - mu values the covariance used), one wave per row, 16-byte loads; row NaN /
// zero counts from k_wcd's column-block partials.
__global__ void __launch_bounds__(BT) k_scores_wcd(pcx_mat m) {
    const int lane = threadIdx.x % WAVE;
    const int64_t ld = m.wcd_ld;
    const int ncb = (int)((ld + WCD_COLS - 1) / WCD_COLS);
    // PCA: the first loading; big-five / fixed-variance: the eigenvalue-weighted sum of the
    // sign-normalised loadings (PCX_M_EIG), i.e. net_score = wcd . g (:377-382, :435-440)
    const double* LD = m.ev + (m.algorithm == 0 ? EV_LD : EV_SPARE) * m.n_events;
    const int64_t row0 = blockIdx.x * (int64_t)(BT / WAVE) + threadIdx.x / WAVE;
    uint64_t kmin = ~0ull, kmax = 0;
    bool anynan = false;
    for (int64_t i = row0; i < m.n_rows; i += (int64_t)gridDim.x * (BT / WAVE)) {
        const double* w = m.wcd + i * ld;
        double acc = 0.0;
#pragma unroll 4
        for (int c = 2 * lane; c < ld; c += 2 * WAVE) {  // wcd positions (M_COV_PLAN order)
            const double2 x = *(const double2*)(w + c);
            const int e0 = m.cov_perm[c], e1 = m.cov_perm[c + 1];
            const double v0 = e0 >= 0 ? LD[e0] : 0.0;
            const double v1 = e1 >= 0 ? LD[e1] : 0.0;
            acc = fma(x.x, v0, acc);
            acc = fma(x.y, v1, acc);
        }
        acc = wave_sum_d(acc);
        if (lane < 2) {
            uint32_t t = 0;
            for (int b = 0; b < ncb; b++) t += m.rowpart[((int64_t)b * m.wcd_rows + i) * 2 + lane];
            m.rowstat[2 * i + lane] = t;
        }
        if (lane == 0) m.rowv[RV_S * m.n_rows + i] = acc;
        if (__builtin_isnan(acc)) anynan = true;
        const uint64_t k = dkey(acc);
        kmin = k < kmin ? k : kmin;
        kmax = k > kmax ? k : kmax;
    }
    if (lane == 0) {
        uint64_t* sk = m.skey + (int64_t)m.rank * 4;
        atomicMin((unsigned long long*)&sk[0], (unsigned long long)kmin);
        atomicMax((unsigned long long*)&sk[1], (unsigned long long)kmax);
        if (anynan) atomicOr((unsigned long long*)&sk[2], 1ull);
    }
}

// k_scores_grid's per-call constants, once (one wave): the loading in wcd position order
// (ev[EV_LDP]) and K = sum_{q >= gb} c_q ld_q (ev[EV_K]).  Computed in every wave before, K's
// dependent gathers cost ~0.1 ms per wave -- the whole pass at a C5 shard's one group per wave.
__global__ void __launch_bounds__(WAVE) k_scores_prep(pcx_mat m) {
    const int lane = threadIdx.x;
    const int E = (int)m.n_events;
    const double* LD = m.ev + (m.algorithm == 0 ? EV_LD : EV_SPARE) * E;
    double* LDp = m.ev + EV_LDP * E;
    const int gb = m.cov_jb * CT, ng = E - gb;
    for (int q = lane; q < gb && q < E; q += WAVE) {
        const int c = m.cov_perm[q];
        LDp[q] = c >= 0 ? LD[c] : 0.0;
        m.ev[EV_MUP * E + q] = c >= 0 ? m.ev[EV_MU * E + c] : 0.0;  // mu in position order (cov_gg8: Fg - mu)
    }
    double kk = 0.0;
    for (int q = lane; q < ng; q += WAVE) {
        const int c = m.cov_perm[gb + q];
        const double l = LD[c];
        LDp[gb + q] = l;
        kk = fma(1.0 - m.ev[EV_MU * E + c], l, kk);
    }
    const double K = wave_sum_d(kk);
    if (lane == 0) m.ev[EV_K * E] = K;
}

// PCX_M_SCORES with mixed_int8 (wcd holds only the general positions): one wave per 16-row
// group; general positions from wcd, grid positions from the int8 codes, F - mu = c + z / 2:
//   s_i = sum_{q < gb} wcd_iq ld_q + K + (1/2) sum_{q >= gb} z_iq ld_q,  K = sum_{q >= gb} c_q ld_q
// (ld in position order and K from k_scores_prep)
__global__ void __launch_bounds__(BT) k_scores_grid(pcx_mat m) {
    const int lane = threadIdx.x % WAVE, wv = threadIdx.x / WAVE;
    const int64_t ld = m.wcd_ld;
    const int ncb = (int)((ld + WCD_COLS - 1) / WCD_COLS);
    const int E = (int)m.n_events;
    const double* LDp = m.ev + EV_LDP * E;
    const int gb = m.cov_jb * CT, ng = E - gb;
    const double K = m.ev[EV_K * E];
    uint64_t kmin = ~0ull, kmax = 0;
    bool anynan = false;
    const int64_t ngrp = (m.n_rows + 15) / 16;
    for (int64_t g = blockIdx.x * (int64_t)(BT / WAVE) + wv; g < ngrp; g += (int64_t)gridDim.x * (BT / WAVE)) {
        double a[16];
#pragma unroll
        for (int r = 0; r < 16; r++) a[r] = 0.0;
        if (m.cov_gg8) {  // no wcd written: F - mu from Fg (k_wcd's own subtraction, bit for bit)
            for (int q = lane; q < gb; q += WAVE) {
                const double l = LDp[q], mu = m.ev[EV_MUP * E + q];
                const double* f = m.Fg + g * 16 * gb + q;
#pragma unroll
                for (int r = 0; r < 16; r++) a[r] = fma(f[r * gb] - mu, l, a[r]);
            }
        } else {
            for (int q = lane; q < gb; q += WAVE) {
                const double l = LDp[q];
                const double* w = m.wcd + g * 16 * ld + q;
#pragma unroll
                for (int r = 0; r < 16; r++) a[r] = fma(w[r * ld], l, a[r]);
            }
        }
        double z[16];
#pragma unroll
        for (int r = 0; r < 16; r++) z[r] = 0.0;
        for (int q = lane; q < ng; q += WAVE) {
            const double l = LDp[gb + q];
            const uint32_t P = zb_packed(m)[g * m.zq + q];
#pragma unroll
            for (int r = 0; r < 16; r++) z[r] = fma((double)zpack_get(P, r), l, z[r]);
        }
        double mine = 0.0;
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const double sr = wave_sum_d(fma(0.5, z[r], a[r])) + K;
            if (lane == r) mine = sr;
        }
        const int64_t i = g * 16 + (lane & 15);
        if (lane < 16 && i < m.n_rows) {
            m.rowv[RV_S * m.n_rows + i] = mine;
            if (__builtin_isnan(mine)) anynan = true;
            const uint64_t k = dkey(mine);
            kmin = k < kmin ? k : kmin;
            kmax = k > kmax ? k : kmax;
        }
        if (lane < 32) {  // row NaN / zero counts from k_wcd's column-block partials
            const int64_t ir = g * 16 + (lane >> 1);
            if (ir < m.n_rows) {
                uint32_t t = 0;
                for (int b = 0; b < ncb; b++) t += m.rowpart[((int64_t)b * m.wcd_rows + ir) * 2 + (lane & 1)];
                m.rowstat[2 * ir + (lane & 1)] = t;
            }
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t a = (uint64_t)__shfl_xor((long long)kmin, o, WAVE);
        const uint64_t b = (uint64_t)__shfl_xor((long long)kmax, o, WAVE);
        kmin = a < kmin ? a : kmin;
        kmax = b > kmax ? b : kmax;
    }
    anynan = __ballot(anynan) != 0;
    if (lane == 0) {
        uint64_t* sk = m.skey + (int64_t)m.rank * 4;
        atomicMin((unsigned long long*)&sk[0], (unsigned long long)kmin);
        atomicMax((unsigned long long*)&sk[1], (unsigned long long)kmax);
        if (anynan) atomicOr((unsigned long long*)&sk[2], 1ull);
    }
}

__global__ void __launch_bounds__(BT) k_scores(pcx_mat m) {
    const int E = (int)m.n_events;
    const int lane = threadIdx.x % WAVE;
    const int64_t row0 = blockIdx.x * (int64_t)(BT / WAVE) + threadIdx.x / WAVE;
    uint64_t kmin = ~0ull, kmax = 0;
    bool anynan = false;
    for (int64_t i = row0; i < m.n_rows; i += (int64_t)gridDim.x * (BT / WAVE)) {
        double acc = 0.0;
        int nn = 0, nz = 0;
        for (int c = lane; c < E; c += WAVE) {
            const ColParam p = col_param(m, c, true);
            const double x = rescale(m.reports[i * E + c], p, m.int_dtype);
            nn += __builtin_isnan(x) ? 1 : 0;
            nz += x == 0.0 ? 1 : 0;
            const double f = missing(x) ? p.guess : x;
            if (m.algorithm == 0) acc = fma(f - p.mu, m.ev[EV_LD * E + c], acc);
        }
        acc = wave_sum_d(acc);
        if (m.scores_given) acc = m.aux_scores[i];  // cokurtosis (:455-457) / given scores
        for (int s = 32; s >= 1; s >>= 1) {
            nn += __shfl_xor(nn, s, WAVE);
            nz += __shfl_xor(nz, s, WAVE);
        }
        if (lane == 0) {
            m.rowv[RV_S * m.n_rows + i] = acc;
            m.rowstat[2 * i] = nn;
            m.rowstat[2 * i + 1] = nz;
        }
        if (__builtin_isnan(acc)) anynan = true;
        const uint64_t k = dkey(acc);
        kmin = k < kmin ? k : kmin;
        kmax = k > kmax ? k : kmax;
    }
    if (lane == 0) {
        uint64_t* sk = m.skey + (int64_t)m.rank * 4;
        atomicMin((unsigned long long*)&sk[0], (unsigned long long)kmin);
        atomicMax((unsigned long long*)&sk[1], (unsigned long long)kmax);
        if (anynan) atomicOr((unsigned long long*)&sk[2], 1ull);
    }
}

__global__ void k_skey_init(pcx_mat m) {
    uint64_t* sk = m.skey + (int64_t)m.rank * 4;
    sk[0] = ~0ull;
    sk[1] = 0;
    sk[2] = 0;
    sk[3] = 0;
}

__device__ __forceinline__ void score_minmax(const pcx_mat& m, double& mn, double& mx) {
    uint64_t kmin = ~0ull, kmax = 0, nan = 0;
    for (int w = 0; w < m.world; w++) {
        const uint64_t* sk = m.skey + (int64_t)w * 4;
        kmin = sk[0] < kmin ? sk[0] : kmin;
        kmax = sk[1] > kmax ? sk[1] : kmax;
        nan |= sk[2];
    }
    mn = nan ? __builtin_nan("") : dkey_inv(kmin);
    mx = nan ? __builtin_nan("") : dkey_inv(kmax);
}

// PCX_M_NCSUMS: sum |set1|, sum |set1|+1, sum |set2|, sum |set2|+1 (normalize, :244-249)
__global__ void __launch_bounds__(BT) k_ncsums(pcx_mat m) {
    __shared__ dd lds[8];
    double mn, mx;
    score_minmax(m, mn, mx);
    acc2 a1, a1p, a2, a2p;
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const double s = m.rowv[RV_S * m.n_rows + i];
        const double v1 = fabs(s + fabs(mn)), v2 = fabs(s - mx);
        a1.add(v1);
        a1p.add(v1 + 1.0);
        a2.add(v2);
        a2p.add(v2 + 1.0);
    }
    const dd r0 = block_sum_dd<BT>(a1.get(), lds), r1 = block_sum_dd<BT>(a1p.get(), lds);
    const dd r2 = block_sum_dd<BT>(a2.get(), lds), r3 = block_sum_dd<BT>(a2p.get(), lds);
    if (threadIdx.x == 0) {
        st_dd(m.spart + blockIdx.x * 8 + 0, r0);
        st_dd(m.spart + blockIdx.x * 8 + 2, r1);
        st_dd(m.spart + blockIdx.x * 8 + 4, r2);
        st_dd(m.spart + blockIdx.x * 8 + 6, r3);
    }
}

// normalize(set) weight of row i: |v| / sum |v| (or (|v|+1)/sum(|v|+1) when sum |v| == 0)
__device__ __forceinline__ double nweight(double v, double S, double Sp) {
    return S == 0.0 ? (v + 1.0) / Sp : v / S;
}

// PCX_M_GEMV2: d1 = normalize(set1) . F, d2 = normalize(set2) . F  (:492-493)
// row weights of the two candidate sets, normalize(set1) and normalize(set2) (:488-493),
// computed once per row (k_gemv2 reads them instead of dividing per element)
// the largest |w| of a weight vector as it is written (bits: a NaN's exceed inf's), for the int8-MFMA
// weighted counts' fixed-point scale: m.wdig's header word `slot` (zeroed once per call by the
// runner; 0: normalize(set1), 1: normalize(set2), 2: smooth_rep), one atomic per wave.  Every lane
// of the wave calls it.
enum wdig_slot { WD_N1 = 0, WD_N2, WD_SMOOTH };
__device__ __forceinline__ void wdig_note(const pcx_mat& m, int slot, uint64_t mx) {
#pragma unroll
    for (int d = WAVE / 2; d >= 1; d >>= 1) {
        const uint64_t o = (uint64_t)__shfl_xor((long long)mx, d, WAVE);
        mx = o > mx ? o : mx;
    }
    if (m.wdig && (threadIdx.x & (WAVE - 1)) == 0 && mx)
        atomicMax(reinterpret_cast<unsigned long long*>(m.wdig) + slot, (unsigned long long)mx);
}
__device__ __forceinline__ uint64_t abs_bits(double w) { return (uint64_t)__double_as_longlong(fabs(w)); }

__global__ void __launch_bounds__(BT) k_nweights(pcx_mat m) {
    double mn, mx;
    score_minmax(m, mn, mx);
    const double S1 = dd_to_double(scl(m, SC_A1)), S1p = dd_to_double(scl(m, SC_A1P));
    const double S2 = dd_to_double(scl(m, SC_A2)), S2p = dd_to_double(scl(m, SC_A2P));
    uint64_t m1 = 0, m2 = 0;
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const double s = m.rowv[RV_S * m.n_rows + i];
        const double a = nweight(fabs(s + fabs(mn)), S1, S1p), b = nweight(fabs(s - mx), S2, S2p);
        m.rowv[RV_N1 * m.n_rows + i] = a;
        m.rowv[RV_N2 * m.n_rows + i] = b;
        m1 = abs_bits(a) > m1 ? abs_bits(a) : m1;
        m2 = abs_bits(b) > m2 ? abs_bits(b) : m2;
    }
    wdig_note(m, WD_N1, m1);
    wdig_note(m, WD_N2, m2);
}

__global__ void __launch_bounds__(BT) k_gemv2(pcx_mat m) {
    const int c = blockIdx.x * BT + threadIdx.x;
    const int E = (int)m.n_events;
    if (c >= E) return;
    const ColParam p = col_param(m, c, true);
    int64_t r0, r1;
    row_range(m, r0, r1);
    acc2 a1, a2;
    struct V3 {
        double x, w1, w2;
    };
    rows_pipelined<PIPE_U>(
        r0, r1,
        [&](int64_t i) {
            return V3{m.reports[i * E + c], m.rowv[RV_N1 * m.n_rows + i], m.rowv[RV_N2 * m.n_rows + i]};
        },
        [&](int64_t, V3 v) {
            const double f = filled(v.x, p, m.int_dtype);
            a1.add_prod(v.w1, f);
            a2.add_prod(v.w2, f);
        });
    double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
    st_dd(pp + 0, a1.get());
    st_dd(pp + 2, a2.get());
}

// Subset sums of a 16-row group's weights for the grid positions' passes: byte j of a 2-bit code
// word (zpack layout) holds rows j, j + 4, j + 8, j + 12, so a lane's four code pairs of that byte
// select a subset of those four rows; entry 16 j + s of the wave's table is the sum of the subset s
// (bit k: row j + 4 k) in double-double (a two_sum chain: exact to ~2^-106 of the sum).  Lane l
// builds entry l.  A position then takes four table reads per byte instead of four per-row
// additions per quantity.
// (the lane's four weights come in wq[k] = wg[j + 4 k], j = lane / 16: loaded a group ahead by
// subset_load, so the table waits for no load)
struct SubW {
    double w[4];
};
// row groups whose subset tables a grid block of the compact passes builds at once (two per wave)
constexpr int SG_NG = 8;
__device__ __forceinline__ SubW subset_load(const double* wg) {
    const int j = (threadIdx.x & (WAVE - 1)) >> 4;
    return SubW{{wg[j], wg[j + 4], wg[j + 8], wg[j + 12]}};
}
__device__ __forceinline__ void subset_table(const SubW& wq, dd* tab) {
    const int l = threadIdx.x & (WAVE - 1), sb = l & 15;
    dd a{0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const dd t = two_sum(a.hi, (sb >> k) & 1 ? wq.w[k] : 0.0);
        a = dd{t.hi, a.lo + t.lo};
    }
    tab[l] = a;
}
// the 4-bit subset index of code byte bits at 0, 2, 4, 6 (x & 0x55)
__device__ __forceinline__ uint32_t sub4_even(uint32_t x) {
    x = (x | (x >> 1)) & 0x33u;
    return (x | (x >> 2)) & 0x0Fu;
}
// ... of missing-word bits j, j + 4, j + 8, j + 12
__device__ __forceinline__ uint32_t sub4_stride4(uint32_t M, int j) {
    uint32_t v = (M >> j) & 0x1111u;
    v = (v | (v >> 3)) & 0x0303u;
    return (v | (v >> 6)) & 0x0Fu;
}

#ifndef PCX_MF_ZBG  // (a build parameter for A/B runs: bit 0 the outcome sums, bit 1 the GEMV2 sums take zbg)
#define PCX_MF_ZBG 3
#endif
// m.wdig: a 256-byte header (the largest |w| bits of each weight vector, wdig_slot, written by the
// kernels that write the weights), then vector v's digits at 256 + v wcd_rows 16 bytes
__device__ __forceinline__ uint64_t* wdig_max(const pcx_mat& m) { return reinterpret_cast<uint64_t*>(m.wdig); }
__device__ __forceinline__ int8_t* wdig_vec(const pcx_mat& m, int v) { return m.wdig + 256 + (int64_t)v * m.wcd_rows * 16; }
__device__ __forceinline__ double wdig_maxabs(const pcx_mat& m, int v) {
    return __longlong_as_double((long long)wdig_max(m)[v]);
}
// the digit passes ran (m.wdig set by the host) and every weight of the vectors in header words s0, s1
// is finite
__device__ __forceinline__ bool wdig_ok(const pcx_mat& m, int s0, int s1 = -1) {
    if (!m.wdig) return false;
    return __builtin_isfinite(wdig_maxabs(m, s0)) && (s1 < 0 || __builtin_isfinite(wdig_maxabs(m, s1)));
}

// M_GEMV2 from the compact sources (m.compact): thread = one wcd position (general positions
// read the filled values Fg, grid positions F = 1 + z / 2 from the 2-bit codes), 16-row groups;
// the same per-row products and compensated sums as k_gemv2, into the same partial slots
// GRID: one launch for the general tile positions [0, gb), one for the grid ones [gb, E) -- the two
// loops differ in registers, and the general one (a latency-bound stream of Fg) keeps its occupancy
template <bool GRID>
__global__ void __launch_bounds__(BT) k_gemv2_c(pcx_mat m) {
    const int64_t gb = (int64_t)m.cov_jb * CT;
    const int q = (GRID ? (int)gb : 0) + blockIdx.x * BT + threadIdx.x;
    const int E = (int)m.n_events;
    if (GRID && wdig_ok(m, WD_N1, WD_N2)) return;  // (k_gemv2_mf summed them)
    int64_t r0, r1;
    row_range(m, r0, r1, 16);
    const double* n1 = m.rowv + RV_N1 * m.n_rows;
    const double* n2 = m.rowv + RV_N2 * m.n_rows;
    // grid positions: sum v F = S_v + (sum v z) / 2 (F = 1 + z / 2, v z exact), S_v the chunk's
    // weight totals (wave reductions, before any lane leaves) -- one compensated add per
    // element and weight vector instead of a compensated product
    dd S1{0.0, 0.0}, S2{0.0, 0.0};
    if (GRID) {
        S1 = chunk_sum_dd(n1, r0, r1);
        S2 = chunk_sum_dd(n2, r0, r1);
    }
    // (every wave of a grid block stays to the end: the block builds the subset tables together)
    if (!GRID && (q >= E || q >= gb)) return;
    if (!GRID && (PCX_MF_ZBG & 2) && q >= m.info[IN_COV_GENERAL] && m.zbg && wdig_ok(m, WD_N1, WD_N2)) return;  // (k_gemv2_mf: zbg)
    const bool live = q < E;
    const int c = live ? m.cov_perm[q] : -1;
    if (!GRID && c < 0) return;  // (padding)
    acc2 a1, a2;
    if constexpr (GRID) {
        // the subset tables of n1 and n2 for SG_NG row groups at a time, built by the block's four
        // waves together (the tables depend on the rows only: every wave used to build the same ones,
        // one group at a time, each behind a wave barrier), read by every wave after one block barrier
        __shared__ dd tabs[SG_NG][2][WAVE];
        const int wv = threadIdx.x / WAVE;
        const uint32_t* zb = zb_packed(m) + (live ? q - gb : 0);
        // whole 16-row groups, then the ragged tail
        const int64_t g0 = r0 / 16, gf = r1 / 16;
        uint32_t Pn = g0 < gf ? zb[g0 * m.zq] : 0u;
        if (__builtin_isfinite(S1.hi) && __builtin_isfinite(S2.hi)) {
            // subset tables (as k_outcomes_c): sum v z = sum over code bytes j of T1 + 2 T2, the
            // subset sums of the rows whose code is 1 / 2, compensated (a non-finite weight: the
            // per-row loop, whose NaN x 0 the result keeps)
            acc2 a1j[4], a2j[4];
            for (int64_t g = g0; g < gf; g += SG_NG) {  // (block-uniform)
                uint32_t Pg[SG_NG];
#pragma unroll
                for (int k = 0; k < SG_NG; k++) Pg[k] = zb[(g + k < gf ? g + k : gf - 1) * m.zq];
#pragma unroll
                for (int t = 0; t < SG_NG / (BT / WAVE); t++) {
                    const int kk = wv * (SG_NG / (BT / WAVE)) + t;
                    if (g + kk < gf) {
                        subset_table(subset_load(n1 + (g + kk) * 16), tabs[kk][0]);
                        subset_table(subset_load(n2 + (g + kk) * 16), tabs[kk][1]);
                    }
                }
                __syncthreads();
#pragma unroll
                for (int k = 0; k < SG_NG; k++) {
                    if (g + k >= gf) break;  // (block-uniform)
                    const uint32_t P = Pg[k];
                    const dd* t1 = tabs[k][0];
                    const dd* t2 = tabs[k][1];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t by = (P >> (8 * j)) & 0xFFu, lo = by & 0x55u, hi = (by >> 1) & 0x55u;
                        const int i1 = 16 * j + (int)sub4_even(lo & ~hi), i2 = 16 * j + (int)sub4_even(hi & ~lo);
                        const dd u1 = t1[i1], u2 = t1[i2], v1 = t2[i1], v2 = t2[i2];
                        a1j[j].add(u1.hi);
                        a1j[j].c += u1.lo;
                        a1j[j].add(2.0 * u2.hi);
                        a1j[j].c += 2.0 * u2.lo;
                        a2j[j].add(v1.hi);
                        a2j[j].c += v1.lo;
                        a2j[j].add(2.0 * v2.hi);
                        a2j[j].c += 2.0 * v2.lo;
                    }
                }
                __syncthreads();  // (the next batch's tables overwrite these)
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const dd x1 = a1j[j].get(), x2 = a2j[j].get();
                a1.add(x1.hi);
                a1.c += x1.lo;
                a2.add(x2.hi);
                a2.c += x2.lo;
            }
        } else {
            for (int64_t g = g0; g < gf; g++) {
                const uint32_t P = Pn;
                if (g + 1 < gf) Pn = zb[(g + 1) * m.zq];
                double w1[16], w2[16];
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    w1[r] = n1[g * 16 + r];
                    w2[r] = n2[g * 16 + r];
                }
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const double z = (double)zpack_get(P, r);
                    a1.add(w1[r] * z);
                    a2.add(w2[r] * z);
                }
            }
        }
        if (!live) return;
        if (r0 < r1 && gf * 16 < r1) {  // (r0 < r1: r0 is 16-aligned; an empty chunk capped at a ragged n_rows has none)
            const uint32_t P = zb[gf * m.zq];
            for (int64_t i = gf * 16; i < r1; i++) {
                const double z = (double)zpack_get(P, (int)(i - gf * 16));
                a1.add(n1[i] * z);
                a2.add(n2[i] * z);
            }
        }
        const dd Z1 = a1.get(), Z2 = a2.get();
        double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
        st_dd(pp + 0, dd_add(S1, dd{0.5 * Z1.hi, 0.5 * Z1.lo}));
        st_dd(pp + 2, dd_add(S2, dd{0.5 * Z2.hi, 0.5 * Z2.lo}));
        return;
    }
    (void)S1;
    (void)S2;
    struct V3 {
        double x, w1, w2;
    };
    rows_pipelined<PIPE_U>(  // (both weights loaded with the value: every load ahead of its use)
        r0, r1, [&](int64_t i) { return V3{m.Fg[i * gb + q], n1[i], n2[i]}; },
        [&](int64_t, V3 v) {
            a1.add_prod(v.w1, v.x);
            a2.add_prod(v.w2, v.x);
        });
    double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
    st_dd(pp + 0, a1.get());
    st_dd(pp + 2, a2.get());
}

// ob_order: the scalar sums of the reference in numpy's pairwise order, written over the dd
// totals of scal[rank] (one thread; N < 9216).  which 0: sum(rep) (np.mean(rep), :461, and
// np.ma.average's denominator, :317); 1: normalize(set1 / set2) totals (:244-249, :491-492);
// 2: normalize(nc * rep / mean) totals (:462)
__global__ void k_ob_sums(pcx_mat m, int which) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int64_t N = m.n_rows;
    double* sc = m.scal + (int64_t)m.rank * SS * 2;
    auto put = [&](int slot, double v) { st_dd(sc + slot * 2, dd{v, 0.0}); };
    if (which == 0) {
        put(SC_REP, pw_sum_dev([&](int64_t i) { return m.rep[i]; }, N));
    } else if (which == 1) {
        double mn, mx;
        score_minmax(m, mn, mx);
        const double* s = m.rowv + RV_S * N;
        put(SC_A1, pw_sum_dev([&](int64_t i) { return fabs(s[i] + fabs(mn)); }, N));
        put(SC_A1P, pw_sum_dev([&](int64_t i) { return fabs(s[i] + fabs(mn)) + 1.0; }, N));
        put(SC_A2, pw_sum_dev([&](int64_t i) { return fabs(s[i] - mx); }, N));
        put(SC_A2P, pw_sum_dev([&](int64_t i) { return fabs(s[i] - mx) + 1.0; }, N));
    } else {
        const double* u = m.rowv + RV_U * N;
        put(SC_U, pw_sum_dev([&](int64_t i) { return u[i]; }, N));
        put(SC_UP, pw_sum_dev([&](int64_t i) { return u[i] + 1.0; }, N));
    }
}

// PCX_M_DECIDE: ranks of old, new1, new2 (scipy rankdata 'average') and the rule (:487-500)
// PCX_M_DECIDE (:491-498): new1/new2, then the three average ranks (scipy rankdata),
// O(E^2) comparisons spread over E/256 blocks; the rank-distance sums are half-integers,
// so the blocks' partial sums add exactly in any order (atomicAdd).
__global__ void __launch_bounds__(BT) k_decide_prep(pcx_mat m) {
    const int E = (int)m.n_events;
    const double* old = m.ev + EV_OLD * E;
    double* n1 = m.ev + EV_D1 * E;   // new1 = normalize(set1) . F + 0.01 * old
    double* n2 = m.ev + EV_D2 * E;   // new2
    double* raw1 = m.pvec + 2 * (m.n_events + 64);  // normalize(set1) . F (continuous rule)
    double* raw2 = pv_y(m);                          // normalize(set2) . F
    const int c = blockIdx.x * BT + threadIdx.x;
    if (c == 0) pv_s(m)[8] = 0.0;
    if (c >= E) return;
    const double a = m.ob_order ? ob_col_dot(m, m.rowv + RV_N1 * m.n_rows, c) : dd_to_double(cst(m, c, 4));
    const double b = m.ob_order ? ob_col_dot(m, m.rowv + RV_N2 * m.n_rows, c) : dd_to_double(cst(m, c, 5));
    const double t = 0.01 * old[c];
    n1[c] = a + t;
    n2[c] = b + t;
    raw1[c] = a;
    raw2[c] = b;
}

// counts of smaller / equal values among one chunk of RK_CH events (blockIdx.y), added into
// cnt[E][6] (integers: any order); k_ranks then forms the average ranks
constexpr int RK_CH = 64;
__global__ void __launch_bounds__(BT) k_rank_counts(pcx_mat m, int* cnt) {
    __shared__ double so[RK_CH], sa[RK_CH], sb[RK_CH];
    const int E = (int)m.n_events;
    const double* old = m.ev + EV_OLD * E;
    const double* n1 = m.ev + EV_D1 * E;
    const double* n2 = m.ev + EV_D2 * E;
    const int k0 = blockIdx.y * RK_CH;
    const int kn = E - k0 < RK_CH ? E - k0 : RK_CH;
    for (int t = threadIdx.x; t < kn; t += BT) {
        so[t] = old[k0 + t];
        sa[t] = n1[k0 + t];
        sb[t] = n2[k0 + t];
    }
    __syncthreads();
    const int c = blockIdx.x * BT + threadIdx.x;
    if (c >= E) return;
    int lt0 = 0, eq0 = 0, lt1 = 0, eq1 = 0, lt2 = 0, eq2 = 0;
    const double o = old[c], a = n1[c], b = n2[c];
    for (int t = 0; t < kn; t++) {
        lt0 += so[t] < o;
        eq0 += so[t] == o;
        lt1 += sa[t] < a;
        eq1 += sa[t] == a;
        lt2 += sb[t] < b;
        eq2 += sb[t] == b;
    }
    int* q = cnt + (int64_t)c * 6;
    atomicAdd(q + 0, lt0);
    atomicAdd(q + 1, eq0);
    atomicAdd(q + 2, lt1);
    atomicAdd(q + 3, eq1);
    atomicAdd(q + 4, lt2);
    atomicAdd(q + 5, eq2);
}

__global__ void __launch_bounds__(BT) k_ranks(pcx_mat m, const int* cnt) {
    __shared__ double red[BT];
    const int E = (int)m.n_events;
    const int c = blockIdx.x * BT + threadIdx.x;
    double e = 0.0;
    if (c < E) {
        const int* q = cnt + (int64_t)c * 6;
        const double r0 = q[0] + (q[1] + 1) * 0.5, r1 = q[2] + (q[3] + 1) * 0.5, r2 = q[4] + (q[5] + 1) * 0.5;
        e = fabs(r1 - r0) - fabs(r2 - r0);
        // rankdata propagates NaN (every rank NaN): any NaN value makes the rule's sum NaN,
        // which the decision reads as "not < 0" (set2), as the reference does
        const double* ev = m.ev;
        if (__builtin_isnan(ev[EV_OLD * E + c]) || __builtin_isnan(ev[EV_D1 * E + c]) ||
            __builtin_isnan(ev[EV_D2 * E + c]))
            e = __builtin_nan("");
    }
    red[threadIdx.x] = e;
    __syncthreads();
    for (int st = BT / 2; st >= 1; st >>= 1) {
        if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(&pv_s(m)[8], red[0]);
}

__global__ void __launch_bounds__(1024) k_decide(pcx_mat m) {
    __shared__ dd lds[16];
    const int E = (int)m.n_events;
    const double* old = m.ev + EV_OLD * E;
    const double* raw1 = m.pvec + 2 * (m.n_events + 64);
    const double* raw2 = pv_y(m);
    const double ref = m.rank_rule ? pv_s(m)[8] : 0.0;  // no rank rule: nonconformity directly
    int branch, pick1;
    if (ref == 0 && m.ob_order) {  // np.sum((new - old)**2) pairwise (:480-481)
        __shared__ int pk;
        if (threadIdx.x == 0) {
            const double s1 = pw_sum_dev([&](int64_t c) { const double a = raw1[c] - old[c]; return a * a; }, E);
            const double s2 = pw_sum_dev([&](int64_t c) { const double b = raw2[c] - old[c]; return b * b; }, E);
            pk = (s1 - s2) <= 0 ? 1 : 0;
        }
        __syncthreads();
        pick1 = pk;
        branch = pick1 ? 3 : 4;
    } else if (ref == 0) {
        acc2 q1, q2;
        for (int c = threadIdx.x; c < E; c += 1024) {
            const double a = raw1[c] - old[c];
            const double b = raw2[c] - old[c];
            q1.add(a * a);
            q2.add(b * b);
        }
        const dd s1 = block_sum_dd<1024>(q1.get(), lds);
        const dd s2 = block_sum_dd<1024>(q2.get(), lds);
        __shared__ int pk;
        if (threadIdx.x == 0) pk = dd_to_double(dd_sub(s1, s2)) <= 0 ? 1 : 0;
        __syncthreads();
        pick1 = pk;
        branch = pick1 ? 3 : 4;
    } else {
        pick1 = ref < 0;
        branch = pick1 ? 1 : 2;
    }
    if (threadIdx.x == 0) {
        m.info[IN_BRANCH] = branch;
        m.info[IN_PICK1] = pick1;
    }
}

// PCX_M_REPU: u_i = |nc_i * (rep_i / mean(rep))| and its sums (:460-462)
__global__ void __launch_bounds__(BT) k_repu(pcx_mat m) {
    __shared__ dd lds[8];
    double mn, mx;
    score_minmax(m, mn, mx);
    const double mean = dd_to_double(scl(m, SC_REP)) / (double)m.n_total;
    const int pick1 = (int)m.info[IN_PICK1];
    acc2 a, ap;
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        double nc = 0.0;
        if (m.algorithm >= 5) {  // the clusterings: nc from the cluster sizes / distances
            nc = m.rowv[RV_N1 * m.n_rows + i];
        } else if (m.algorithm != 1) {  // "absolute": nc = 0 (Q13)
            const double s = m.rowv[RV_S * m.n_rows + i];
            nc = pick1 ? s + fabs(mn) : s - mx;
        }
        const double u = fabs(nc * (m.rep[i] / mean));
        m.rowv[RV_U * m.n_rows + i] = u;
        a.add(u);
        ap.add(u + 1.0);
    }
    const dd r0 = block_sum_dd<BT>(a.get(), lds), r1 = block_sum_dd<BT>(ap.get(), lds);
    if (threadIdx.x == 0) {
        st_dd(m.spart + blockIdx.x * 8 + 0, r0);
        st_dd(m.spart + blockIdx.x * 8 + 2, r1);
    }
}

// PCX_M_SMOOTH: this_rep = normalize(u); smooth_rep = alpha*this + (1-alpha)*rep (:460-472)
__global__ void __launch_bounds__(BT) k_smooth(pcx_mat m) {
    const double S = dd_to_double(scl(m, SC_U)), Sp = dd_to_double(scl(m, SC_UP));
    const double a = m.alpha, oma = 1.0 - m.alpha;
    uint64_t ms = 0;
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const double t = nweight(m.rowv[RV_U * m.n_rows + i], S, Sp);
        const double w = a * t + oma * m.rep[i];
        m.rowv[RV_THIS * m.n_rows + i] = t;
        m.rowv[RV_SMOOTH * m.n_rows + i] = w;
        ms = abs_bits(w) > ms ? abs_bits(w) : ms;
    }
    wdig_note(m, WD_SMOOTH, ms);
}

// PCX_M_OUTCOMES: smooth . F (:510), smooth . na (:559), certainty bins for binary events
__global__ void __launch_bounds__(BT) k_outcomes(pcx_mat m) {
    const int c = blockIdx.x * BT + threadIdx.x;
    const int E = (int)m.n_events;
    if (c >= E) return;
    const ColParam p = col_param(m, c, true);
    int64_t r0, r1;
    row_range(m, r0, r1);
    // raw (np.dot(smooth_rep, F), :510) decides the catch: compensated.  The participation and
    // certainty sums (:542, :558) are continuous outputs: plain sums (error ~N ulp << 1e-9)
    acc2 raw;
    double pc = 0, b1 = 0, b15 = 0, b2 = 0;
    double n1 = 0, n15 = 0, n2 = 0;
    rows_pipelined<PIPE_U>(
        r0, r1, [&](int64_t i) { return XW{m.reports[i * E + c], m.rowv[RV_SMOOTH * m.n_rows + i]}; },
        [&](int64_t, XW v) {
            const double x = rescale(v.x, p, m.int_dtype);
            const bool ms = missing(x);
            const double f = ms ? p.guess : x;
            const double w = v.w;
            raw.add_prod(w, f);
            pc += w * (ms ? 1.0 : 0.0);  // np.dot(smooth_rep, na_mat): a NaN weight propagates
            b1 += f == 1.0 ? w : 0.0;
            b15 += f == 1.5 ? w : 0.0;
            b2 += f == 2.0 ? w : 0.0;
            n1 += f == 1.0 ? 1.0 : 0.0;
            n15 += f == 1.5 ? 1.0 : 0.0;
            n2 += f == 2.0 ? 1.0 : 0.0;
        });
    double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
    st_dd(pp + 0, raw.get());
    st_dd(pp + 2, {pc, 0.0});
    st_dd(pp + 4, {b1, 0.0});
    st_dd(pp + 6, {b15, 0.0});
    st_dd(pp + 8, {b2, 0.0});
    st_dd(pp + 10, {n1, 0.0});
    st_dd(pp + 12, {n15, 0.0});
    st_dd(pp + 14, {n2, 0.0});
}

// M_OUTCOMES from the compact sources (m.compact): as k_gemv2_c, with the missing bits nam
// the general positions' (GRID false) and the grid positions' bodies; S: the chunk's weight total.
// tab: the calling wave's subset table (GRID); live: the lane holds a position (every lane of a
// grid wave runs the body: the table takes all 64)
template <bool GRID>
__device__ __forceinline__ void outcomes_c_body(const pcx_mat& m, int q, int64_t r0, int64_t r1, dd S, dd* tab,
                                                bool live, bool mf = false) {
    const int64_t gb = (int64_t)m.cov_jb * CT, ld = m.wcd_ld;
    const int E = (int)m.n_events;
    const double* sm = m.rowv + RV_SMOOTH * m.n_rows;
    const int c = live ? m.cov_perm[q] : -1;
    if (!GRID && live && c < 0) return;  // (padding: none below gb)
    acc2 raw;
    double pc = 0, b1 = 0, b15 = 0, b2 = 0;
    double n1 = 0, n15 = 0, n2 = 0;
    auto cell = [&](double f, double w, bool ms) {
        raw.add_prod(w, f);
        pc += w * (ms ? 1.0 : 0.0);  // np.dot(smooth_rep, na_mat): a NaN weight propagates
        b1 += f == 1.0 ? w : 0.0;
        b15 += f == 1.5 ? w : 0.0;
        b2 += f == 2.0 ? w : 0.0;
        n1 += f == 1.0 ? 1.0 : 0.0;
        n15 += f == 1.5 ? 1.0 : 0.0;
        n2 += f == 2.0 ? 1.0 : 0.0;
    };
    const bool general = !GRID;
    const int64_t qn = live ? q : 0;  // (a lane past the positions reads a valid word, unused)
    const bool scl = general && (!live || (m.scaled && m.scaled[c]));
    // (k_outcomes_mf took the scaled positions' missing rows and the grid events of the general tiles)
    if (mf && (scl || q >= ((PCX_MF_ZBG & 1) ? m.info[IN_COV_GENERAL] : gb))) return;
    if (general && __all(scl)) {  // (a wave of scaled events only: the subset tables need every lane)
        // a scaled event's raw is its weighted median (:520-523) and its certainty comes from
        // the selection (:540-546): only np.dot(smooth_rep, na_mat) (:559) is read here, from
        // the missing bits alone (no filled values), in the same row order and arithmetic
        // whole 16-row groups, four at a time (words and weights loaded together): the missing
        // rows' weight from the wave's subset table (four reads per group, four independent
        // sums); a group with a non-finite weight adds row by row, so that NaN x 0 reaches pc as
        // in np.dot.  (Row by row with the weights loaded per group this pass took 2.4 of
        // k_outcomes_c's 3.3 ms at C5 for a quarter of its positions: latency, not issue.)
        const int64_t g0 = r0 / 16, gf = r1 / 16;
        constexpr int GB = 4;
        double pcj[4] = {0, 0, 0, 0};
        for (int64_t g = g0; g < gf; g += GB) {
            uint32_t Mg[GB];
            SubW wg[GB];
#pragma unroll
            for (int k = 0; k < GB; k++) {
                const int64_t gk = g + k < gf ? g + k : gf - 1;
                Mg[k] = m.nam[gk * ld + qn];
                wg[k] = subset_load(sm + gk * 16);
            }
#pragma unroll
            for (int k = 0; k < GB; k++) {
                if (g + k >= gf) break;  // (wave-uniform)
                const uint32_t M = Mg[k];
                const bool fin = __builtin_isfinite(wg[k].w[0]) && __builtin_isfinite(wg[k].w[1]) &&
                                 __builtin_isfinite(wg[k].w[2]) && __builtin_isfinite(wg[k].w[3]);
                if (__all(fin)) {  // (wave-uniform)
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                    subset_table(wg[k], tab);
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
#pragma unroll
                    for (int j = 0; j < 4; j++) pcj[j] += tab[16 * j + sub4_stride4(M, j)].hi;
                } else {
                    const int64_t gg = g + k;
#pragma unroll
                    for (int r = 0; r < 16; r++) pcj[r & 3] += sm[gg * 16 + r] * (((M >> r) & 1u) ? 1.0 : 0.0);
                }
            }
        }
        pc = (pcj[0] + pcj[1]) + (pcj[2] + pcj[3]);
        if (!live) return;
        if (r0 < r1 && gf * 16 < r1) {  // the ragged tail (r0 < r1: r0 is 16-aligned)
            const uint32_t M = m.nam[gf * ld + q];
            for (int64_t i = gf * 16; i < r1; i++) pc += sm[i] * (((M >> (i - gf * 16)) & 1u) ? 1.0 : 0.0);
        }
        double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
        st_dd(pp + 2, {pc, 0.0});
        return;
    }
    if (scl) {  // a scaled event in a wave with other kinds of position: row by row
        if (!live) return;
        const int64_t g0 = r0 / 16, gf = r1 / 16;
        uint32_t Mn = g0 < gf ? m.nam[g0 * ld + q] : 0u;
        for (int64_t g = g0; g < gf; g++) {
            const uint32_t M = Mn;
            if (g + 1 < gf) Mn = m.nam[(g + 1) * ld + q];
            double w[16];
#pragma unroll
            for (int r = 0; r < 16; r++) w[r] = sm[g * 16 + r];
#pragma unroll
            for (int r = 0; r < 16; r++) pc += w[r] * (((M >> r) & 1u) ? 1.0 : 0.0);
        }
        if (r0 < r1 && gf * 16 < r1) {
            const uint32_t M = m.nam[gf * ld + q];
            for (int64_t i = gf * 16; i < r1; i++) pc += sm[i] * (((M >> (i - gf * 16)) & 1u) ? 1.0 : 0.0);
        }
        double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
        st_dd(pp + 2, {pc, 0.0});
        return;
    }
    if constexpr (GRID) {
        // grid event: F = 1 + z / 2, z in {0, 1, 2} from the 2-bit codes.  raw = sum w F =
        // S + (sum w z) / 2 with S = sum w over the chunk (the same for every column: one dd
        // sum per wave) and w z exact, so one compensated add per element replaces the
        // product's; b1 / b15 / b2 are the same plain row-order sums as the general path's
        // and the counts are popcounts of the code bits (code 1 = value 1.5, 2 = value 2)
        const uint32_t* zb = zb_packed(m) + (live ? q - gb : 0);
        acc2 zs;
        uint32_t c15 = 0, c2 = 0;
        auto row = [&](uint32_t z, double w, uint32_t ms) {
            zs.add(w * (double)z);
            pc += w * (ms ? 1.0 : 0.0);
            b1 += z == 0u ? w : 0.0;
            b15 += z == 1u ? w : 0.0;
            b2 += z == 2u ? w : 0.0;
        };
        // whole 16-row groups (the next group's code and missing words in flight during this
        // group's adds), then the ragged tail
        const int64_t g0 = r0 / 16, gf = r1 / 16;
        uint32_t Pn = 0, Mn = 0;
        if (g0 < gf) {
            Pn = zb[g0 * m.zq];
            Mn = m.nam[g0 * ld + qn];
        }
        if (__builtin_isfinite(S.hi)) {
            // subset tables (round 5): per code byte j, the weights of the rows whose code is 0, 1
            // or 2 and of the missing rows are four table reads; Σ w z = Σ_j (T1 + 2 T2) stays
            // compensated, b1 / b15 / b2 / pc are plain sums of the subset sums (np.dot / the
            // certainty sums: any order within rounding).  With a non-finite weight in the chunk
            // the per-row loop below keeps NaN × 0 propagating into pc as np.dot does.
            // four groups' words and weights loaded at once (one group ahead left every group
            // waiting on its loads: the pass is latency-bound, not issue-bound)
            constexpr int GB = 4;
            // one accumulator per code byte j: four independent chains (one chain of dependent
            // compensated adds per quantity held every wave on the fp64 latency: SQ_WAIT_INST_ANY
            // was half the wave cycles)
            acc2 zj[4];
            double b1j[4] = {0, 0, 0, 0}, b15j[4] = {0, 0, 0, 0}, b2j[4] = {0, 0, 0, 0}, pcj[4] = {0, 0, 0, 0};
            for (int64_t g = g0; g < gf; g += GB) {
                uint32_t Pg[GB], Mg[GB];
                SubW wg[GB];
#pragma unroll
                for (int k = 0; k < GB; k++) {
                    const int64_t gk = g + k < gf ? g + k : gf - 1;
                    Pg[k] = zb[gk * m.zq];
                    Mg[k] = m.nam[gk * ld + qn];
                    wg[k] = subset_load(sm + gk * 16);
                }
#pragma unroll
                for (int k = 0; k < GB; k++) {
                    if (g + k >= gf) break;  // (wave-uniform)
                    const uint32_t P = Pg[k], M = Mg[k];
                    __builtin_amdgcn_wave_barrier();  // the previous group's reads are done
                    asm volatile("" ::: "memory");
                    subset_table(wg[k], tab);
                    __builtin_amdgcn_wave_barrier();
                    asm volatile("" ::: "memory");
                    c15 += __popc(P & 0x55555555u);
                    c2 += __popc(P & 0xAAAAAAAAu);
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t by = (P >> (8 * j)) & 0xFFu, lo = by & 0x55u, hi = (by >> 1) & 0x55u;
                        const dd T0 = tab[16 * j + sub4_even(0x55u & ~(lo | hi))];
                        const dd T1 = tab[16 * j + sub4_even(lo & ~hi)];
                        const dd T2 = tab[16 * j + sub4_even(hi & ~lo)];
                        const dd TM = tab[16 * j + sub4_stride4(M, j)];
                        zj[j].add(T1.hi);
                        zj[j].c += T1.lo;
                        zj[j].add(2.0 * T2.hi);
                        zj[j].c += 2.0 * T2.lo;
                        b1j[j] += T0.hi;
                        b15j[j] += T1.hi;
                        b2j[j] += T2.hi;
                        pcj[j] += TM.hi;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const dd z = zj[j].get();
                zs.add(z.hi);
                zs.c += z.lo;
            }
            b1 = (b1j[0] + b1j[1]) + (b1j[2] + b1j[3]);
            b15 = (b15j[0] + b15j[1]) + (b15j[2] + b15j[3]);
            b2 = (b2j[0] + b2j[1]) + (b2j[2] + b2j[3]);
            pc = (pcj[0] + pcj[1]) + (pcj[2] + pcj[3]);
        } else {
            for (int64_t g = g0; g < gf; g++) {
                const uint32_t P = Pn, M = Mn;
                if (g + 1 < gf) {
                    Pn = zb[(g + 1) * m.zq];
                    Mn = m.nam[(g + 1) * ld + qn];
                }
                c15 += __popc(P & 0x55555555u);
                c2 += __popc(P & 0xAAAAAAAAu);
                double w[16];
#pragma unroll
                for (int r = 0; r < 16; r++) w[r] = sm[g * 16 + r];
#pragma unroll
                for (int r = 0; r < 16; r++) row(zpack_get(P, r), w[r], (M >> r) & 1u);
            }
        }
        if (!live) return;
        if (r0 < r1 && gf * 16 < r1) {  // (r0 < r1: r0 is 16-aligned; an empty chunk capped at a ragged n_rows has none)
            const uint32_t P = zb[gf * m.zq], M = m.nam[gf * ld + q];
            for (int64_t i = gf * 16; i < r1; i++) {
                const int r = (int)(i - gf * 16);
                const uint32_t z = zpack_get(P, r);
                c15 += z == 1u;
                c2 += z == 2u;
                row(z, sm[i], (M >> r) & 1u);
            }
        }
        const dd Z = zs.get();
        const double rows = (double)(r1 > r0 ? r1 - r0 : 0);
        n15 = (double)c15;
        n2 = (double)c2;
        n1 = rows - n15 - n2;
        double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
        st_dd(pp + 0, dd_add(S, dd{0.5 * Z.hi, 0.5 * Z.lo}));
        st_dd(pp + 2, {pc, 0.0});
        st_dd(pp + 4, {b1, 0.0});
        st_dd(pp + 6, {b15, 0.0});
        st_dd(pp + 8, {b2, 0.0});
        st_dd(pp + 10, {n1, 0.0});
        st_dd(pp + 12, {n15, 0.0});
        st_dd(pp + 14, {n2, 0.0});
        return;
    }
    (void)S;
    // a general binary event (off the grid): the filled values Fg
    for (int64_t g = r0 / 16; r0 < r1 && g * 16 < r1; g++) {  // (an empty range capped at a ragged n_rows)
        const uint32_t M = m.nam[g * ld + q];
        double fv[16], w[16];
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const bool in = g * 16 + r < r1;
            fv[r] = in ? m.Fg[(g * 16 + r) * gb + q] : 0.0;
            w[r] = in ? sm[g * 16 + r] : 0.0;
        }
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int64_t i = g * 16 + r;
            if (i < r1) cell(fv[r], w[r], (M >> r) & 1u);
        }
    }
    double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
    st_dd(pp + 0, raw.get());
    st_dd(pp + 2, {pc, 0.0});
    st_dd(pp + 4, {b1, 0.0});
    st_dd(pp + 6, {b15, 0.0});
    st_dd(pp + 8, {b2, 0.0});
    st_dd(pp + 10, {n1, 0.0});
    st_dd(pp + 12, {n15, 0.0});
    st_dd(pp + 14, {n2, 0.0});
}

// A block of grid positions only (the general tiles end at a multiple of 128, so at most one block
// per row chunk mixes the two): outcomes_c_body<true>'s finite-weight path with the subset tables of
// SG_NG row groups at a time built by the block's four waves together -- the tables depend on the
// rows only, and every wave used to build the same ones a group at a time, each behind a wave
// barrier.  The same reads and adds in the same order: bit-identical.
__device__ void outcomes_grid_block(const pcx_mat& m, int q, int64_t r0, int64_t r1, dd S, bool live) {
    __shared__ dd tabs[SG_NG][WAVE];
    const int64_t gb = (int64_t)m.cov_jb * CT, ld = m.wcd_ld;
    const int E = (int)m.n_events;
    const double* sm = m.rowv + RV_SMOOTH * m.n_rows;
    const int wv = threadIdx.x / WAVE;
    const int c = live ? m.cov_perm[q] : -1;
    const int64_t qn = live ? q : gb;
    const uint32_t* zb = zb_packed(m) + (qn - gb);
    acc2 zs;
    uint32_t c15 = 0, c2 = 0;
    double pc = 0, b1 = 0, b15 = 0, b2 = 0;
    const int64_t g0 = r0 / 16, gf = r1 / 16;
    acc2 zj[4];
    double b1j[4] = {0, 0, 0, 0}, b15j[4] = {0, 0, 0, 0}, b2j[4] = {0, 0, 0, 0}, pcj[4] = {0, 0, 0, 0};
    for (int64_t g = g0; g < gf; g += SG_NG) {  // (block-uniform)
        uint32_t Pg[SG_NG], Mg[SG_NG];
#pragma unroll
        for (int k = 0; k < SG_NG; k++) {
            const int64_t gk = g + k < gf ? g + k : gf - 1;
            Pg[k] = zb[gk * m.zq];
            Mg[k] = m.nam[gk * ld + qn];
        }
#pragma unroll
        for (int t = 0; t < SG_NG / (BT / WAVE); t++) {
            const int kk = wv * (SG_NG / (BT / WAVE)) + t;
            if (g + kk < gf) subset_table(subset_load(sm + (g + kk) * 16), tabs[kk]);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < SG_NG; k++) {
            if (g + k >= gf) break;  // (block-uniform)
            const uint32_t P = Pg[k], M = Mg[k];
            const dd* tab = tabs[k];
            c15 += __popc(P & 0x55555555u);
            c2 += __popc(P & 0xAAAAAAAAu);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t by = (P >> (8 * j)) & 0xFFu, lo = by & 0x55u, hi = (by >> 1) & 0x55u;
                const dd T0 = tab[16 * j + sub4_even(0x55u & ~(lo | hi))];
                const dd T1 = tab[16 * j + sub4_even(lo & ~hi)];
                const dd T2 = tab[16 * j + sub4_even(hi & ~lo)];
                const dd TM = tab[16 * j + sub4_stride4(M, j)];
                zj[j].add(T1.hi);
                zj[j].c += T1.lo;
                zj[j].add(2.0 * T2.hi);
                zj[j].c += 2.0 * T2.lo;
                b1j[j] += T0.hi;
                b15j[j] += T1.hi;
                b2j[j] += T2.hi;
                pcj[j] += TM.hi;
            }
        }
        __syncthreads();  // (the next batch's tables overwrite these)
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const dd z = zj[j].get();
        zs.add(z.hi);
        zs.c += z.lo;
    }
    b1 = (b1j[0] + b1j[1]) + (b1j[2] + b1j[3]);
    b15 = (b15j[0] + b15j[1]) + (b15j[2] + b15j[3]);
    b2 = (b2j[0] + b2j[1]) + (b2j[2] + b2j[3]);
    pc = (pcj[0] + pcj[1]) + (pcj[2] + pcj[3]);
    if (!live) return;
    if (r0 < r1 && gf * 16 < r1) {  // the ragged tail, row by row (as outcomes_c_body)
        const uint32_t P = zb[gf * m.zq], M = m.nam[gf * ld + q];
        for (int64_t i = gf * 16; i < r1; i++) {
            const int r = (int)(i - gf * 16);
            const uint32_t z = zpack_get(P, r);
            const double w = sm[i];
            c15 += z == 1u;
            c2 += z == 2u;
            zs.add(w * (double)z);
            pc += w * (((M >> r) & 1u) ? 1.0 : 0.0);
            b1 += z == 0u ? w : 0.0;
            b15 += z == 1u ? w : 0.0;
            b2 += z == 2u ? w : 0.0;
        }
    }
    const dd Z = zs.get();
    const double rows = (double)(r1 > r0 ? r1 - r0 : 0);
    const double n15 = (double)c15, n2 = (double)c2, n1 = rows - n15 - n2;
    double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
    st_dd(pp + 0, dd_add(S, dd{0.5 * Z.hi, 0.5 * Z.lo}));
    st_dd(pp + 2, {pc, 0.0});
    st_dd(pp + 4, {b1, 0.0});
    st_dd(pp + 6, {b15, 0.0});
    st_dd(pp + 8, {b2, 0.0});
    st_dd(pp + 10, {n1, 0.0});
    st_dd(pp + 12, {n15, 0.0});
    st_dd(pp + 14, {n2, 0.0});
}

// one launch over every position (unlike k_gemv2_c: here the general positions of a scaled event
// read only their missing bits, and the two ranges' blocks fill the chip together)
__global__ void __launch_bounds__(BT) k_outcomes_c(pcx_mat m) {
    const int64_t gb = (int64_t)m.cov_jb * CT;
    const int q = blockIdx.x * BT + threadIdx.x;
    // k_outcomes_mf ran (finite weights): what is left are the general binary positions
    const bool mf = wdig_ok(m, WD_SMOOTH);
    if (mf && (q & ~(WAVE - 1)) >= gb) return;  // (wave-uniform)
    int64_t r0, r1;
    row_range(m, r0, r1, 16);
    // the chunk's weight total for the grid positions, by every lane of a wave holding one
    // (before any lane leaves: the sum is a wave reduction)
    __shared__ dd tabs[BT / WAVE][WAVE];  // the grid waves' subset tables
    dd S{0.0, 0.0};
    if ((q | (WAVE - 1)) >= gb) S = chunk_sum_dd(m.rowv + RV_SMOOTH * m.n_rows, r0, r1);
    if ((int64_t)blockIdx.x * BT >= gb && __builtin_isfinite(S.hi)) {  // (block-uniform)
        outcomes_grid_block(m, q, r0, r1, S, q < m.n_events);
        return;
    }
    if ((q & ~(WAVE - 1)) >= m.n_events) return;  // (wave-uniform: a grid wave runs all its lanes)
    if (q >= gb)  // (gb is a multiple of 128: a wave is all grid or all general)
        outcomes_c_body<true>(m, q, r0, r1, S, tabs[threadIdx.x / WAVE], q < m.n_events);
    else
        outcomes_c_body<false>(m, q, r0, r1, S, tabs[threadIdx.x / WAVE], q < m.n_events, mf);
}

// ---- M_OUTCOMES on int8 MFMA.  Every sum of the pass over a grid position is a weighted count --
// sum w [z = 1] (b15), sum w [z = 2] (b2), sum w [missing] (pc) and the chunk's sum w (S), whence
// b1 = S - b15 - b2 and raw = S + (b15 + 2 b2) / 2 -- and a general scaled position needs pc only:
// a 0/1 matrix (positions x rows) times the weight vector.  The weights are held as fixed-point
// integers round(w 2^s) (|w| 2^s < 2^125: s from the rank's largest |w|), sixteen balanced base-256
// digits each (k_wdigits), so every 0/1 x digit product is an exact v_mfma_i32_16x16x64_i8 (16
// positions x 16 digits x 64 rows) and a chunk's sums are exact integers per digit (|sum| <= 128 x
// rows < 2^31: chunks of at most 2^24 rows), then one double-double per quantity.  Against the
// fp64 subset tables: the same sums to ~2^-100 of the largest weight (those were plain fp64 sums,
// raw a compensated one), the 0/1 operands unpacked from the 2-bit codes and the missing bits
// beside the MFMAs.  A non-finite weight (NaN x 0 must reach the sums as in np.dot) leaves the pass
// to k_outcomes_c.
__device__ __forceinline__ int wdig_scale(double mxw) { return mxw > 0.0 ? 124 - ilogb(mxw) : 0; }

// digits n = 0..15 of row i at wdig_vec(v)[(i / 16) 256 + 16 n + i % 16]: one 16-byte MFMA B fragment
// per (16 rows, digit); rows past n_rows (to the next multiple of 16) zero
__global__ void __launch_bounds__(BT) k_wdigits(pcx_mat m, const double* w, int v, int slot) {
    const double mxw = wdig_maxabs(m, slot);
    if (!__builtin_isfinite(mxw)) return;
    const int s = wdig_scale(mxw);
    int8_t* dst = wdig_vec(m, v);
    const int64_t rows = (m.n_rows + 15) / 16 * 16;
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < rows; i += (int64_t)gridDim.x * BT) {
        double t = i < m.n_rows ? rint(ldexp(w[i], s)) : 0.0;  // an integer, |t| < 2^125
        int8_t* o = dst + (i >> 4) * 256 + (i & 15);
        // t = sum d_n 256^n, d_n in [-128, 127]: every step exact (t mod 256 and (t - d) / 256 are
        // integers a double holds)
#pragma unroll
        for (int n = 0; n < 16; n++) {
            const double r = t - 256.0 * floor(t * (1.0 / 256.0));  // [0, 256)
            const double d = r >= 128.0 ? r - 256.0 : r;
            o[16 * n] = (int8_t)(int)d;
            t = (t - d) * (1.0 / 256.0);
        }
    }
}

// digit sums (lane: digit lc of four positions) -> the double-double of sum_n v_n 256^n 2^-s over
// the 16 lanes of the lane's row of the wave (every lane of that row gets it)
__device__ __forceinline__ dd wdig_value(int64_t v, int lc, int s) {
    dd a{ldexp((double)v, 8 * lc - s), 0.0};  // exact (|v| < 2^53)
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) a = dd_add(a, dd{__shfl_xor(a.hi, d, WAVE), __shfl_xor(a.lo, d, WAVE)});
    return a;
}

// the 0/1 fragment of a lane's 16 missing bits (byte r = bit r)
__device__ __forceinline__ v4i wdig_bits16(uint32_t M) {
    v4i z;
#pragma unroll
    for (int k = 0; k < 4; k++) z[k] = (int)((((M >> (4 * k)) & 0xFu) * 0x00204081u) & 0x01010101u);
    return z;
}

// The grid events the general tiles end with (positions [n_general, gb), fewer than 128: gb is the
// next multiple of 128) as 2-bit codes in zbg [row / 16][128] (the zpack layout of zB), from their
// filled values Fg -- on the grid by the plan -- for k_outcomes_mf / k_gemv2_mf.  Thread = (position,
// 16-row group); the lanes of a wave read consecutive positions of a row.  (Written inside k_wcd:
// the same C5 time on one box, 20.5 vs 20.2-20.6 ms, with two more VGPRs and 14 more scalar spills in
// its row loop; this pass reads 1 GB at C5.)
__global__ void __launch_bounds__(BT) k_zbg(pcx_mat m) {
    const int64_t gb = (int64_t)m.cov_jb * CT, ngen = m.info[IN_COV_GENERAL];
    const int64_t p = (gb - 128) + (threadIdx.x & 127), g = (int64_t)blockIdx.x * (BT / 128) + (threadIdx.x >> 7);
    if (p < ngen || p >= gb || g * 16 >= m.n_rows) return;
    uint32_t P = 0;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int64_t i = g * 16 + r;
        const double F = i < m.n_rows ? m.Fg[i * gb + p] : 1.0;
        P |= (F == 2.0 ? 2u : (F == 1.5 ? 1u : 0u)) * zpack_bit(r);
    }
    m.zbg[g * 128 + (p - (gb - 128))] = P;
}

// one wave per 16 positions and row chunk (the chunks of k_outcomes_c / k_col_finish); gb is a
// multiple of 128, so a wave's positions are all general or all grid
__global__ void __launch_bounds__(BT) k_outcomes_mf(pcx_mat m) {
    if (!wdig_ok(m, WD_SMOOTH)) return;
    const int sc = wdig_scale(wdig_maxabs(m, WD_SMOOTH));
    const int E = (int)m.n_events;
    const int64_t gb = (int64_t)m.cov_jb * CT, ld = m.wcd_ld;
    const int lane = threadIdx.x & (WAVE - 1), lc = lane & 15, lg = lane >> 4;
    const int q0 = (blockIdx.x * (BT / WAVE) + threadIdx.x / WAVE) * 16;
    if (q0 >= E) return;  // (wave-uniform)
    const bool grid = q0 >= gb;
    const int qa = q0 + lc;  // this lane's A row (position); lg: its 16-row group of the 64-row k-step
    const bool alive = qa < E;
    int64_t r0, r1;
    row_range(m, r0, r1, 16);
    // (an empty trailing chunk is [n_rows, n_rows): no group, also when n_rows % 16 != 0)
    const int64_t g0 = r0 / 16, gf = r0 < r1 ? (r1 + 15) / 16 : g0;
    const uint16_t* nm = m.nam + (alive ? qa : 0);
    const v4i* wd = reinterpret_cast<const v4i*>(wdig_vec(m, 0)) + lc;  // + 16 group: digit lc of 16 rows
    // positions [n_general, gb) of the general tiles hold grid events too (the general tiles end at a
    // multiple of 128): their codes come from zbg (k_wcd)
    const int64_t ngen = (PCX_MF_ZBG & 1) ? m.info[IN_COV_GENERAL] : gb;
    const bool lbin = !grid && alive && qa >= ngen;
    const bool full = grid || q0 + 15 >= ngen;  // (wave-uniform: the code sums run)
    const uint32_t* zsrc = grid && alive ? zb_packed(m) + (qa - gb) : (lbin ? m.zbg + (qa - (gb - 128)) : nullptr);
    const int64_t zst = grid ? m.zq : 128;
    constexpr uint32_t O = 0x01010101u, M2 = 0x03030303u;
    const v4i ones{(int)O, (int)O, (int)O, (int)O};
    v4i a1{0, 0, 0, 0}, a2{0, 0, 0, 0}, am{0, 0, 0, 0}, a0{0, 0, 0, 0};
    uint32_t c15 = 0, c2 = 0;
    // U k-steps' loads issued together, then their MFMAs (the loads' latency, not the MFMAs, is
    // the chain here)
    constexpr int U = 4;
    for (int64_t gs = g0; gs < gf; gs += 4 * U) {
        v4i B[U];
        uint32_t P[U], M[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t g = gs + 4 * u + lg;
            const bool in = g < gf;
            B[u] = in ? wd[g * 16] : v4i{0, 0, 0, 0};
            M[u] = in && alive ? (uint32_t)nm[g * ld] : 0u;
            P[u] = in && zsrc ? zsrc[g * zst] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (gs + 4 * u >= gf) break;  // (wave-uniform)
            am = __builtin_amdgcn_mfma_i32_16x16x64_i8(wdig_bits16(M[u]), B[u], am, 0, 0, 0);
            if (full) {
                v4i z1, z2;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t zk = (P[u] >> (2 * k)) & M2;
                    z1[k] = (int)(zk & O);
                    z2[k] = (int)((zk >> 1) & O);
                }
                a1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(z1, B[u], a1, 0, 0, 0);
                a2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(z2, B[u], a2, 0, 0, 0);
                a0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, B[u], a0, 0, 0, 0);
                c15 += __popc(P[u] & 0x55555555u);
                c2 += __popc(P[u] & 0xAAAAAAAAu);
            }
        }
    }
    // counts of position lc over the four row groups
    c15 += __shfl_xor(c15, 16, WAVE);
    c15 += __shfl_xor(c15, 32, WAVE);
    c2 += __shfl_xor(c2, 16, WAVE);
    c2 += __shfl_xor(c2, 32, WAVE);
    // D layout: lane (lc, lg) element r = position 4 lg + r, digit lc
    const double rows = (double)(r1 > r0 ? r1 - r0 : 0);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int p = 4 * lg + r, q = q0 + p;
        const dd pc = wdig_value(am[r], lc, sc);
        dd raw{0.0, 0.0}, b1{0.0, 0.0}, b15{0.0, 0.0}, b2{0.0, 0.0};
        uint32_t n15 = 0, n2 = 0;
        if (full) {  // (wave-uniform)
            const int64_t S = a0[r], v15 = a1[r], v2 = a2[r];
            raw = wdig_value(2 * S + v15 + 2 * v2, lc, sc + 1);  // (S + (b15 + 2 b2) / 2)
            b1 = wdig_value(S - v15 - v2, lc, sc);
            b15 = wdig_value(v15, lc, sc);
            b2 = wdig_value(v2, lc, sc);
            n15 = (uint32_t)__shfl((int)c15, p, WAVE);
            n2 = (uint32_t)__shfl((int)c2, p, WAVE);
        }
        if (lc != 0 || q >= E) continue;
        const int c = m.cov_perm[q];
        double* pp = m.part + ((int64_t)blockIdx.y * E + c) * 16;
        if (!grid && q < ngen) {  // (general off-grid binary positions: k_outcomes_c)
            if (m.scaled && m.scaled[c]) st_dd(pp + 2, {dd_to_double(pc), 0.0});
            continue;
        }
        st_dd(pp + 0, raw);
        st_dd(pp + 2, {dd_to_double(pc), 0.0});
        st_dd(pp + 4, {dd_to_double(b1), 0.0});
        st_dd(pp + 6, {dd_to_double(b15), 0.0});
        st_dd(pp + 8, {dd_to_double(b2), 0.0});
        st_dd(pp + 10, {rows - (double)n15 - (double)n2, 0.0});
        st_dd(pp + 12, {(double)n15, 0.0});
        st_dd(pp + 14, {(double)n2, 0.0});
    }
}

// M_GEMV2's grid positions on int8 MFMA (as k_outcomes_mf): sum v F = S_v + (sum v z) / 2 for the
// weight vectors v = normalize(set1), normalize(set2) -- the 2-bit codes z in {0, 1, 2} are the A
// operand as they are, the weights' digits (vectors 0 and 1) the B operands, and all-ones A rows give
// the chunk totals S_v
__global__ void __launch_bounds__(BT) k_gemv2_mf(pcx_mat m) {
    if (!wdig_ok(m, WD_N1, WD_N2)) return;
    const int s1 = wdig_scale(wdig_maxabs(m, WD_N1)), s2 = wdig_scale(wdig_maxabs(m, WD_N2));
    const int E = (int)m.n_events;
    const int64_t gb = (int64_t)m.cov_jb * CT;
    const int lane = threadIdx.x & (WAVE - 1), lc = lane & 15, lg = lane >> 4;
    // from the first 16 positions holding a grid event (the general tiles' tail [n_general, gb): zbg)
    const int64_t ngen = (PCX_MF_ZBG & 2) ? m.info[IN_COV_GENERAL] : gb;
    const int q0 = (int)(gb > ngen ? ngen / 16 * 16 : gb) + (blockIdx.x * (BT / WAVE) + threadIdx.x / WAVE) * 16;
    if (q0 >= E) return;  // (wave-uniform)
    const int qa = q0 + lc;
    const bool alive = qa < E && qa >= ngen;
    int64_t r0, r1;
    row_range(m, r0, r1, 16);
    // (an empty trailing chunk is [n_rows, n_rows): no group, also when n_rows % 16 != 0)
    const int64_t g0 = r0 / 16, gf = r0 < r1 ? (r1 + 15) / 16 : g0;
    const uint32_t* zb = !alive ? nullptr : (qa >= gb ? zb_packed(m) + (qa - gb) : m.zbg + (qa - (gb - 128)));
    const int64_t zst = qa >= gb ? m.zq : 128;
    const v4i* w1 = reinterpret_cast<const v4i*>(wdig_vec(m, 0)) + lc;
    const v4i* w2 = reinterpret_cast<const v4i*>(wdig_vec(m, 1)) + lc;
    constexpr uint32_t O = 0x01010101u, M2 = 0x03030303u;
    const v4i ones{(int)O, (int)O, (int)O, (int)O};
    v4i z1{0, 0, 0, 0}, z2{0, 0, 0, 0}, t1{0, 0, 0, 0}, t2{0, 0, 0, 0};
    constexpr int U = 4;
    for (int64_t gs = g0; gs < gf; gs += 4 * U) {
        v4i B1[U], B2[U];
        uint32_t P[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t g = gs + 4 * u + lg;
            const bool in = g < gf;
            B1[u] = in ? w1[g * 16] : v4i{0, 0, 0, 0};
            B2[u] = in ? w2[g * 16] : v4i{0, 0, 0, 0};
            P[u] = in && alive ? zb[g * zst] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (gs + 4 * u >= gf) break;  // (wave-uniform)
            v4i z;
#pragma unroll
            for (int k = 0; k < 4; k++) z[k] = (int)((P[u] >> (2 * k)) & M2);
            z1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(z, B1[u], z1, 0, 0, 0);
            z2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(z, B2[u], z2, 0, 0, 0);
            t1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, B1[u], t1, 0, 0, 0);
            t2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ones, B2[u], t2, 0, 0, 0);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int q = q0 + 4 * lg + r;
        const dd d1 = wdig_value(2 * (int64_t)t1[r] + z1[r], lc, s1 + 1);
        const dd d2 = wdig_value(2 * (int64_t)t2[r] + z2[r], lc, s2 + 1);
        if (lc != 0 || q >= E || q < ngen) continue;
        double* pp = m.part + ((int64_t)blockIdx.y * E + m.cov_perm[q]) * 16;
        st_dd(pp + 0, d1);
        st_dd(pp + 2, d2);
    }
}

// certainty of an event no reporter matched (:542): NaN on the PCA path (smooth_rep is a
// MaskedArray, Q11), 0.0 for the other algorithms (plain ndarray, builtin sum of nothing)
__device__ __forceinline__ double empty_certainty(const pcx_mat& m) {
    return m.algorithm == 0 ? __builtin_nan("") : 0.0;
}

// PCX_M_EVENTS: binary outcomes (:526-531), certainty of binary events (:540-546)
__global__ void __launch_bounds__(BT) k_events(pcx_mat m) {
    const int c = blockIdx.x * BT + threadIdx.x;
    const int E = (int)m.n_events;
    if (c >= E) return;
    const bool sc = m.scaled && m.scaled[c];
    m.ev[EV_PC * E + c] = 1.0 - dd_to_double(cst(m, c, 7));
    if (sc) return;  // scaled events: phase-2 median
    // np.dot(smooth_rep, F) (:510)
    const double raw = m.ob_order ? ob_col_dot(m, m.rowv + RV_SMOOTH * m.n_rows, c) : dd_to_double(cst(m, c, 6));
    const double adj = catch_value(raw, m.catch_tolerance);
    const int slot = adj == 1.0 ? 8 : (adj == 1.5 ? 9 : 10);
    const double cnt = dd_to_double(cst(m, c, slot + 3));
    m.ev[EV_RAW * E + c] = raw;
    m.ev[EV_ADJ * E + c] = adj;
    m.ev[EV_FIN * E + c] = adj;
    m.ev[EV_CERT * E + c] = cnt > 0 ? dd_to_double(cst(m, c, slot)) : empty_certainty(m);
}

// ================================================================== weighted median selection
// weightedstats.weighted_median (:303 over the present reports of a scaled event with
// weights rep/sum(rep); :520-523 over the filled column with smooth_rep) in three tiers:
//
//  1. exact selection: an order-preserving u64 key per value, weights as exact fixed-point
//     limbs; 8-bit histogram passes narrow the key range to the run of equal values where
//     the exact prefix crosses half the total.  Every per-rank partial reduces with a plain
//     SUM / MIN / MAX, so the result does not depend on the sharding.
//  2. equal weights (reputation=None: every weight of the column is one double): the
//     reference's float walk depends on the count alone, and pcx_seqsum.h replays it in
//     O(log n) -- crossing index k* and the DBL_EPSILON half test -- after which an exact
//     count selection fetches the k*-th value (and its predecessor for an exact half).
//  3. the exact crossing is decisive unless the prefix at either end of the run lies
//     within the sequential-sum error bound of half the total; such events (and dominant
//     weights at the bound) are "hard" and are replayed in the reference's own float order
//     (k_hard_*: gather in row order, sequential totals, (value, weight) sort, walk).
enum sel_word {
    SW_STATUS = 0,   // 0 done, 1 histogram pass pending, 2 dominant weight (first argmax row), 3 hard
    SW_LO, SW_HI, SW_SHIFT,           // current key range and bucket shift
    SW_BELOW0, SW_BELOW1, SW_BELOW2,  // exact weight before the range
    SW_TOT0, SW_TOT1, SW_TOT2,        // exact total weight
    SW_BELOW_MAX, SW_HAS_BELOW,       // largest key before the range
    SW_RESULT,                        // result bits (status 0)
    SW_WMAX,                          // max weight bits
    SW_MODE,                          // 0 weight walk, 1 count rank (equal weights)
    SW_NEED,                          // phase 1: the event has missing reports
    SW_COUNT,                         // elements
    SW_TARGET,                        // count mode: 0-based rank of the crossing element
    SW_CNT_BELOW,                     // count mode: elements before the range
    SW_HALF,                          // count mode: 1 exact half (mean with predecessor), 2 half at k*=1
    SW_INRANGE,                       // elements (all ranks) in [LO, HI] after the last step
    SW_CMODE,                         // 1: this rank's in-range elements are compacted in cbuf
    SW_GN, SW_GW0, SW_GW1, SW_GW2,    // phase 2, this rank: filled (missing) rows -- all at the fill
                                      // value -- count and raw weight limb sums, binned once per pass
    SW_WB0, SW_WB1,                   // first pass: the bucket window gathered into cbuf (sampled)
    SW_CERTN, SW_CW0, SW_CW1, SW_CW2, // phase 2, weight walk ended on one key: the elements (all ranks)
                                      // holding it and their exact weight -- the certainty (:540-546)
    SW_NWORDS
};
static_assert(SW_NWORDS <= SELS, "sel_state words");

__device__ __forceinline__ L3 ld_l3(const uint64_t* p) { return {p[0], p[1], p[2]}; }
__device__ __forceinline__ void st_l3(uint64_t* p, L3 v) {
    p[0] = v.a;
    p[1] = v.b;
    p[2] = v.c;
}
// x - y for x >= y (both normalised)
__device__ __forceinline__ L3 l3_sub(L3 x, L3 y) {
    const uint64_t M = (1ull << 43);
    uint64_t c = x.c, b = x.b, a = x.a;
    if (c < y.c) {
        c += M;
        if (b == 0) {
            b += M;
            a -= 1;
        }
        b -= 1;
    }
    c -= y.c;
    if (b < y.b) {
        b += M;
        a -= 1;
    }
    b -= y.b;
    a -= y.a;
    return l3_norm({a, b, c});
}
__device__ __forceinline__ L3 l3_absdiff(L3 x, L3 y) { return l3_cmp(x, y) >= 0 ? l3_sub(x, y) : l3_sub(y, x); }

// |2 P - T| within the sequential-sum error bound of T?  The reference's cumulative
// weights and midpoint are float sums of n terms (each <= (n-1) u sum|w|, weights >= 0;
// phase 1 also divides every weight by a float total): both sides move by < (2n + 2) u T.
// The bound doubles that and adds the weightedstats DBL_EPSILON test (weights sum to ~1).
__device__ __forceinline__ bool near_half(L3 P, L3 T, uint64_t n) {
    const double d = l3_to_double(l3_absdiff(l3_twice(P), T));
    const double t = l3_to_double(T);
    const double bound = t * ((4.0 * (double)n + 64.0) * 0x1p-53) + 16.0 * 0x1p-52;
    return d <= bound;
}

__device__ __forceinline__ XW sel_load(const pcx_mat& m, int s, int64_t i) {
    // phase 1 with reputation=None: every weight is rep = 1 / N (k_rep_local) -- not loaded
    if (m.sel_phase == 1 && !m.rep_raw) return XW{m.T[(int64_t)s * m.n_rows + i], 1.0 / (double)m.n_total};
    return XW{m.T[(int64_t)s * m.n_rows + i], m.sel_phase == 1 ? m.rep[i] : m.rowv[RV_SMOOTH * m.n_rows + i]};
}

__device__ __forceinline__ bool sel_decode(const pcx_mat& m, int s, XW v, double& x, double& w) {
    if (m.sel_phase == 1) {
        if (__builtin_isnan(v.x)) return false;
        x = v.x;
    } else {
        x = __builtin_isnan(v.x) ? m.ev[EV_GUESS * m.n_events + m.scaled_cols[s]] : v.x;
        if (__builtin_isnan(x)) return false;
    }
    w = v.w;
    return true;
}

__device__ __forceinline__ bool sel_elem(const pcx_mat& m, int s, int64_t i, double& x, double& w) {
    return sel_decode(m, s, sel_load(m, s, i), x, w);
}

__device__ __forceinline__ void sel_done(uint64_t* st, double r) {
    st[SW_RESULT] = __double_as_longlong(r);
    st[SW_STATUS] = 0;
}

// phase setup: which scaled events run a selection (phase 1: those with missing reports)
__global__ void __launch_bounds__(BT) k_sel_setup(pcx_mat m) {
    const int s = blockIdx.x * BT + threadIdx.x;
    if (s >= m.n_scaled) return;
    if (s == 0) m.info[IN_SEL_WLIMB] = 0;  // (k_sel_wlimbs ORs this phase's limb use in)
    uint64_t* st = m.sel_state + (int64_t)s * SELS;
    const int c = m.scaled_cols[s];
    const bool need = m.sel_phase == 1 ? m.ev[EV_MISS * m.n_events + c] > 0 : true;
    for (int k = 0; k < SELS; k++) st[k] = 0;
    st[SW_STATUS] = need ? 1 : 0;
    st[SW_NEED] = need ? 1 : 0;
    if (m.sel_phase == 2 || need) m.hard[c] = HARD_NONE;
}

__device__ __forceinline__ int shift_for(uint64_t lo, uint64_t hi) {
    const uint64_t d = hi - lo;
    if (d == 0) return 0;
    const int bits = 64 - __clzll(d);
    return bits > 8 ? bits - 8 : 0;
}

// PCX selection init: the key range of every needed event without reading the column --
// phase 1: the present values' extremes (M_COLSTATS, all ranks); phase 2: those and the fill
// value (every missing row takes it, :310-312).  The first histogram pass (sel_first) then
// covers that range and also collects what the reference's walk needs first: the exact total
// weight, the count, the weight extremes and the filled rows' sums.  reputation=None in
// phase 1: every weight is the same double, so that pass counts only (count mode).
__global__ void __launch_bounds__(BT) k_sel_range(pcx_mat m) {
    const int s = blockIdx.x * BT + threadIdx.x;
    if (s >= m.n_scaled) return;
    uint64_t* st = m.sel_state + (int64_t)s * SELS;
    if (st[SW_STATUS] != 1) return;
    const int E = (int)m.n_events;
    const int c = m.scaled_cols[s];
    double mn = m.ev[EV_MINX * E + c], mx = m.ev[EV_MAXX * E + c];
    if (m.sel_phase == 2 && m.ev[EV_MISS * E + c] > 0) {
        const double g = m.ev[EV_GUESS * E + c];
        if (!__builtin_isnan(g)) {
            mn = fmin(mn, g);
            mx = fmax(mx, g);
        }
    }
    uint64_t lo = 1, hi = 0;  // no element: an empty range
    if (mn <= mx) {
        lo = dkey(mn);
        hi = dkey(mx);
    }
    st[SW_LO] = lo;
    st[SW_HI] = hi;
    st[SW_SHIFT] = lo <= hi ? shift_for(lo, hi) : 0;
    st[SW_INRANGE] = 0;  // (with SW_COUNT = 0: the first pass never compacts)
    st[SW_COUNT] = 0;
    st[SW_MODE] = (m.sel_phase == 1 && !m.rep_raw) ? 1 : 0;
}


__device__ __forceinline__ void mark_hard(const pcx_mat& m, int s, uint64_t* st) {
    st[SW_STATUS] = 3;
    m.hard[m.scaled_cols[s]] = HARD_MEDIAN;
}

// start: totals of all ranks (already reduced); empty / no positive weight -> None (NaN);
// equal weights -> the reference's walk by pcx_seqsum.h, then a count selection; else the
// dominant-weight test (:any(w > midpoint)) and the exact weight selection
// The totals come from the first pass's histogram (all ranks, reduced): exact integer sums of
// its bucket counts and weight limbs, the extreme keys of its buckets; one thread per event of
// that pass (active index a), whose histogram row k_sel_step then narrows in the same pass.
// One wave per event: the lanes read the histogram row's buckets (coalesced) and reduce the
// exact integer totals and key extremes; lane 0 then decides.
__global__ void __launch_bounds__(BT) k_sel_start(pcx_mat m) {
    const int a = blockIdx.x * (BT / WAVE) + threadIdx.x / WAVE;
    const int lane = threadIdx.x % WAVE;
    if (a >= (int)m.info[IN_SEL_ACTIVE]) return;  // wave-uniform
    const int s = m.sel_act[a];
    uint64_t* st = m.sel_state + (int64_t)s * SELS;
    if (st[SW_STATUS] != 1) return;
    const bool wsum = st[SW_MODE] == 0;  // the first pass summed weight limbs
    const int64_t o = (int64_t)a * NB;
    uint64_t ta = 0, tb = 0, tc = 0, n = 0, kmin = ~0ull, kmax = 0;
    for (int b = lane; b < NB; b += WAVE) {
        const uint64_t c = m.hist_n[o + b];
        if (!c) continue;
        n += c;
        if (wsum) {
            ta += m.hist_w[(o + b) * 3 + 0];
            tb += m.hist_w[(o + b) * 3 + 1];
            tc += m.hist_w[(o + b) * 3 + 2];
        }
        const uint64_t bmin = ~m.hist_min[o + b];  // (stored complemented: one MAX reduce, pcx_internal.h)
        kmin = bmin < kmin ? bmin : kmin;
        kmax = m.hist_max[o + b] > kmax ? m.hist_max[o + b] : kmax;
    }
#pragma unroll
    for (int d = WAVE / 2; d >= 1; d >>= 1) {  // exact integer sums: any order
        ta += __shfl_xor(ta, d, WAVE);
        tb += __shfl_xor(tb, d, WAVE);
        tc += __shfl_xor(tc, d, WAVE);
        n += __shfl_xor(n, d, WAVE);
        const uint64_t omn = __shfl_xor(kmin, d, WAVE), omx = __shfl_xor(kmax, d, WAVE);
        kmin = omn < kmin ? omn : kmin;
        kmax = omx > kmax ? omx : kmax;
    }
    if (lane != 0) return;
    const uint64_t wminb = ~m.sel_imin[s * 2 + 1], wmaxb = m.sel_imax[s * 2 + 1];
    // weights outside [0, 2^8) -- a negative reputation (rep / sum(rep) keeps its sign,
    // __init__.py:142-145; smooth_rep inherits it, :472) or one above 256 times the total: the
    // exact limbs hold only [0, 2^8) (pcx_device.h to_limbs), so replay in the reference's order.
    // Over bit patterns (the MAX reduce): a sign bit, or [bits(256), bits(+inf)]; NaN keeps the
    // limb path (NaN limbs are zero, as the generic conversion gives).
    if (wsum && ((wmaxb >> 63) || (wmaxb >= 0x4070000000000000ull && wmaxb <= 0x7ff0000000000000ull))) {
        mark_hard(m, s, st);
        return;
    }
    // count mode known up front (equal weights): the total only needs to be nonzero
    const L3 tot = wsum ? l3_norm({ta, tb, tc}) : L3{n && wmaxb ? 1ull : 0ull, 0, 0};
    if (!wsum && wminb != wmaxb) {  // (cannot happen: reputation=None gives one weight) exact replay
        mark_hard(m, s, st);
        return;
    }
    st_l3(st + SW_TOT0, tot);
    st_l3(st + SW_BELOW0, {0, 0, 0});
    st[SW_BELOW_MAX] = 0;
    st[SW_HAS_BELOW] = 0;
    st[SW_CNT_BELOW] = 0;
    st[SW_WMAX] = wmaxb;
    st[SW_COUNT] = n;
    // SW_LO / SW_HI / SW_SHIFT stay the first pass's (k_sel_step narrows that histogram)
    st[SW_INRANGE] = n;
    if (n == 0 || !(tot.a | tot.b | tot.c)) {  // weighted_median returns None -> NaN
        sel_done(st, __builtin_nan(""));
        return;
    }
    if (wminb == wmaxb) {
        // equal weights: W0 = w (phase 1: w / sequential total, :294-302); mid = 0.5 * sum
        const double w = __longlong_as_double(wmaxb);
        const double W0 = m.sel_phase == 1 ? w / seqsum_const(w, (int64_t)n) : w;
        const double mid = 0.5 * seqsum_const(W0, (int64_t)n);
        if (W0 > mid) {  // dominant weight: data[first argmax] = the first element
            st[SW_STATUS] = 2;
            atomicAdd((unsigned long long*)&m.info[IN_SEL_ARGMAX], 1ull);
            return;
        }
        if (!(W0 > 0.0)) {
            sel_done(st, __builtin_nan(""));
            return;
        }
        const int64_t ks = seqsum_first_above(W0, mid, (int64_t)n);
        const double before = seqsum_const(W0, ks) - W0;
        const bool half = fabs(before - mid) < 2.220446049250313080847e-16;
        st[SW_MODE] = 1;
        st[SW_TARGET] = (uint64_t)(ks - 1);
        st[SW_HALF] = half ? (ks >= 2 ? 1 : (n == 1 ? 0 : 2)) : 0;
    } else {
        const L3 wmax = l3_of(__longlong_as_double(wmaxb));
        if (near_half(wmax, tot, n)) {
            mark_hard(m, s, st);
            return;
        }
        if (l3_cmp(l3_twice(wmax), tot) > 0) {  // any(w > mid)
            st[SW_STATUS] = 2;
            atomicAdd((unsigned long long*)&m.info[IN_SEL_ARGMAX], 1ull);
            return;
        }
        st[SW_MODE] = 0;
    }
    if (kmin == kmax) {  // one distinct value: every crossing returns it
        sel_done(st, st[SW_HALF] == 2 ? __builtin_nan("") : dkey_inv(kmin));
    }
}

// dominant weight: first global row (data order) holding the max weight -> sel_arg[s][0] (MIN)
__global__ void __launch_bounds__(BT) k_sel_argmax(pcx_mat m) {
    const int s = blockIdx.x;
    const uint64_t* st = m.sel_state + (int64_t)s * SELS;
    if (st[SW_STATUS] != 2) return;
    const uint64_t wmaxb = st[SW_WMAX];
    __shared__ unsigned long long best;
    if (threadIdx.x == 0) best = ~0ull;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < m.n_rows; i += BT) {
        double x, w;
        if (sel_elem(m, s, i, x, w) && (uint64_t)__double_as_longlong(w) == wmaxb) {
            atomicMin(&best, (unsigned long long)(m.row_offset + i));
            break;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        m.sel_arg[s] = best;
        m.sel_arg[m.n_scaled + s] = 0;
    }
}

// the rank owning that row publishes its value key -> sel_arg[s][1] (MAX)
__global__ void __launch_bounds__(BT) k_sel_value(pcx_mat m) {
    const int s = blockIdx.x * BT + threadIdx.x;
    if (s >= m.n_scaled) return;
    const uint64_t* st = m.sel_state + (int64_t)s * SELS;
    if (st[SW_STATUS] != 2) return;
    const uint64_t gi = m.sel_arg[s];
    uint64_t key = 0;
    if (gi != ~0ull && (int64_t)gi >= m.row_offset && (int64_t)gi < m.row_offset + m.n_rows) {
        double x, w;
        sel_elem(m, s, (int64_t)gi - m.row_offset, x, w);
        key = dkey(x);
    }
    m.sel_arg[m.n_scaled + s] = key;
}

__global__ void __launch_bounds__(BT) k_sel_value_finish(pcx_mat m) {
    const int s = blockIdx.x * BT + threadIdx.x;
    if (s >= m.n_scaled) return;
    uint64_t* st = m.sel_state + (int64_t)s * SELS;
    if (st[SW_STATUS] != 2) return;
    const uint64_t key = m.sel_arg[m.n_scaled + s];
    sel_done(st, key ? dkey_inv(key) : __builtin_nan(""));
}

// ordered compaction of [0, n) by pred into out[] (block-wide, order preserving); returns count
template <class PRED, class EMIT>
__device__ int64_t block_compact(int64_t n, PRED pred, EMIT emit) {
    __shared__ int wsum[16];
    __shared__ int64_t base_s;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
    if (tid == 0) base_s = 0;
    __syncthreads();
    for (int64_t c0 = 0; c0 < n; c0 += blockDim.x) {
        const int64_t i = c0 + tid;
        const bool p = i < n && pred(i);
        const uint64_t bal = __ballot(p);
        const int before_lane = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wv] = __popcll(bal);
        __syncthreads();
        int off = 0;
        for (int k = 0; k < wv; k++) off += wsum[k];
        const int64_t base = base_s;
        if (p) emit(i, base + off + before_lane);
        __syncthreads();
        if (tid == 0) {
            int t = 0;
            for (int k = 0; k < nw; k++) t += wsum[k];
            base_s = base + t;
        }
        __syncthreads();
    }
    return base_s;
}

// active events (status 1) in event order -> sel_act, count -> info[IN_SEL_ACTIVE]; how many
// of them walk weights (not counts) -> info[IN_SEL_WACTIVE] (their limb histograms are exchanged)
__global__ void __launch_bounds__(1024) k_sel_compact(pcx_mat m) {
    __shared__ unsigned long long nw;
    if (threadIdx.x == 0) nw = 0;
    __syncthreads();
    const int64_t cnt = block_compact(
        m.n_scaled, [&](int64_t s) { return m.sel_state[s * SELS + SW_STATUS] == 1; },
        [&](int64_t s, int64_t pos) {
            m.sel_act[pos] = (int32_t)s;
            if (m.sel_state[s * SELS + SW_MODE] == 0) atomicAdd(&nw, 1ull);
        });
    if (threadIdx.x == 0) {
        m.info[IN_SEL_ACTIVE] = cnt;
        m.info[IN_SEL_WACTIVE] = (int64_t)nw;
    }
    // and the events marked for the exact replay so far (k_hard_list's list): after the pass that
    // leaves no event active, the host's one read of info[IN_SEL_ACTIVE ..] also has their count
    if (m.hard_cols) {
        __syncthreads();  // (every thread has read block_compact's count before it is reset)
        const int64_t nh = block_compact(
            m.n_events, [&](int64_t c) { return m.hard[c] != HARD_NONE; },
            [&](int64_t c, int64_t pos) {
                m.hard_cols[pos] = (int32_t)c;
                m.hard_modes[pos] = m.hard[c];
            });
        if (threadIdx.x == 0) m.info[IN_HARD] = nh;
    }
}

// which of the three weight limbs any of this rank's rows uses in this phase (bit 0: L0, bit 2:
// L2; bit 3: computed) -> info[IN_SEL_WLIMB].  k_sel_hist skips the LDS sums of a limb that is zero
// for every row (C5's phase-2 weights, ~1e-6, leave L2 empty): a local saving, the histograms
// and their exchange are unchanged.  (Measured, not kept: the counts carried in L0's sums from
// bit 40 up when both fit, one atomic per element fewer -- 4.16 vs 4.14 ms at C5.)
__global__ void __launch_bounds__(BT) k_sel_wlimbs(pcx_mat m) {
    const double* w = m.sel_phase == 1 ? m.rep : m.rowv + RV_SMOOTH * m.n_rows;
    uint64_t any0 = 0, any2 = 0;
    for (int64_t i = (int64_t)blockIdx.x * BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const limbs3 L = to_limbs(w[i]);
        any0 |= L.l0;
        any2 |= L.l2;
    }
    __shared__ unsigned long long bits;
    if (threadIdx.x == 0) bits = 8;
    __syncthreads();
    const bool b0 = __ballot(any0 != 0) != 0, b2 = __ballot(any2 != 0) != 0;
    if (threadIdx.x % WAVE == 0 && (b0 || b2)) atomicOr(&bits, (b0 ? 1ull : 0ull) | (b2 ? 4ull : 0ull));
    __syncthreads();
    // one global atomic per block, and only when it adds a bit (thousands of ORs into one word
    // serialise at its L2 channel: 50 us)
    if (threadIdx.x == 0) {
        unsigned long long* f = (unsigned long long*)&m.info[IN_SEL_WLIMB];
        if ((__atomic_load_n(f, __ATOMIC_RELAXED) & bits) != bits) atomicOr(f, bits);
    }
}

// The first pass's window: a sample of the column (1 / SEL_SAMPLE of its rows, all ranks'
// samples summed) histogrammed in the first pass's buckets; the bucket where the sample's
// weight crosses half, +- SEL_WIN buckets, is the window the first pass also gathers into cbuf.
// When the exact crossing bucket lies inside it (nearly always) the later passes read only
// cbuf -- one read of the column per phase instead of two.  A miss (or a cbuf overflow) only
// falls back to the plain passes: the sample never decides a result.
constexpr int SEL_SAMPLE = 64;
constexpr int SEL_WIN = 3;
__device__ __forceinline__ double* sel_sample_row(const pcx_mat& m, int a) {
    return reinterpret_cast<double*>(m.hist_w) + (int64_t)a * NB * 3;  // [NB] weight, [NB] count
}

__global__ void __launch_bounds__(BT) k_sel_sample(pcx_mat m) {
    const int a = blockIdx.x;
    if (a >= (int)m.info[IN_SEL_ACTIVE]) return;
    const int s = m.sel_act[a];
    const uint64_t* st = m.sel_state + (int64_t)s * SELS;
    __shared__ double sw[NB], sn[NB];
    for (int b = threadIdx.x; b < NB; b += BT) sw[b] = sn[b] = 0.0;
    __syncthreads();
    const uint64_t lo = st[SW_LO], hi = st[SW_HI];
    const int sh = (int)st[SW_SHIFT];
    // runs of SEL_RUN consecutive rows every SEL_RUN * SEL_SAMPLE rows (the same 1/64 of the column
    // as every 64th row, in whole cache lines: a strided sample read a line per element)
    constexpr int SEL_RUN = 16;
    const int64_t span = (int64_t)SEL_RUN * SEL_SAMPLE, full = m.n_rows / span;
    const int64_t rem = m.n_rows - full * span;
    const int64_t ns = full * SEL_RUN + (rem < SEL_RUN ? rem : SEL_RUN);
    for (int64_t j = threadIdx.x; j < ns; j += BT) {
        double x, w;
        const XW v = sel_load(m, s, (j / SEL_RUN) * span + (j % SEL_RUN));
        if (!sel_decode(m, s, v, x, w)) continue;
        const uint64_t k = dkey(x);
        if (k < lo || k > hi) continue;
        const int b = (int)((k - lo) >> sh);
        atomicAdd(&sw[b], w);
        // phase 2: a filled row (all at the fill value) is binned once by k_sel_hist, never
        // gathered into cbuf -- it weighs in the crossing, not in the window's size estimate
        if (!(m.sel_phase == 2 && __builtin_isnan(v.x))) atomicAdd(&sn[b], 1.0);
    }
    __syncthreads();
    double* o = sel_sample_row(m, a);
    for (int b = threadIdx.x; b < NB; b += BT) {
        o[b] = sw[b];
        o[NB + b] = sn[b];
    }
}

// exact weight / count histogram of the keys inside [lo, hi] (NB buckets) of active event a
// One block per active event.  Once the key range holds at most ccap elements (all ranks),
// the pass that reads the whole column also compacts this rank's in-range (key, weight)
// pairs into cbuf; later passes read only those (the histogram is a set of exact integer
// sums / minima / maxima, so the compacted order does not matter).
// NT threads per event: 256, or 1,024 when the active events leave CUs idle (C4: 250 events on 256
// CUs -- one 256-thread workgroup per CU kept four waves streaming each column)
// CM: phase 1 under reputation=None, where every pass counts (every weight is 1 / N): no weight
// loads, limbs or weight extremes, 32-bit counts (n_rows < 2^32, sel_hist), a 16-row load batch
// held to 64 VGPRs (eight waves per SIMD: 2.30 -> 2.03 ms at C5 against 8-row batches; 65 VGPRs
// unforced cost a wave per SIMD)
template <int NT, bool CM>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(CM ? 8 : PCX_SEL_WWAVES))) k_sel_hist(pcx_mat m) {
    const int a = blockIdx.x;
    if (a >= (int)m.info[IN_SEL_ACTIVE]) return;  // the first pass is launched for every scaled event
    const int s = m.sel_act[a];
    uint64_t* st = m.sel_state + (int64_t)s * SELS;
    // SEL_HC copies of every bucket, bucket b's copy c at b SEL_HC + c and a thread binning into
    // copy threadIdx.x % SEL_HC: lanes of a wave whose keys share a bucket split over the copies
    // (same-address LDS atomics serialise); the copies merge exactly (integer sums, min, max)
    constexpr int HC = CM ? 4 : SEL_HC;  // (count mode, half the arrays: four copies, 2.38 -> 2.26 ms at C5)
    constexpr int HW = CM ? 1 : NB * HC;
    __shared__ unsigned long long ha[HW], hb[HW], hc[HW], hmin[NB * HC], hmax[NB * HC];
    // (32-bit LDS counts in the weight-mode kernel measured: no faster)
    typedef typename std::conditional<CM, unsigned int, unsigned long long>::type hn_t;
    __shared__ hn_t hn[NB * HC];
    __shared__ unsigned long long gcount, f_wlo, f_whi, f_ga, f_gb, f_gc, f_gn;
    for (int b = threadIdx.x; b < NB * HC; b += NT) {
        if constexpr (!CM) ha[b] = hb[b] = hc[b] = 0;
        hn[b] = 0;
        hmin[b] = ~0ull;
        hmax[b] = 0;
    }
    if (threadIdx.x == 0) {
        gcount = 0;
        f_wlo = ~0ull;
        f_whi = 0;
        f_ga = f_gb = f_gc = f_gn = 0;
    }
    __syncthreads();
    // first pass (sel_first): the weight extremes of every element, and in phase 2 the filled
    // rows (all at the fill value) summed apart and binned once at the end
    const bool first = m.sel_first != 0;
    const bool gfirst = !CM && first && m.sel_phase == 2;
    uint64_t wlo = ~0ull, whi = 0, ga = 0, gb = 0, gc = 0, gn = 0;
    __shared__ int win_s[2];
    if (first && threadIdx.x == 0) {  // the sampled window (k_sel_sample, all ranks)
        const double* smp = sel_sample_row(m, a);
        const bool wm = st[SW_MODE] == 0;
        double tot = 0.0;
        for (int b = 0; b < NB; b++) tot += wm ? smp[b] : smp[NB + b];
        int b0 = 1, b1 = 0;  // empty
        if (tot > 0.0 && m.cbuf) {
            double cum = 0.0;
            int bx = NB - 1;
            for (int b = 0; b < NB; b++) {
                cum += wm ? smp[b] : smp[NB + b];
                if (2.0 * cum >= tot) {
                    bx = b;
                    break;
                }
            }
            // widen by up to SEL_WIN buckets a side while this rank's estimated share of the
            // window (sampled count x SEL_SAMPLE / world) stays within half of cbuf; a crossing
            // bucket denser than that gets no window (the plain passes narrow it first)
            // (and within 1/8 of the column: a wider window re-reads about as much from cbuf
            // as the plain pass reads from the column, after paying for the gather)
            const double share = fmin(0.5 * (double)m.ccap, (double)m.n_rows / 8.0);
            const double cap = share * (double)m.world / (double)SEL_SAMPLE;
            double est = smp[NB + bx];
            if (est <= cap) {
                b0 = b1 = bx;
                for (int r = 1; r <= SEL_WIN; r++) {
                    const double l = bx - r >= 0 ? smp[NB + bx - r] : 0.0;
                    const double h = bx + r < NB ? smp[NB + bx + r] : 0.0;
                    if (est + l + h > cap) break;
                    est += l + h;
                    b0 = bx - r >= 0 ? bx - r : 0;
                    b1 = bx + r < NB ? bx + r : NB - 1;
                }
            }
        }
        win_s[0] = b0;
        win_s[1] = b1;
        st[SW_WB0] = (uint64_t)b0;
        st[SW_WB1] = (uint64_t)b1;
    }
    __syncthreads();
    const int wb0 = first ? win_s[0] : 1, wb1 = first ? win_s[1] : 0;
    const bool wgather = first && wb0 <= wb1;
    const uint64_t lo = st[SW_LO], hi = st[SW_HI];
    const int sh = (int)st[SW_SHIFT];
    const bool wmode = !CM && st[SW_MODE] == 0;
    const bool from_buf = st[SW_CMODE] == 1;
    // phase 2: the filled rows all sit at the fill value -- binned once, not per element
    const bool gties = !CM && m.sel_phase == 2 && st[SW_GN] > 0;
    const uint64_t gk = gties ? dkey(m.ev[EV_GUESS * m.n_events + m.scaled_cols[s]]) : 0;
    const bool gin = gties && gk >= lo && gk <= hi;
    const uint64_t ties_all = gin ? (uint64_t)m.ev[EV_MISS * m.n_events + m.scaled_cols[s]] : 0;  // all ranks
    const uint64_t need = st[SW_INRANGE] > ties_all ? st[SW_INRANGE] - ties_all : 0;
    // gather only once the range has narrowed: later passes then read 16 B per in-range element
    // instead of the column, which pays when the range holds a small part of it (a shard whose
    // whole column fits cbuf would otherwise gather everything and re-read it per pass)
    const bool gather = !from_buf && m.cbuf && st[SW_INRANGE] > 0 && need <= (uint64_t)m.ccap &&
                        8 * need <= st[SW_COUNT];
    uint64_t* cb = m.cbuf ? m.cbuf + (int64_t)s * m.ccap * 2 : nullptr;
    const int hcp = HC > 1 ? (int)(threadIdx.x % HC) : 0;
    const int64_t wl = CM ? 0 : m.info[IN_SEL_WLIMB];  // (k_sel_wlimbs: a limb no row uses is not summed)
    const bool use0 = !(wl & 8) || (wl & 1), use2 = !(wl & 8) || (wl & 4);
    // Phase 2's first pass bins the present values of phase 1's first pass (the same rows, the
    // same keys) plus the filled rows, which it bins apart: over the same range and shift the
    // buckets' counts and key extremes of the present values are the ones phase 1 counted.  Phase
    // 1's first pass keeps them (this rank's, before the reduction: vsave), and phase 2's takes
    // them instead of three LDS atomics per element -- the weight limbs are new, the rest is not.
    // (A filled row's fill value may lie outside phase 1's range, int_dtype truncating it: a
    // changed range recounts.)
    uint64_t* const vkey = m.vsave ? m.vsave + (int64_t)m.n_scaled * NB * 3 + (int64_t)s * 4 : nullptr;
    const bool vput = first && m.sel_phase == 1 && vkey;
    const bool vreuse = !CM && first && m.sel_phase == 2 && vkey && vkey[3] == 1 && vkey[0] == lo &&
                        vkey[1] == hi && vkey[2] == (uint64_t)sh;
    auto bin = [&](uint64_t k, double w) {
        const int b = (int)((k - lo) >> sh) * HC + hcp;
        if constexpr (!CM) {
            if (wmode) {
                const limbs3 L = to_limbs(w);
                if (use0) atomicAdd(&ha[b], (unsigned long long)L.l0);
                atomicAdd(&hb[b], (unsigned long long)L.l1);
                if (use2) atomicAdd(&hc[b], (unsigned long long)L.l2);
            }
        }
        if (!CM && vreuse) return;
        atomicAdd(&hn[b], (hn_t)1);
        // (measured: reading the extremes first and skipping the atomics that cannot change them
        // is slower, 9.4 -> 12.0 ms at C5 -- the read's latency sits in every element's path,
        // where the no-return atomics are fire-and-forget; min / max interleaved in one array,
        // 9.4 -> 9.7 ms -- twice the bank conflicts of two arrays; exact extremes only inside the
        // sampled window, nominal bounds elsewhere, 9.4 -> 9.7 ms)
        atomicMin(&hmin[b], (unsigned long long)k);
        atomicMax(&hmax[b], (unsigned long long)k);
    };
    if (from_buf) {
        const int64_t nc = m.ccount[s];
        for (int64_t j = threadIdx.x; j < nc; j += NT) {
            const uint64_t k = cb[2 * j];
            if (k < lo || k > hi) continue;
            bin(k, __longlong_as_double(cb[2 * j + 1]));
        }
    } else {
        const double* const tcol = m.T + (int64_t)s * m.n_rows;
        const double wc = 1.0 / (double)m.n_total;  // (CM: sel_load's weight)
        rows_strided<(CM ? 16 : SEL_WUNROLL)>(threadIdx.x, NT, m.n_rows, [&](int64_t i) {
                                     if constexpr (CM) return XW{tcol[i], wc};
                                     else return sel_load(m, s, i);
                                 },
                                 [&](int64_t, XW v) {
            double x, w;
            if (gties && __builtin_isnan(v.x)) return;  // a filled row
            if constexpr (CM) {
                if (__builtin_isnan(v.x)) return;
                x = v.x;
                w = v.w;
            } else if (!sel_decode(m, s, v, x, w)) return;
            if (!CM && first) {
                const uint64_t wb = (uint64_t)__double_as_longlong(w);  // weights >= 0 order like their bits
                wlo = wb < wlo ? wb : wlo;
                whi = wb > whi ? wb : whi;
                if (gfirst && __builtin_isnan(v.x)) {  // a filled row: summed here, binned once below
                    if (wmode) {
                        const limbs3 L = to_limbs(w);
                        ga += L.l0;
                        gb += L.l1;
                        gc += L.l2;
                    }
                    gn++;
                    return;
                }
            }
            const uint64_t k = dkey(x);
            if (k < lo || k > hi) return;
            bin(k, w);
            if (wgather || gather) {
                const int b = (int)((k - lo) >> sh);
                const bool put = gather || (b >= wb0 && b <= wb1);
                // one LDS atomic per wave: the lanes that append take consecutive slots
                const uint64_t pm = __ballot(put);
                if (pm) {
                    const int lead = __ffsll((long long)pm) - 1;
                    const int lane = threadIdx.x % WAVE;
                    unsigned long long base = 0;
                    if (lane == lead) base = atomicAdd(&gcount, (unsigned long long)__popcll(pm));
                    base = (unsigned long long)__shfl((long long)base, lead, WAVE);
                    const unsigned long long j = base + __popcll(pm & ((1ull << lane) - 1ull));
                    if (put && j < (unsigned long long)m.ccap) {
                        cb[2 * j] = k;
                        cb[2 * j + 1] = (uint64_t)__double_as_longlong(w);
                    }
                }
            }
        });
    }
    if (first) {
        if (CM) wlo = whi = (uint64_t)__double_as_longlong(1.0 / (double)m.n_total);
        atomicMin(&f_wlo, (unsigned long long)wlo);
        atomicMax(&f_whi, (unsigned long long)whi);
        if (gn) {
            atomicAdd(&f_ga, (unsigned long long)ga);
            atomicAdd(&f_gb, (unsigned long long)gb);
            atomicAdd(&f_gc, (unsigned long long)gc);
            atomicAdd(&f_gn, (unsigned long long)gn);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            m.sel_imin[s * 2 + 1] = ~f_wlo;  // all ranks: (complemented) MAX before k_sel_start
            m.sel_imax[s * 2 + 1] = f_whi;
            if (!CM && f_gn) {  // this rank's filled rows, all at the fill value (inside [lo, hi])
                st[SW_GN] = f_gn;
                st[SW_GW0] = f_ga;
                st[SW_GW1] = f_gb;
                st[SW_GW2] = f_gc;
                const uint64_t fk = dkey(m.ev[EV_GUESS * m.n_events + m.scaled_cols[s]]);
                const int b = (int)((fk - lo) >> sh) * HC;
                if constexpr (!CM) {
                    if (wmode) {
                        atomicAdd(&ha[b], f_ga);
                        atomicAdd(&hb[b], f_gb);
                        atomicAdd(&hc[b], f_gc);
                    }
                }
                atomicAdd(&hn[b], (hn_t)f_gn);
                atomicMin(&hmin[b], (unsigned long long)fk);
                atomicMax(&hmax[b], (unsigned long long)fk);
            }
        }
    }
    if (gin && threadIdx.x == 0) {
        const int b = (int)((gk - lo) >> sh) * HC;
        if constexpr (!CM) {
            if (wmode) {
                atomicAdd(&ha[b], (unsigned long long)st[SW_GW0]);
                atomicAdd(&hb[b], (unsigned long long)st[SW_GW1]);
                atomicAdd(&hc[b], (unsigned long long)st[SW_GW2]);
            }
        }
        atomicAdd(&hn[b], (hn_t)st[SW_GN]);
        atomicMin(&hmin[b], (unsigned long long)gk);
        atomicMax(&hmax[b], (unsigned long long)gk);
    }
    __syncthreads();
    if (gather && threadIdx.x == 0) {
        m.ccount[s] = (int64_t)gcount;
        st[SW_CMODE] = 1;
    }
    if (wgather && threadIdx.x == 0) {  // pending: valid once the crossing bucket is inside the window
        const bool fits = gcount <= (unsigned long long)m.ccap;
        m.ccount[s] = fits ? (int64_t)gcount : 0;
        st[SW_CMODE] = fits ? 2 : 0;
    }
    if (vput && threadIdx.x == 0) {
        vkey[0] = lo;
        vkey[1] = hi;
        vkey[2] = (uint64_t)sh;
        vkey[3] = 1;
    }
    const int64_t o = (int64_t)a * NB;
    for (int b = threadIdx.x; b < NB; b += NT) {
        unsigned long long sa = 0, sb = 0, sc = 0, mn = ~0ull, mx = 0;
        uint64_t sn = 0;
#pragma unroll
        for (int c = 0; c < HC; c++) {
            if constexpr (!CM) {
                sa += ha[b * HC + c];
                sb += hb[b * HC + c];
                sc += hc[b * HC + c];
            }
            sn += (uint64_t)hn[b * HC + c];
            mn = hmin[b * HC + c] < mn ? hmin[b * HC + c] : mn;
            mx = hmax[b * HC + c] > mx ? hmax[b * HC + c] : mx;
        }
        uint64_t* const vs = m.vsave ? m.vsave + ((int64_t)s * NB + b) * 3 : nullptr;
        if (vput) {  // this rank's present values of the range (before the reduction over ranks)
            vs[0] = sn;
            vs[1] = mn;
            vs[2] = mx;
        } else if (vreuse) {
            sn += vs[0];
            mn = vs[1] < mn ? vs[1] : mn;
            mx = vs[2] > mx ? vs[2] : mx;
        }
        if (wmode) {
            m.hist_w[(o + b) * 3 + 0] = sa;
            m.hist_w[(o + b) * 3 + 1] = sb;
            m.hist_w[(o + b) * 3 + 2] = sc;
        }
        m.hist_n[o + b] = sn;
        m.hist_min[o + b] = ~mn;  // complemented: the ranks' minima and maxima reduce in one MAX
        m.hist_max[o + b] = mx;
    }
}

// walk the buckets (reduced over ranks): weight mode keeps the bucket where the exact
// prefix crosses half the total, count mode the one holding rank `target`; a single-key
// bucket resolves (weight mode: unless the crossing is near a rounding-decided half)
// one wave per active event: lane l owns buckets PB*l .. PB*l+PB-1.  The exact prefix sums
// of the bucket counts and weight limbs come from a wave scan (integer limbs: order-free), the
// first bucket whose prefix crosses the half (weights) / target (counts) by ballot, and that
// bucket's lane applies the narrowing (a 256-step serial scan per event before).
constexpr int SEL_PB = NB / WAVE;
__device__ __forceinline__ uint64_t scan_add_u64(uint64_t v, int lane) {  // inclusive
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        const uint64_t u = __shfl_up(v, d, WAVE);
        if (lane >= d) v += u;
    }
    return v;
}
__device__ __forceinline__ uint64_t scan_max_u64(uint64_t v, int lane) {  // inclusive
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        const uint64_t u = __shfl_up(v, d, WAVE);
        if (lane >= d) v = u > v ? u : v;
    }
    return v;
}

__global__ void __launch_bounds__(BT) k_sel_step(pcx_mat m, int n_active) {
    const int a = blockIdx.x * (BT / WAVE) + threadIdx.x / WAVE;
    const int lane = threadIdx.x % WAVE;
    if (a >= n_active || a >= (int)m.info[IN_SEL_ACTIVE]) return;  // wave-uniform
    const int s = m.sel_act[a];
    uint64_t* st = m.sel_state + (int64_t)s * SELS;
    if (st[SW_STATUS] != 1) return;  // the first pass's start may have finished it
    const bool wmode = st[SW_MODE] == 0;
    const L3 tot = ld_l3(st + SW_TOT0);
    const uint64_t n_all = st[SW_COUNT], target = st[SW_TARGET];
    const L3 below0 = ld_l3(st + SW_BELOW0);
    const uint64_t cbelow0 = st[SW_CNT_BELOW], below_max0 = st[SW_BELOW_MAX];
    const bool has_below0 = st[SW_HAS_BELOW] != 0;
    const int64_t o = (int64_t)a * NB;
    uint64_t nb[SEL_PB], kmn[SEL_PB], kmx[SEL_PB];
    L3 hw[SEL_PB];
    uint64_t sc = 0, sa = 0, sb = 0, sl = 0, smax = 0;  // lane totals (counts, limbs), last key
#pragma unroll
    for (int j = 0; j < SEL_PB; j++) {
        const int b = lane * SEL_PB + j;
        nb[j] = m.hist_n[o + b];
        const uint64_t* hs = m.hist_w + (o + b) * 3;
        hw[j] = (wmode && nb[j]) ? l3_norm({hs[0], hs[1], hs[2]}) : L3{0, 0, 0};
        kmn[j] = ~m.hist_min[o + b];
        kmx[j] = m.hist_max[o + b];
        sc += nb[j];
        sa += hw[j].a;
        sb += hw[j].b;
        sl += hw[j].c;
        if (nb[j]) smax = kmx[j];  // keys rise with the bucket index
    }
    // exclusive prefixes over the lanes below
    const uint64_t ic = scan_add_u64(sc, lane), ia = scan_add_u64(sa, lane), ib = scan_add_u64(sb, lane),
                   il = scan_add_u64(sl, lane), imax = scan_max_u64(smax, lane);
    uint64_t pc = ic - sc, pa = ia - sa, pb = ib - sb, pl = il - sl;
    uint64_t pmax = __shfl_up(imax, 1, WAVE);
    if (lane == 0) pmax = 0;
    int first = SEL_PB;  // this lane's first crossing bucket
    L3 below{}, upto{};
    uint64_t cbelow = 0, below_max = 0;
    bool has_below = false;
#pragma unroll
    for (int j = 0; j < SEL_PB; j++) {
        const L3 bl = l3_norm({below0.a + pa, below0.b + pb, below0.c + pl});
        const L3 up = l3_norm({bl.a + hw[j].a, bl.b + hw[j].b, bl.c + hw[j].c});
        const bool cross = nb[j] && (wmode ? l3_cmp(l3_twice(up), tot) > 0 : cbelow0 + pc + nb[j] > target);
        if (cross && first == SEL_PB) {
            first = j;
            below = bl;
            upto = up;
            cbelow = cbelow0 + pc;
            const bool any = pmax != 0 || pc != 0;  // nonempty buckets passed in this pass
            below_max = any ? pmax : below_max0;
            has_below = has_below0 || any;
        }
        pc += nb[j];
        pa += hw[j].a;
        pb += hw[j].b;
        pl += hw[j].c;
        if (nb[j]) pmax = kmx[j];
    }
    const uint64_t mask = __ballot(first < SEL_PB);
    if (mask == 0) {  // no crossing (cannot happen with exact sums)
        if (lane == 0) sel_done(st, __builtin_nan(""));
        return;
    }
    if (lane != __ffsll((long long)mask) - 1) return;
    const uint64_t n = nb[first], kmin = kmn[first], kmax = kmx[first];
    if (kmin == kmax) {
        const double xs = dkey_inv(kmin);
        if (wmode) {
            if (near_half(below, tot, n_all) || near_half(upto, tot, n_all)) {
                mark_hard(m, s, st);
                return;
            }
            if (m.sel_phase == 2) {  // every element equal to the outcome is in this bucket
                st[SW_CERTN] = n;
                st_l3(st + SW_CW0, hw[first]);
            }
            sel_done(st, xs);
        } else {
            double r = xs;
            if (st[SW_HALF] == 2) {
                r = __builtin_nan("");
            } else if (st[SW_HALF] == 1) {
                const double pred = target >= cbelow + 1 ? xs : dkey_inv(below_max);
                r = (pred + xs) / 2.0;  // sum(bounds) / float(len(bounds))
            }
            sel_done(st, r);
        }
    } else {
        // the first pass's window holds this rank's elements of the crossing bucket when the
        // bucket lies inside it: later passes read cbuf (else the column, as without a window)
        if (st[SW_CMODE] == 2) {
            const int b = lane * SEL_PB + first;
            st[SW_CMODE] = (b >= (int)st[SW_WB0] && b <= (int)st[SW_WB1]) ? 1 : 0;
        }
        st[SW_LO] = kmin;
        st[SW_HI] = kmax;
        st[SW_SHIFT] = shift_for(kmin, kmax);
        st[SW_INRANGE] = n;
        st_l3(st + SW_BELOW0, below);
        st[SW_CNT_BELOW] = cbelow;
        st[SW_BELOW_MAX] = below_max;
        st[SW_HAS_BELOW] = has_below ? 1 : 0;
    }
}

// results into guess (phase 1; int dtype truncates, :312) / outcomes (phase 2, :537-538)
__global__ void __launch_bounds__(BT) k_sel_finish(pcx_mat m) {
    const int s = blockIdx.x * BT + threadIdx.x;
    if (s >= m.n_scaled) return;
    const int E = (int)m.n_events;
    const int c = m.scaled_cols[s];
    uint64_t* st = m.sel_state + (int64_t)s * SELS;
    const double r = __longlong_as_double(st[SW_RESULT]);
    if (m.sel_phase == 1) {
        if (st[SW_NEED]) m.ev[EV_GUESS * E + c] = m.int_dtype ? trunc(r) : r;
    } else {
        m.ev[EV_RAW * E + c] = r;
        m.ev[EV_ADJ * E + c] = r;
        double f = r * (m.hi[c] - m.lo[c]);  // :537-538, two roundings
        f = f + m.lo[c];
        m.ev[EV_FIN * E + c] = f;
    }
}

// Exact replay of weightedstats.weighted_median with the reference's float arithmetic,
// for one scaled event whose element count fits the block (n <= SEL_EXACT_MAX; single
// rank).  Phase 1 (:287-303): weights rep_j / (sequential sum of present rep), over the
// present reports in row order.  Phase 2 (:520-523): weights smooth_rep over all rows.
// mid = 0.5 * builtin sum (row order); dominant weight -> first argmax; else bitonic sort
// by (value, weight) and the sequential walk with the DBL_EPSILON exact-half test.
__global__ void __launch_bounds__(1024) k_sel_exact(pcx_mat m) {
    const int s = blockIdx.x;
    uint64_t* st = m.sel_state + (int64_t)s * SELS;
    if (st[SW_STATUS] == 0) return;
    __shared__ double xs[SEL_EXACT_MAX];
    __shared__ double ws[SEL_EXACT_MAX];
    __shared__ uint32_t pres[SEL_EXACT_MAX / 32];  // the rows' present bits (phase 1: a report; 2: a value)
    __shared__ int cnt;
    __shared__ double mid_s, wmax_s;
    __shared__ int first_s;
    const int tid = threadIdx.x;
    const int n_rows = (int)m.n_rows;
    // the column's (x, w) in row order into LDS by every thread (coalesced; thread 0 read them one
    // dependent global load at a time: 0.7 ms of a 1k x 100 consensus), the present bits beside;
    // an absent row holds (+inf, +inf), which the sort puts after every present pair, so nothing is
    // compacted (an in-place compaction by one thread waited on its own LDS stores)
    const bool ph1 = m.sel_phase == 1;
    for (int k = tid; k < SEL_EXACT_MAX / 32; k += 1024) pres[k] = 0;
    __syncthreads();
    for (int i = tid; i < n_rows; i += 1024) {
        double x = 0.0, w = 0.0;
        const bool ok = sel_elem(m, s, i, x, w);
        if (ok) atomicOr(&pres[i >> 5], 1u << (i & 31));
        xs[i] = ok ? x : __builtin_inf();
        ws[i] = ok ? w : __builtin_inf();
    }
    __syncthreads();
    auto present = [&](int i) { return ((pres[i >> 5] >> (i & 31)) & 1u) != 0; };
    __shared__ double tot_s;
    if (ph1 && tid == 0) {  // the present total, sequential in row order (read only: the loads pipeline)
        double tot = 0.0;
        for (int i = 0; i < n_rows; i++)
            if (present(i)) tot += ws[i];
        tot_s = tot;
    }
    __syncthreads();
    if (ph1)  // rep_j / tot, each its own division
        for (int i = tid; i < n_rows; i += 1024)
            if (present(i)) ws[i] = ws[i] / tot_s;
    __syncthreads();
    if (tid == 0) {
        int k = 0;
        double W = 0.0;
        for (int i = 0; i < n_rows; i++)
            if (present(i)) {
                W += ws[i];
                k++;
            }
        cnt = k;
        mid_s = 0.5 * W;
        first_s = n_rows;
        wmax_s = 0.0;
    }
    __syncthreads();
    const int n = cnt;
    const double mid = mid_s;
    // dominance: any(w > mid) -> data[first index of max(w)]; any positive weight (exact
    // reductions over the present rows, spread over the block)
    {
        __shared__ double red[1024];
        __shared__ int dom_s, first_p;
        if (tid == 0) {
            dom_s = 0;
            first_p = n_rows;
        }
        double mx = -__builtin_inf();
        bool dom = false, pos = false;
        for (int i = tid; i < n_rows; i += 1024) {
            if (!present(i)) continue;
            mx = fmax(mx, ws[i]);
            dom |= ws[i] > mid;
            pos |= ws[i] > 0.0;
            atomicMin(&first_p, i);
        }
        red[tid] = mx;
        dom = __syncthreads_or(dom);
        pos = __syncthreads_or(pos);
        for (int h = 512; h >= 1; h >>= 1) {
            if (tid < h) red[tid] = fmax(red[tid], red[tid + h]);
            __syncthreads();
        }
        // (the sequential max of the SPEC starts at the first present weight: a NaN there stays,
        // and nothing equals it)
        const double mxa = (n > 0 && __builtin_isnan(ws[first_p])) ? __builtin_nan("") : red[0];
        if (dom)
            for (int i = tid; i < n_rows; i += 1024)
                if (present(i) && ws[i] == mxa) atomicMin(&first_s, i);
        if (tid == 0) {
            dom_s = dom ? 1 : 0;
            wmax_s = pos ? 1.0 : 0.0;
        }
        __syncthreads();
        if (tid == 0 && !dom_s) first_s = -1;
        __syncthreads();
    }
    if (first_s >= 0) {
        if (tid == 0) sel_done(st, xs[first_s]);
        return;
    }
    if (wmax_s == 0.0) {  // no positive weight: None
        if (tid == 0) sel_done(st, __builtin_nan(""));
        return;
    }
    // bitonic sort of (x, w) pairs, padded to a power of two with +inf (the absent rows are too)
    int P = 1;
    while (P < n_rows) P <<= 1;
    for (int k = n_rows + tid; k < P; k += 1024) {
        xs[k] = __builtin_inf();
        ws[k] = __builtin_inf();
    }
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < P / 2; t += 1024) {
                const int lo = 2 * stride * (t / stride) + (t % stride);
                const int hi = lo + stride;
                const bool up = ((lo & size) == 0);
                const double xa = xs[lo], xb = xs[hi], wa = ws[lo], wb = ws[hi];
                const bool gt = (xa > xb) || (xa == xb && wa > wb);
                if (gt == up) {
                    xs[lo] = xb;
                    xs[hi] = xa;
                    ws[lo] = wb;
                    ws[hi] = wa;
                }
            }
            __syncthreads();
        }
    if (tid == 0) {
        double cum = 0.0;
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
        double res;
        if (fail) {
            res = __builtin_nan("");
        } else {
            const double before = cum - ws[k - 1];
            if (fabs(before - mid) < 2.220446049250313080847e-16) {
                if (k >= 2)
                    res = (xs[k - 2] + xs[k - 1]) / 2.0;
                else
                    res = n == 1 ? xs[0] / 1.0 : __builtin_nan("");
            } else {
                res = xs[k - 1];
            }
        }
        sel_done(st, res);
    }
}

// ------------------------------------------------------------------ hard replay
// Events whose decision sits within rounding of a threshold are replayed in the
// reference's own order.  Phase 1 (interpolate, :287-309): the present reports of the
// event in row order with weights rep_j / (sequential total); binary events: the
// sequential weighted mean then catch; scaled events: weightedstats on those pairs.
// Phase 2 (:519-523): weightedstats over the filled column with smooth_rep.

// this rank's elements of hard event j in row order -> send[j][0 .. cnt)
__global__ void __launch_bounds__(1024) k_hard_gather(pcx_mat m, HardArgs h) {
    const int j = blockIdx.x;
    const int c = h.cols[j];
    const ColParam p = col_param(m, c, true);
    double* out = h.send + (int64_t)j * h.cap * 2;
    const double* wsrc = m.sel_phase == 1 ? m.rep : m.rowv + RV_SMOOTH * m.n_rows;
    const int64_t E = m.n_events;
    const int sidx = m.scaled_index ? m.scaled_index[c] : -1;
    if (h.modes[j] == HARD_MEDIAN && sidx >= 0) {
        // a median's values come from T (k_colstats: the rescaled present value, NaN where missing,
        // one contiguous column) instead of a strided column of the row-major reports
        const double* Tc = m.T + (int64_t)sidx * m.n_rows;
        const double g = p.guess;
        const int64_t nt = block_compact(
            m.n_rows,
            [&](int64_t i) {
                const double v = Tc[i];
                if (m.sel_phase == 1) return !__builtin_isnan(v);
                return !__builtin_isnan(__builtin_isnan(v) ? g : v);
            },
            [&](int64_t i, int64_t pos) {
                const double v = Tc[i];
                out[pos * 2 + 0] = __builtin_isnan(v) ? g : v;
                out[pos * 2 + 1] = wsrc[i];
            });
        if (threadIdx.x == 0) h.send_cnt[j] = nt;
        return;
    }
    const int64_t n = block_compact(
        m.n_rows,
        [&](int64_t i) {
            const double x = rescale(m.reports[i * E + c], p, m.int_dtype);
            if (m.sel_phase == 1) return !missing(x);
            return !__builtin_isnan(missing(x) ? p.guess : x);
        },
        [&](int64_t i, int64_t pos) {
            const double x = rescale(m.reports[i * E + c], p, m.int_dtype);
            out[pos * 2 + 0] = missing(x) ? p.guess : x;
            out[pos * 2 + 1] = wsrc[i];
        });
    if (threadIdx.x == 0) h.send_cnt[j] = n;
}

// The hard replay's sequential fp64 chains (weightedstats' builtin sums and its walk) run on one
// lane: a dependent add per element is the floor (~8 cycles).  The lane reads its operands from
// an LDS tile in 16-element chunks, the next chunk's loads issued before the current chunk's adds,
// so the LDS latency (~50-60 cycles) hides behind the chain instead of stalling it every 8
// elements; the tiles are double-buffered: waves 1.. fill tile t+1 while lane 0 chains tile t.
constexpr int CHAIN = 16;

// acc + t[0] + t[1] + ... + t[len-1], left to right
__device__ __forceinline__ double chain_add(const double* t, int len, double acc) {
    double a[CHAIN], b[CHAIN];
    int k = 0;
    if (len >= CHAIN) {
#pragma unroll
        for (int j = 0; j < CHAIN; j++) a[j] = t[j];
        for (; k + 2 * CHAIN <= len; k += 2 * CHAIN) {
#pragma unroll
            for (int j = 0; j < CHAIN; j++) b[j] = t[k + CHAIN + j];
#pragma unroll
            for (int j = 0; j < CHAIN; j++) acc = acc + a[j];
            if (k + 3 * CHAIN <= len) {
#pragma unroll
                for (int j = 0; j < CHAIN; j++) a[j] = t[k + 2 * CHAIN + j];
            }
#pragma unroll
            for (int j = 0; j < CHAIN; j++) acc = acc + b[j];
        }
        if (k + CHAIN <= len) {  // a chunk loaded into a[] and not yet added
#pragma unroll
            for (int j = 0; j < CHAIN; j++) acc = acc + a[j];
            k += CHAIN;
        }
    }
    for (; k < len; k++) acc = acc + t[k];
    return acc;
}

// sequential left-to-right fp64 sum of f(k), k in [0, n): lane 0 chains, waves 1.. stage the
// tiles (tile: 2 * TILE doubles of LDS)
template <class F>
__device__ double block_serial_sum(int64_t n, F f, double* tile, int TILE) {
    __shared__ double acc_s;
    double acc = 0.0;
    const int loaders = (int)blockDim.x - WAVE;
    for (int k = threadIdx.x; k < TILE && k < n; k += blockDim.x) tile[k] = f(k);
    __syncthreads();
    int it = 0;
    for (int64_t t0 = 0; t0 < n; t0 += TILE, it++) {
        const int len = (int)(n - t0 < TILE ? n - t0 : TILE);
        const double* cur = tile + (it & 1) * TILE;
        double* nxt = tile + ((it + 1) & 1) * TILE;
        if (threadIdx.x == 0) {
            acc = chain_add(cur, len, acc);
        } else if ((int)threadIdx.x >= WAVE) {
            const int64_t n0 = t0 + TILE;
            const int nl = (int)(n - n0 < TILE ? (n - n0 > 0 ? n - n0 : 0) : TILE);
            for (int k = threadIdx.x - WAVE; k < nl; k += loaders) nxt[k] = f(n0 + k);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) acc_s = acc;
    __syncthreads();
    return acc_s;
}

constexpr int HARD_TILE = 4096;

__global__ void __launch_bounds__(1024) k_hard_prep(pcx_mat m, HardArgs h) {
    __shared__ double tile[2 * HARD_TILE];
    __shared__ unsigned long long wkey_s, first_s;
    __shared__ int pos_s, dom_s, neg_s;
    const int j = blockIdx.x;
    const int c = h.cols[j];
    const int mode = h.modes[j];
    const int64_t N = m.n_total;
    double* X = h.X + (int64_t)j * N;
    double* W = h.W + (int64_t)j * N;
    double* hs = h.hs + (int64_t)j * 4;
    // concatenate the ranks' rows (rank order = row order)
    int64_t n = 0;
    for (int w = 0; w < m.world; w++) {
        const int64_t cw = h.recv_cnt[(int64_t)w * h.n_hard + j];
        const double* src = h.recv + ((int64_t)w * h.n_hard + j) * h.cap * 2;
        for (int64_t k = threadIdx.x; k < cw; k += blockDim.x) {
            X[n + k] = src[2 * k];
            W[n + k] = src[2 * k + 1];
        }
        n += cw;
    }
    __syncthreads();
    if (m.sel_phase == 1) {  // weights rep_j / sequential total of the present rep (:294-302)
        const double tot = block_serial_sum(n, [&](int64_t k) { return W[k]; }, tile, HARD_TILE);
        for (int64_t k = threadIdx.x; k < n; k += blockDim.x) W[k] = W[k] / tot;
        __syncthreads();
    }
    const int s = m.scaled_index ? m.scaled_index[c] : -1;
    if (mode == HARD_MEAN) {  // guess = sum_seq(w * x) then catch (:304-309)
        const double g = block_serial_sum(n, [&](int64_t k) { return W[k] * X[k]; }, tile, HARD_TILE);
        if (threadIdx.x == 0) {
            double v = n > 0 ? catch_value(g, m.catch_tolerance) : catch_value(0.0, m.catch_tolerance);
            if (m.int_dtype) v = trunc(v);
            m.ev[EV_GUESS * m.n_events + c] = v;
            hs[2] = 0.0;
        }
        return;
    }
    uint64_t* st = m.sel_state + (int64_t)s * SELS;
    const double mid = 0.5 * block_serial_sum(n, [&](int64_t k) { return W[k]; }, tile, HARD_TILE);
    // dominance: any(w > mid) -> data[first index of max(w)]; no positive weight -> None.
    // Weights may be negative (a negative reputation): max over order-preserving keys.
    if (threadIdx.x == 0) {
        wkey_s = 0;
        first_s = ~0ull;
        pos_s = 0;
        dom_s = 0;
        neg_s = 0;
    }
    __syncthreads();
    double wl = -__builtin_inf();
    int posl = 0, doml = 0, negl = 0;
    for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
        wl = fmax(wl, W[k]);
        posl |= W[k] > 0.0;
        doml |= W[k] > mid;
        negl |= W[k] < 0.0;
    }
    if (negl) neg_s = 1;
    wl = wave_max_d(wl);
    if ((threadIdx.x & 63) == 0) atomicMax(&wkey_s, (unsigned long long)dkey(wl));
    if (posl) pos_s = 1;
    if (doml) dom_s = 1;
    __syncthreads();
    if (dom_s) {
        const double wmax = dkey_inv(wkey_s);  // some W[k] > mid: the max is a finite element
        for (int64_t k = threadIdx.x; k < n; k += blockDim.x)
            if (W[k] == wmax) {
                atomicMin(&first_s, (unsigned long long)k);
                break;
            }
        __syncthreads();
        if (threadIdx.x == 0) {
            sel_done(st, X[first_s]);
            hs[2] = 0.0;
        }
        return;
    }
    if (!pos_s) {
        if (threadIdx.x == 0) {
            sel_done(st, __builtin_nan(""));
            hs[2] = 0.0;
        }
        return;
    }
    uint64_t* keys = h.keys + (int64_t)j * h.P * 2;
    for (int64_t k = threadIdx.x; k < h.P; k += blockDim.x) {
        keys[2 * k + 0] = k < n ? dkey(X[k]) : ~0ull;
        keys[2 * k + 1] = k < n ? dkey(W[k]) : ~0ull;
    }
    if (threadIdx.x == 0) {
        hs[0] = mid;
        hs[1] = (double)n;
        hs[2] = 1.0;  // sort + walk pending
        hs[3] = neg_s ? 1.0 : 0.0;  // some weight < 0: the walk's partial sums are not monotone
    }
}

// bitonic sort of every segment keys[j][0 .. P) by (value key, weight key)
__device__ __forceinline__ bool key_gt(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    return ah > bh || (ah == bh && al > bl);
}

constexpr int BS_TILE = 4096;  // elements sorted in LDS per block (64 KB)

// stages size <= min(P, BS_TILE) of the network (init) or strides < BS_TILE of one size (merge)
__global__ void __launch_bounds__(1024) k_bsort_lds(uint64_t* keys, int64_t P, int64_t size_only) {
    __shared__ uint64_t kh[BS_TILE], kl[BS_TILE];
    const int64_t tile = P < BS_TILE ? P : BS_TILE;
    const int64_t base = (int64_t)blockIdx.x * tile;  // global element index (segments are contiguous)
    for (int k = threadIdx.x; k < tile; k += 1024) {
        kh[k] = keys[2 * (base + k)];
        kl[k] = keys[2 * (base + k) + 1];
    }
    __syncthreads();
    const int64_t s0 = size_only ? size_only : 2;
    const int64_t s1 = size_only ? size_only : tile;
    for (int64_t size = s0; size <= s1; size <<= 1) {
        for (int64_t stride = (size_only ? tile : size) >> 1; stride > 0; stride >>= 1) {
            if (stride >= size) continue;
            for (int t = threadIdx.x; t < tile / 2; t += 1024) {
                const int lo = (int)(2 * stride * (t / stride) + (t % stride));
                const int hi = lo + (int)stride;
                const int64_t g = (base + lo) % P;  // index within the segment: direction
                const bool up = (g & size) == 0;
                const bool gt = key_gt(kh[lo], kl[lo], kh[hi], kl[hi]);
                if (gt == up) {
                    const uint64_t a = kh[lo], b = kl[lo];
                    kh[lo] = kh[hi];
                    kl[lo] = kl[hi];
                    kh[hi] = a;
                    kl[hi] = b;
                }
            }
            __syncthreads();
        }
    }
    for (int k = threadIdx.x; k < tile; k += 1024) {
        keys[2 * (base + k)] = kh[k];
        keys[2 * (base + k) + 1] = kl[k];
    }
}

__global__ void __launch_bounds__(BT) k_bsort_global(uint64_t* keys, int64_t P, int64_t total, int64_t size,
                                                     int64_t stride) {
    for (int64_t t = blockIdx.x * (int64_t)BT + threadIdx.x; t < total / 2; t += (int64_t)gridDim.x * BT) {
        const int64_t lo = 2 * stride * (t / stride) + (t % stride);
        const int64_t hi = lo + stride;
        const bool up = ((lo % P) & size) == 0;
        const uint64_t ah = keys[2 * lo], al = keys[2 * lo + 1], bh = keys[2 * hi], bl = keys[2 * hi + 1];
        if (key_gt(ah, al, bh, bl) == up) {
            keys[2 * lo] = bh;
            keys[2 * lo + 1] = bl;
            keys[2 * hi] = ah;
            keys[2 * hi + 1] = al;
        }
    }
}

// the walk (:weighted_median while loop) over the sorted pairs of each pending event
__global__ void __launch_bounds__(1024) k_hard_walk(pcx_mat m, HardArgs h) {
    constexpr int TWS = HARD_TILE + 2 * CHAIN;  // a tile and the padding the chain's prefetch reads
    __shared__ double tw[2 * TWS];
    __shared__ int done_s;
    __shared__ int64_t k_s;
    __shared__ double cum_s;
    const int j = blockIdx.x;
    double* hs = h.hs + (int64_t)j * 4;
    if (h.modes[j] != HARD_MEDIAN || hs[2] != 1.0) return;
    const int c = h.cols[j];
    uint64_t* st = m.sel_state + (int64_t)m.scaled_index[c] * SELS;
    const uint64_t* keys = h.keys + (int64_t)j * h.P * 2;
    const double mid = hs[0];
    const int64_t n = (int64_t)hs[1];
    const bool monotone = hs[3] == 0.0;  // every weight >= 0: a chunk's last partial is its largest
    if (threadIdx.x == 0) {
        done_s = 0;
        k_s = 0;
        cum_s = 0.0;
    }
    // (a partial tile is followed by zeros: a chunk that runs past the last weight adds + 0.0)
    for (int k = threadIdx.x; k < TWS; k += blockDim.x) tw[k] = k < n && k < HARD_TILE ? dkey_inv(keys[2 * k + 1]) : 0.0;
    __syncthreads();
    // cum += w while cum <= mid (weightedstats' walk; mid > 0 here, so the first add always runs):
    // lane 0 adds a chunk's weights unconditionally -- partial sums up to the first one above mid
    // are exactly the walk's -- then finds that first one; waves 1.. stage the next tile meanwhile
    const int loaders = (int)blockDim.x - WAVE;
    int it = 0;
    for (int64_t t0 = 0; t0 < n; t0 += HARD_TILE, it++) {
        const int len = (int)(n - t0 < HARD_TILE ? n - t0 : HARD_TILE);
        const double* cur = tw + (it & 1) * TWS;
        double* nxt = tw + ((it + 1) & 1) * TWS;
        if (threadIdx.x == 0) {
            // static register indices only (a dynamic p[hit] sends the array to scratch); the tiles
            // are padded by 2 CHAIN so the next chunk's loads need no bounds test
            double cum = cum_s, hit_cum = 0.0;
            int hit_at = -1;
            double nv[CHAIN];
#pragma unroll
            for (int q = 0; q < CHAIN; q++) nv[q] = cur[q];
            for (int k = 0; k < len; k += CHAIN) {
                double v[CHAIN], p[CHAIN];
#pragma unroll
                for (int q = 0; q < CHAIN; q++) v[q] = nv[q];  // (past len: the tile's zero padding)
#pragma unroll
                for (int q = 0; q < CHAIN; q++) nv[q] = cur[k + CHAIN + q];  // the next chunk, in flight
                double acc = cum;
#pragma unroll
                for (int q = 0; q < CHAIN; q++) {
                    acc = acc + v[q];
                    p[q] = acc;
                }
                if (monotone && !(acc > mid)) {  // no partial of this chunk exceeds mid
                    cum = acc;
                    continue;
                }
                int h = -1;
                double hc = 0.0;
#pragma unroll
                for (int q = CHAIN - 1; q >= 0; q--)
                    if (p[q] > mid) {  // (padded partials repeat the last real one)
                        h = q;
                        hc = p[q];
                    }
                if (h >= 0) {
                    hit_at = k + h;
                    hit_cum = hc;
                    break;
                }
                cum = acc;
            }
            if (hit_at >= 0) {
                cum_s = hit_cum;
                k_s = t0 + hit_at + 1;
                done_s = 1;
            } else {
                cum_s = cum;
                k_s = t0 + len;
            }
        } else if ((int)threadIdx.x >= WAVE) {
            const int64_t n0 = t0 + HARD_TILE;
            const int nl = (int)(n - n0 < HARD_TILE ? (n - n0 > 0 ? n - n0 : 0) : HARD_TILE);
            for (int k = threadIdx.x - WAVE; k < TWS; k += loaders) nxt[k] = k < nl ? dkey_inv(keys[2 * (n0 + k) + 1]) : 0.0;
        }
        __syncthreads();
        if (done_s) break;
    }
    if (threadIdx.x == 0) {
        double res;
        const int64_t k = k_s;
        if (!done_s) {
            res = __builtin_nan("");  // the walk ran off the end (the reference raises IndexError)
        } else {
            const double wk = dkey_inv(keys[2 * (k - 1) + 1]);
            const double before = cum_s - wk;
            const double xk = dkey_inv(keys[2 * (k - 1)]);
            if (fabs(before - mid) < 2.220446049250313080847e-16) {
                if (k >= 2)
                    res = (dkey_inv(keys[2 * (k - 2)]) + xk) / 2.0;
                else
                    res = n == 1 ? xk / 1.0 : __builtin_nan("");
            } else {
                res = xk;
            }
        }
        sel_done(st, res);
        hs[2] = 0.0;
    }
}

// events marked hard (m.hard[c] != 0) in event order -> cols / modes, count -> info[IN_HARD]
__global__ void __launch_bounds__(1024) k_hard_list(pcx_mat m, int32_t* cols, int32_t* modes) {
    const int64_t cnt = block_compact(
        m.n_events, [&](int64_t c) { return m.hard[c] != HARD_NONE; },
        [&](int64_t c, int64_t pos) {
            cols[pos] = (int32_t)c;
            modes[pos] = m.hard[c];
        });
    if (threadIdx.x == 0) m.info[IN_HARD] = cnt;
}

// PCX_M_SCALED_CERT: sum of smooth_rep over rows whose filled value equals the outcome
__global__ void __launch_bounds__(BT) k_scaled_cert(pcx_mat m) {
    __shared__ dd lds[8];
    __shared__ double cnts[BT];
    const int s = blockIdx.x;
    const int E = (int)m.n_events;
    const int c = m.scaled_cols[s];
    const double adj = m.ev[EV_ADJ * E + c];
    const uint64_t* st = m.sel_state + (int64_t)s * SELS;
    if (st[SW_CERTN] != 0 && adj != 0.0 && !m.int_dtype) {
        // the selection's last histogram bucket held exactly the elements equal to the outcome
        // (all ranks, exact weight limbs): no pass over the column.  (+-0.0 and the int dtype's
        // truncated fills -- which may fold -0.0 -- take the pass.)
        if (threadIdx.x == 0) {
            const bool r0 = m.rank == 0;  // the totals are global: rank 0 carries them
            const double w = r0 ? l3_to_double(ld_l3(st + SW_CW0)) : 0.0;
            st_dd(m.cstat + (((int64_t)m.rank * E + c) * CS + 14) * 2, {w, 0.0});
            st_dd(m.cstat + (((int64_t)m.rank * E + c) * CS + 15) * 2, {r0 ? (double)st[SW_CERTN] : 0.0, 0.0});
        }
        return;
    }
    acc2 a;
    double n = 0.0;
    const double guess = m.ev[EV_GUESS * E + c];
    rows_strided<ROW_UNROLL>(
        threadIdx.x, BT, m.n_rows,
        [&](int64_t i) { return XW{m.T[(int64_t)s * m.n_rows + i], m.rowv[RV_SMOOTH * m.n_rows + i]}; },
        [&](int64_t, XW v) {
            const double f = __builtin_isnan(v.x) ? guess : v.x;
            if (f == adj) {
                a.add(v.w);
                n += 1.0;
            }
        });
    const dd r = block_sum_dd<BT>(a.get(), lds);
    cnts[threadIdx.x] = n;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tn = 0.0;
        for (int k = 0; k < BT; k++) tn += cnts[k];
        st_dd(m.cstat + (((int64_t)m.rank * E + c) * CS + 14) * 2, r);
        st_dd(m.cstat + (((int64_t)m.rank * E + c) * CS + 15) * 2, {tn, 0.0});
    }
}

// PCA: a NaN total of |u| leaves the reference's this_rep / smooth_rep fully MASKED, and
// participation_columns, reporter_bonus and author_bonus are then numpy.ma's data of fully masked
// results (oracle/pcx_oracle_batched.c rep_masked)
__device__ __forceinline__ bool rep_fully_masked(const pcx_mat& m) {
    return m.algorithm == 0 && __builtin_isnan(dd_to_double(scl(m, SC_U)));
}

// PCX_M_FINAL: certainty of scaled events, consensus_reward, participation, author bonus
__global__ void __launch_bounds__(1024) k_final(pcx_mat m) {
    __shared__ dd lds[16];
    __shared__ double sh[4];
    const int E = (int)m.n_events;
    for (int c = threadIdx.x; c < E; c += 1024)
        if (m.scaled && m.scaled[c]) {
            const double cnt = dd_to_double(cst(m, c, 15));
            m.ev[EV_CERT * E + c] = cnt > 0 ? dd_to_double(cst(m, c, 14)) : empty_certainty(m);
        }
    __syncthreads();
    acc2 sc, scp, spc, spcp;
    for (int c = threadIdx.x; c < E; c += 1024) {
        const double a = fabs(m.ev[EV_CERT * E + c]);
        sc.add(a);
        scp.add(a + 1.0);
        const double p = fabs(m.ev[EV_PC * E + c]);
        spc.add(p);
        spcp.add(p + 1.0);
    }
    const dd r0 = block_sum_dd<1024>(sc.get(), lds), r1 = block_sum_dd<1024>(scp.get(), lds);
    const dd r2 = block_sum_dd<1024>(spc.get(), lds), r3 = block_sum_dd<1024>(spcp.get(), lds);
    acc2 cs, ps;
    for (int c = threadIdx.x; c < E; c += 1024) {
        cs.add(m.ev[EV_CERT * E + c]);
        ps.add(m.ev[EV_PC * E + c]);
    }
    const dd r4 = block_sum_dd<1024>(cs.get(), lds), r5 = block_sum_dd<1024>(ps.get(), lds);
    if (threadIdx.x == 0) {
        sh[0] = dd_to_double(r0);
        sh[1] = dd_to_double(r1);
        sh[2] = dd_to_double(r2);
        sh[3] = dd_to_double(r3);
        const double avg_cert = dd_to_double(r4) / (double)E;
        const double pna = 1.0 - dd_to_double(r5) / (double)E;
        m.pvec[3 * (m.n_events + 64) + 4] = pna;
        if (m.scalars) {
            m.scalars[0] = 1.0 - pna;
            m.scalars[1] = avg_cert;
        }
    }
    __syncthreads();
    const double pna = m.pvec[3 * (m.n_events + 64) + 4];
    const bool rep_masked = rep_fully_masked(m);
    for (int c = threadIdx.x; c < E; c += 1024) {
        const double cert = m.ev[EV_CERT * E + c];
        const double reward = nweight(fabs(cert), sh[0], sh[1]);
        const double pc = m.ev[EV_PC * E + c];
        const double relc = nweight(fabs(pc), sh[2], sh[3]);
        if (m.adj_first_loadings) m.adj_first_loadings[c] = m.ev[EV_LD * E + c];
        if (m.outcomes_raw) m.outcomes_raw[c] = m.ev[EV_RAW * E + c];
        if (m.outcomes_adjusted) m.outcomes_adjusted[c] = m.ev[EV_ADJ * E + c];
        if (m.outcomes_final) m.outcomes_final[c] = m.ev[EV_FIN * E + c];
        if (m.certainty) m.certainty[c] = cert;
        if (m.consensus_reward) m.consensus_reward[c] = reward;
        if (m.nas_filled) m.nas_filled[c] = m.ev[EV_NZERO * E + c];
        if (m.participation_columns) m.participation_columns[c] = rep_masked ? 1.0 : pc;
        if (m.author_bonus) m.author_bonus[c] = rep_masked ? 1.0 : relc * pna + reward * (1.0 - pna);
    }
}

// PCX_M_ROWSUMS: sums for normalize(participation_rows) -- fully-NaN rows are masked (Q15)
__global__ void __launch_bounds__(BT) k_rowsums(pcx_mat m) {
    __shared__ dd lds[8];
    const int E = (int)m.n_events;
    acc2 a, ap;
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const bool masked = (int)m.rowstat[2 * i] == E;
        const double pr = 1.0 - (double)m.rowstat[2 * i + 1] / (double)E;
        if (!masked) {
            a.add(fabs(pr));
            ap.add(fabs(pr) + 1.0);
        }
    }
    const dd r0 = block_sum_dd<BT>(a.get(), lds), r1 = block_sum_dd<BT>(ap.get(), lds);
    if (threadIdx.x == 0) {
        st_dd(m.spart + blockIdx.x * 8 + 0, r0);
        st_dd(m.spart + blockIdx.x * 8 + 2, r1);
    }
}

// PCX_M_AGENTS: per-reporter outputs of this rank (:576-577, 586-595)
__global__ void __launch_bounds__(BT) k_agents(pcx_mat m) {
    const int E = (int)m.n_events;
    const double S = dd_to_double(scl(m, SC_AR)), Sp = dd_to_double(scl(m, SC_ARP));
    const double pna = m.pvec[3 * (m.n_events + 64) + 4];
    const bool rep_masked = rep_fully_masked(m);
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const bool masked = (int)m.rowstat[2 * i] == E;
        const double narow = (double)m.rowstat[2 * i + 1];
        const double pr = 1.0 - narow / (double)E;
        const double rel = masked ? fabs(pr) : nweight(fabs(pr), S, Sp);
        const double sm = m.rowv[RV_SMOOTH * m.n_rows + i];
        if (m.old_rep) m.old_rep[i] = m.rep[i];
        if (m.this_rep) m.this_rep[i] = m.rowv[RV_THIS * m.n_rows + i];
        if (m.smooth_rep) m.smooth_rep[i] = sm;
        if (m.scores) m.scores[i] = m.algorithm != 1 ? m.rowv[RV_S * m.n_rows + i] : 0.0;
        if (m.na_row) m.na_row[i] = narow;
        if (m.participation_rows) m.participation_rows[i] = pr;
        if (m.relative_part) m.relative_part[i] = rel;
        if (m.reporter_bonus) m.reporter_bonus[i] = (masked || rep_masked) ? rel : rel * pna + sm * (1.0 - pna);
    }
}

// PCX_M_MATRICES: rescaled (result["original"]) and filled (result["filled"]) reports
// grid (ceil(E/BT), G): thread = one event column over a chunk of rows (the column
// parameters loaded once)
__global__ void __launch_bounds__(BT) k_matrices(pcx_mat m) {
    const int c = blockIdx.x * BT + threadIdx.x;
    if (c >= m.n_events) return;
    const int E = (int)m.n_events;
    const ColParam p = col_param(m, c, true);
    int64_t r0, r1;
    row_range(m, r0, r1);
    rows_unrolled<ROW_UNROLL>(
        r0, r1, [&](int64_t i) { return m.reports[i * E + c]; },
        [&](int64_t i, double v) {
            const double x = rescale(v, p, m.int_dtype);
            const double xo = __builtin_isnan(x) ? v : x;  // (a NaN keeps its own bits, as in k_wcd)
            if (m.original) m.original[i * E + c] = xo;
            if (m.orig_inplace && p.scaled) const_cast<double*>(m.reports)[i * E + c] = xo;
            if (m.filled) m.filled[i * E + c] = missing(x) ? p.guess : x;
        });
}

__global__ void k_info_clear(pcx_mat m, int slot) { m.info[slot] = 0; }

// nonconformity entry: nc = set1 or set2 (:494-498, :482-484)
__global__ void __launch_bounds__(BT) k_nc_out(pcx_mat m) {
    double mn, mx;
    score_minmax(m, mn, mx);
    const int pick1 = (int)m.info[IN_PICK1];
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const double s = m.rowv[RV_S * m.n_rows + i];
        m.nc_out[i] = pick1 ? s + fabs(mn) : s - mx;
    }
}

// wpca entry: weighted_mean (:317-319)
__global__ void __launch_bounds__(BT) k_wmean_out(pcx_mat m) {
    const int c = blockIdx.x * BT + threadIdx.x;
    if (c < m.n_events) m.weighted_mean[c] = m.ev[EV_MU * m.n_events + c];
}

// lower triangle of the E x E covariance <-> packed buffer (row-major p >= q): the
// cross-rank SUM then moves E (E + 1) / 2 doubles instead of E^2; unpack mirrors
__global__ void __launch_bounds__(BT) k_tri_pack(double* C, double* buf, int64_t E, int unpack) {
    const int64_t n = E * (E + 1) / 2;
    for (int64_t t = blockIdx.x * (int64_t)BT + threadIdx.x; t < n; t += (int64_t)gridDim.x * BT) {
        int64_t p = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
        while ((p + 1) * (p + 2) / 2 <= t) p++;
        while (p * (p + 1) / 2 > t) p--;
        const int64_t q = t - p * (p + 1) / 2;
        if (unpack) {
            const double v = buf[t];
            C[p * E + q] = v;
            C[q * E + p] = v;
        } else {
            buf[t] = C[p * E + q];
        }
    }
}

// strided 2-D copy (slot exchange pack / unpack)
__global__ void __launch_bounds__(BT) k_copy2d(double* dst, int64_t dpitch, const double* src, int64_t spitch,
                                               int64_t width, int64_t rows) {
    const int64_t n = width * rows;
    for (int64_t t = blockIdx.x * (int64_t)BT + threadIdx.x; t < n; t += (int64_t)gridDim.x * BT) {
        const int64_t r = t / width, c = t % width;
        dst[r * dpitch + c] = src[r * spitch + c];
    }
}


__global__ void k_zero_loading(pcx_mat m) {
    for (int j = threadIdx.x; j < m.n_events; j += blockDim.x) m.ev[EV_LD * m.n_events + j] = 0.0;
}

// ---------------------------------------------------------------- PCX_M_EIG helpers
// gather diag(C) and the first component of every eigenvector (row k of the
// row-major view of rocSOLVER's column-major eigenvector matrix)
__global__ void __launch_bounds__(BT) k_eig_gather(const double* C, const double* U, int E, double* out) {
    for (int j = blockIdx.x * BT + threadIdx.x; j < E; j += gridDim.x * BT) {
        out[j] = C[(int64_t)j * E + j];
        out[E + j] = U[(int64_t)j * E];
    }
}

// g_j = sum_c coef_c * u_{idx_c, j} (components in order; coef = Sigma * sign)
__global__ void __launch_bounds__(BT) k_eig_combine(const double* U, int E, const double* coef, const int* idx,
                                                    int k, double* g) {
    for (int j = blockIdx.x * BT + threadIdx.x; j < E; j += gridDim.x * BT) {
        double acc = 0.0;
        for (int c = 0; c < k; c++) acc = fma(coef[c], U[(int64_t)idx[c] * E + j], acc);
        g[j] = acc;
    }
}

// numpy pairwise add.reduce (np.trace of the diagonal)
double np_pairwise(const double* a, int64_t n) {
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; i++) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; k++) r[k] = a[k];
        int64_t i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; k++) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
}

// one rocBLAS handle per (host thread, device): rocblas_set_stream + dsyevd on a handle
// shared between the threads of virtual ranks would race (handles are not thread-safe)
rocblas_handle blas_handle(int device) {
    struct Handles {
        std::map<int, rocblas_handle> h;
        ~Handles() {
            for (auto& kv : h) rocblas_destroy_handle(kv.second);
        }
    };
    static thread_local Handles handles;
    auto it = handles.h.find(device);
    if (it != handles.h.end()) return it->second;
    rocblas_handle h = nullptr;
    if (rocblas_create_handle(&h) != rocblas_status_success) return nullptr;
    handles.h[device] = h;
    return h;
}

hipError_t eig_stage(pcx_mat& m, hipStream_t st, std::string& err) {
    const int E = (int)m.n_events;
    const int64_t nn = (int64_t)E * E;
    double* U = m.Mw;                 // eigenvectors (in place of the copy of C)
    double* D = m.Mw + nn;            // eigenvalues, ascending
    double* work = D + E;             // tridiagonal off-diagonal
    double* tmp = work + E;           // [2E] diag(C), u_k[0]
    double* coef = tmp + 2 * E;       // [E]
    int* idx = (int*)(coef + E);      // [E]
    rocblas_int* info = (rocblas_int*)(idx + E + 2);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    rocblas_handle h = blas_handle(dev);
    if (!h) {
        err = "PCX_M_EIG: rocblas_create_handle failed";
        return hipErrorInvalidValue;
    }
    if ((e = hipMemcpyAsync(U, m.C, nn * sizeof(double), hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    rocblas_set_stream(h, st);
    if (rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, E, U, E, D, work, info) !=
        rocblas_status_success) {
        err = "PCX_M_EIG: rocsolver_dsyevd failed";
        return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(k_eig_gather, dim3((E + BT - 1) / BT), dim3(BT), 0, st, (const double*)m.C, (const double*)U,
                       E, tmp);
    std::vector<double> lam(E), dg(E), u0(E);
    rocblas_int hinfo = 0;
    if ((e = hipMemcpyAsync(lam.data(), D, E * sizeof(double), hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(dg.data(), tmp, E * sizeof(double), hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(u0.data(), tmp + E, E * sizeof(double), hipMemcpyDeviceToHost, st)) != hipSuccess)
        return e;
    if ((e = hipMemcpyAsync(&hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    if (hinfo != 0) {
        err = "PCX_M_EIG: dsyevd did not converge (info " + std::to_string(hinfo) + ")";
        return hipErrorInvalidValue;
    }
    std::vector<double> sig(E);
    std::vector<int> order(E);
    for (int j = 0; j < E; j++) sig[j] = std::fabs(lam[j]);
    std::iota(order.begin(), order.end(), 0);
    // singular values descending; equal ones keep the eigen-solver's (ascending) order reversed
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return sig[x] > sig[y]; });
    const double trace = np_pairwise(dg.data(), E);
    int k = m.algorithm == 2 ? std::min(std::max(m.max_components, 1), E) : E;
    if (m.algorithm == 3) {
        double ve = 0.0;
        for (int c = 0; c < E; c++) {
            ve = ve + sig[order[c]] / trace;
            if (ve >= m.variance_threshold) {
                k = c + 1;
                break;
            }
        }
    }
    std::vector<double> hc(k);
    std::vector<int> hi(k);
    for (int c = 0; c < k; c++) {
        hi[c] = order[c];
        hc[c] = sig[order[c]] * (u0[order[c]] < 0.0 ? -1.0 : 1.0);  // loading *= -1 if loading[0] < 0
    }
    if ((e = hipMemcpyAsync(coef, hc.data(), k * sizeof(double), hipMemcpyHostToDevice, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(idx, hi.data(), k * sizeof(int), hipMemcpyHostToDevice, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_eig_combine, dim3((E + BT - 1) / BT), dim3(BT), 0, st, (const double*)U, E,
                       (const double*)coef, (const int*)idx, k, m.ev + EV_SPARE * E);
    m.components = m.algorithm == 3 ? k : -1;
    return hipStreamSynchronize(st);
}

int grid_rows(int64_t n, int per_block) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;
    return (int)g;
}

// ================================================================== clustering algorithms
// "k-means" (:392-405), "hierarchical" (:407-419) and "clusterfeck" (:148-242, :421-424) on
// one rank, any N x E, in the operation order of the batched SPEC (oracle/
// pcx_oracle_batched.c hier_nc / kmeans_nc / feck_nc, pinned to 525 reference cases), which
// these kernels generalise from one 64 x 32 round.  Each algorithm turns the filled matrix
// into the nonconformity vector nc (rowv[RV_N1]); the common tail (:459-611) follows.

// np.ma.average(F, axis=0, weights) (:317, :167): column sums sequential over rows (pairwise
// when E == 1) over the pairwise total of the weights
__global__ void __launch_bounds__(BT) k_cl_mu(pcx_mat m, ClusterArgs a, double* out) {
    const int c = blockIdx.x * BT + threadIdx.x;
    const int E = (int)m.n_events;
    if (c >= E) return;
    const ColParam p = col_param(m, c, true);
    const int64_t N = m.n_rows;
    const double* w = a.weights;
    auto F = [&](int64_t i) { return filled(m.reports[i * E + c], p, m.int_dtype); };
    const double den = pw_sum_dev([&](int64_t i) { return w[i]; }, N);
    double num;
    if (E == 1) {
        num = pw_sum_dev([&](int64_t i) { return F(i) * w[i]; }, N);
    } else {
        num = F(0) * w[0];
        for (int64_t i = 1; i < N; i++) num = num + F(i) * w[i];
    }
    out[c] = num / den;
}

// reptokens with the zeros clusterfeck rewrites (:202-204)
__global__ void __launch_bounds__(BT) k_cl_wtok(pcx_mat m, ClusterArgs a) {
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT)
        a.wtok[i] = m.tok[i] == 0.0 ? 0.00001 : m.tok[i];
}

// X = F - mu (wcd, :322) or X = F
__global__ void __launch_bounds__(BT) k_cl_x(pcx_mat m, ClusterArgs a, int centre) {
    const int64_t E = m.n_events, n = m.n_rows * E;
    for (int64_t idx = blockIdx.x * (int64_t)BT + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * BT) {
        const int c = (int)(idx % E);
        const ColParam p = col_param(m, c, true);
        const double f = filled(m.reports[idx], p, m.int_dtype);
        a.X[idx] = centre ? f - a.mu[c] : f;
    }
}

// whiten (:395): population std of each wcd column (np.std axis 0: sequential column sums,
// pairwise when E == 1), zero -> 1
__global__ void __launch_bounds__(BT) k_cl_sd(pcx_mat m, ClusterArgs a) {
    const int c = blockIdx.x * BT + threadIdx.x;
    const int64_t E = m.n_events, N = m.n_rows;
    if (c >= E) return;
    const double* X = a.X;
    double s = 0.0;
    if (E == 1) s = pw_sum_dev([&](int64_t i) { return X[i]; }, N);
    else
        for (int64_t i = 0; i < N; i++) s = s + X[i * E + c];
    const double mean = s / (double)N;
    double v = 0.0;
    if (E == 1) {
        v = pw_sum_dev([&](int64_t i) { return (X[i] - mean) * (X[i] - mean); }, N);
    } else {
        for (int64_t i = 0; i < N; i++) {
            const double d = X[i * E + c] - mean;
            v = v + d * d;
        }
    }
    double sd = sqrt(v / (double)N);
    a.sd[c] = sd == 0.0 ? 1.0 : sd;
}

__global__ void __launch_bounds__(BT) k_cl_div(pcx_mat m, ClusterArgs a) {
    const int64_t E = m.n_events, n = m.n_rows * E;
    for (int64_t idx = blockIdx.x * (int64_t)BT + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * BT)
        a.X[idx] = a.X[idx] / a.sd[idx % E];
}

// lock-free union-find: parents point to smaller indices (no cycles), path halving by CAS
__device__ __forceinline__ int uf_load(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ int uf_find(int* par, int x) {
    for (;;) {
        const int q = uf_load(par + x);
        if (q == x) return x;
        const int r = uf_load(par + q);
        if (r != q) atomicCAS(par + x, q, r);
        x = q;
    }
}
__device__ void uf_unite(int* par, int a, int b) {
    for (;;) {
        a = uf_find(par, a);
        b = uf_find(par, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(par + a, a, b) == a) return;
    }
}

__global__ void __launch_bounds__(BT) k_cl_iota(pcx_mat m, ClusterArgs a) {
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        a.par[i] = (int)i;
        a.cnt[i] = 0;
    }
}

// hierarchical (:407-419): scipy fclusterdata(wcd, t, 'distance') with single linkage on
// euclidean pdist = connected components of {d_ij <= t}; d_ij = sqrt(sum_k (x_ik - x_jk)^2),
// sequential in k, no fma (scipy's pdist order).  16 x 16 row pairs per block, 32 events per
// LDS stage (the k order is kept across stages).
constexpr int CLT = 16, CLK = 32;
__global__ void __launch_bounds__(CLT * CLT) k_cl_hier(pcx_mat m, ClusterArgs a) {
    const int I = blockIdx.y, J = blockIdx.x;
    if (I > J) return;
    __shared__ double xi[CLT][CLK + 1], xj[CLT][CLK + 1];
    const int64_t N = m.n_rows, E = m.n_events;
    const int ti = threadIdx.x / CLT, tj = threadIdx.x % CLT;
    const int64_t i = (int64_t)I * CLT + ti, j = (int64_t)J * CLT + tj;
    double d2 = 0.0;
    for (int64_t k0 = 0; k0 < E; k0 += CLK) {
        for (int e = threadIdx.x; e < 2 * CLT * CLK; e += CLT * CLT) {
            const int side = e / (CLT * CLK), r = (e / CLK) % CLT, k = e % CLK;
            const int64_t row = (int64_t)(side ? J : I) * CLT + r;
            const double v = (row < N && k0 + k < E) ? a.X[row * E + k0 + k] : 0.0;
            if (side) xj[r][k] = v;
            else xi[r][k] = v;
        }
        __syncthreads();
        const int kn = (int)(E - k0 < CLK ? E - k0 : CLK);
        for (int k = 0; k < kn; k++) {
            const double df = xi[ti][k] - xj[tj][k];
            d2 = d2 + df * df;
        }
        __syncthreads();
    }
    if (i < j && j < N && sqrt(d2) <= a.thr) uf_unite(a.par, (int)i, (int)j);
}

// members per union-find root
__global__ void __launch_bounds__(BT) k_cl_roots(pcx_mat m, ClusterArgs a) {
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const int r = uf_find(a.par, (int)i);
        a.lab[i] = r;
        atomicAdd(a.cnt + r, 1);
    }
}

// nc from the cluster sizes (:398-405, :412-419): (size - min size) / sum, integer sums
// exact; all clusters the same size give 0 / 0 = NaN like numpy.  size_i = cnt[lab[i]].
__global__ void __launch_bounds__(1024) k_cl_nc(pcx_mat m, ClusterArgs a) {
    __shared__ int mn;
    __shared__ unsigned long long tot;
    const int64_t N = m.n_rows;
    if (threadIdx.x == 0) {
        mn = 0x7fffffff;
        tot = 0;
    }
    __syncthreads();
    int lmin = 0x7fffffff;
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) lmin = min(lmin, a.cnt[a.lab[i]]);
    atomicMin(&mn, lmin);
    __syncthreads();
    unsigned long long lt = 0;
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) lt += (unsigned long long)(a.cnt[a.lab[i]] - mn);
    atomicAdd(&tot, lt);
    __syncthreads();
    double* nc = m.rowv + RV_N1 * N;
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x)
        nc[i] = (double)(a.cnt[a.lab[i]] - mn) / (double)tot;
}

// ---------------------------------------------------------------- clusterfeck
// block-wide argmin of (d, x) (first minimum) / argmax of (v, x) (first maximum)
__device__ void cl_argbest(double& v, int& x, bool mx, double* sv, int* sx) {
    const int t = threadIdx.x;
    sv[t] = v;
    sx[t] = x;
    __syncthreads();
    for (int s = blockDim.x / 2; s >= 1; s >>= 1) {
        if (t < s) {
            const double v2 = sv[t + s];
            const int x2 = sx[t + s];
            const bool take = x2 >= 0 && (sx[t] < 0 || (mx ? v2 > sv[t] : v2 < sv[t]) || (v2 == sv[t] && x2 < sx[t]));
            if (take) {
                sv[t] = v2;
                sx[t] = x2;
            }
        }
        __syncthreads();
    }
    v = sv[0];
    x = sx[0];
    __syncthreads();
}

// mean vector of cluster x (newMean, :151-157): a singleton's row, else running sums / weight
__device__ __forceinline__ double feck_mean_k(const ClusterArgs& a, int64_t E, int x, int64_t k) {
    return a.cnt[x] == 1 ? a.X[(int64_t)a.par[x] * E + k] : a.S[(int64_t)x * E + k] / a.crep[x];
}

// L2dist (:148-149): sqrt(np.sum((v1 - v2)**2)), numpy pairwise sum
template <class A, class B>
__device__ __forceinline__ double feck_l2(A u, B v, int64_t E) {
    return sqrt(pw_sum_dev([&](int64_t k) { const double d = u(k) - v(k); return d * d; }, E));
}

// Oracle.cluster (:194-230): rows in order join the nearest cluster (first minimum) when its
// mean is closer than thr, else found a new cluster (rows with NaN never do); returns the mode
// (first cluster of largest weight, :162-165)
__device__ int feck_pass(const pcx_mat& m, const ClusterArgs& a, double thr, double* sv, int* sx, int* nclus) {
    const int64_t N = m.n_rows, E = m.n_events;
    if (threadIdx.x == 0) *nclus = 0;
    __syncthreads();
    for (int64_t i = 0; i < N; i++) {
        const int n = *nclus;
        double bd = 0x1p255;
        int bx = -1;
        for (int x = threadIdx.x; x < n; x += blockDim.x) {
            const double d = feck_l2([&](int64_t k) { return a.X[i * E + k]; },
                                     [&](int64_t k) { return feck_mean_k(a, E, x, k); }, E);
            if (d < bd) {
                bd = d;
                bx = x;
            }
        }
        cl_argbest(bd, bx, false, sv, sx);
        if (bx >= 0 && bd < thr) {
            const double wi = a.wtok[i];
            for (int64_t k = threadIdx.x; k < E; k += blockDim.x)
                a.S[(int64_t)bx * E + k] = a.S[(int64_t)bx * E + k] + a.X[i * E + k] * wi;
            __syncthreads();  // the sums read cnt == 1 rows above: bump the count after them
            if (threadIdx.x == 0) {
                a.crep[bx] = a.crep[bx] + wi;
                a.cnt[bx] += 1;
                a.lab[i] = bx;
            }
        } else {
            int nan = 0;
            for (int64_t k = threadIdx.x; k < E; k += blockDim.x) nan |= __builtin_isnan(a.X[i * E + k]) ? 1 : 0;
            nan = __syncthreads_or(nan);
            if (!nan) {
                const double wi = a.wtok[i];
                for (int64_t k = threadIdx.x; k < E; k += blockDim.x) a.S[(int64_t)n * E + k] = a.X[i * E + k] * wi;
                if (threadIdx.x == 0) {
                    a.par[n] = (int)i;
                    a.cnt[n] = 1;
                    a.crep[n] = wi;
                    a.lab[i] = n;
                    *nclus = n + 1;
                }
            } else if (threadIdx.x == 0) {
                a.lab[i] = -1;
            }
        }
        __syncthreads();
    }
    const int n = *nclus;
    double top = 0.0;
    int mode = -1;
    for (int x = threadIdx.x; x < n; x += blockDim.x)
        if (a.crep[x] > top) {
            top = a.crep[x];
            mode = x;
        }
    cl_argbest(top, mode, true, sv, sx);
    return mode;
}

// per-row distance of its cluster's mean to the mode's mean (:177-183), into dm
__device__ void feck_rowdist(const pcx_mat& m, const ClusterArgs& a, int mode, int n, double* dm) {
    const int64_t N = m.n_rows, E = m.n_events;
    for (int x = threadIdx.x; x < n; x += blockDim.x)
        a.dist[x] = feck_l2([&](int64_t k) { return feck_mean_k(a, E, mode, k); },
                            [&](int64_t k) { return feck_mean_k(a, E, x, k); }, E);
    __syncthreads();
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) dm[i] = a.lab[i] >= 0 ? a.dist[a.lab[i]] : 0.0;
    __syncthreads();
}

// clusterfeck: outsideCluster(reports_filled, reptokens) (:185-196, :150-183), one workgroup
__global__ void __launch_bounds__(1024) k_cl_feck(pcx_mat m, ClusterArgs a) {
    __shared__ double sv[1024];
    __shared__ int sx[1024];
    __shared__ int nclus;
    __shared__ double dsh[2];
    const int64_t N = m.n_rows, E = m.n_events;
    const int mode1 = feck_pass(m, a, a.thr, sv, sx, &nclus);
    if (threadIdx.x == 0)
        dsh[0] = mode1 < 0 ? __builtin_nan("")
                           : feck_l2([&](int64_t k) { return feck_mean_k(a, E, mode1, k); },
                                     [&](int64_t k) { return a.outc[k]; }, E);
    __syncthreads();
    const double d1 = dsh[0];
    if (mode1 >= 0) feck_rowdist(m, a, mode1, nclus, a.dm);
    if (d1 > 1.07) {  // a far mode re-clusters once with 3 x the threshold (:172-174)
        const int mode2 = feck_pass(m, a, a.thr * 3.0, sv, sx, &nclus);
        if (threadIdx.x == 0)
            dsh[1] = mode2 < 0 ? __builtin_nan("")
                               : feck_l2([&](int64_t k) { return feck_mean_k(a, E, mode2, k); },
                                         [&](int64_t k) { return a.outc[k]; }, E);
        __syncthreads();
        if (dsh[1] < d1) feck_rowdist(m, a, mode2, nclus, a.dm);
    }
    if (threadIdx.x == 0) {  // np.amax (NaN propagates); rv = 1 - dm / (max + 1e-8); normalize
        double mx = a.dm[0];
        for (int64_t i = 1; i < N; i++) {
            const double v = a.dm[i];
            if (__builtin_isnan(v) || v > mx) mx = __builtin_isnan(mx) ? mx : v;
        }
        dsh[0] = mx;
    }
    __syncthreads();
    const double mx = dsh[0];
    double* rv = a.dist;
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) rv[i] = fabs(1.0 - a.dm[i] / (mx + 0.00000001));
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = pw_sum_dev([&](int64_t i) { return rv[i]; }, N);
        dsh[0] = s;
        dsh[1] = s == 0.0 ? pw_sum_dev([&](int64_t i) { return rv[i] + 1.0; }, N) : s;
    }
    __syncthreads();
    double* nc = m.rowv + RV_N1 * N;
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) nc[i] = nweight(rv[i], dsh[0], dsh[1]);
}

// ---------------------------------------------------------------- k-means
enum km_state { KS_PREV0 = 0, KS_PREV1, KS_BEST, KS_CONT, KS_NCODES, KS_BESTN, KS_IT, KS_FIRST };

// scipy _vq distance^2 (SPEC vq_d2): E < 5 the naive loop; else -2 x.c (one fma chain for
// E < 32, eight interleaved chains summed as a tree from 32) + |x|^2 + |c|^2
__device__ __forceinline__ double km_d2(const double* x, const double* c, int64_t E, double xs, double cs) {
    if (E < 5) {
        double s = 0.0;
        for (int64_t k = 0; k < E; k++) {
            const double d = x[k] - c[k];
            s = s + d * d;
        }
        return s;
    }
    double dot;
    if (E < 32) {
        dot = 0.0;
        for (int64_t k = 0; k < E; k++) dot = fma(x[k], c[k], dot);
    } else {
        double q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int64_t k = 0; k < E; k++) q[k & 7] = fma(x[k], c[k], q[k & 7]);
        dot = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
    }
    return (-2.0 * dot + xs) + cs;
}

__device__ __forceinline__ double km_sq(const double* x, int64_t E) {
    double s = 0.0;
    for (int64_t k = 0; k < E; k++) s = s + x[k] * x[k];
    return s;
}

__global__ void __launch_bounds__(BT) k_km_init(pcx_mat m, ClusterArgs a) {
    const int64_t E = m.n_events, n = (int64_t)a.k * E;
    for (int64_t idx = blockIdx.x * (int64_t)BT + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * BT) {
        const int64_t c = idx / E, k = idx % E;
        a.book[idx] = a.X[(int64_t)a.kinit[(int64_t)a.restart * a.k + c] * E + k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.kst[KS_PREV0] = __builtin_inf();
        a.kst[KS_PREV1] = __builtin_inf();
        a.kst[KS_NCODES] = a.k;
        a.kst[KS_IT] = 0;
        a.kst[KS_FIRST] = 1;
        a.kst[KS_CONT] = 1;
        if (a.restart == 0) {
            a.kst[KS_BEST] = __builtin_inf();
            a.kst[KS_BESTN] = 0;
        }
    }
}

__global__ void __launch_bounds__(BT) k_km_cs(pcx_mat m, ClusterArgs a, const double* book) {
    const int c = blockIdx.x * BT + threadIdx.x;
    if (c < (int)a.kst[KS_NCODES]) a.cs[c] = km_sq(book + (int64_t)c * m.n_events, m.n_events);
}

// vq (:397-398): nearest code (first minimum) and its distance of every row
__global__ void __launch_bounds__(BT) k_km_vq(pcx_mat m, ClusterArgs a, const double* book) {
    const int64_t E = m.n_events;
    const int nc = (int)a.kst[KS_NCODES];
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) {
        const double* x = a.X + i * E;
        const double xs = km_sq(x, E);
        double low = __builtin_inf();
        int l = 0;
        for (int c = 0; c < nc; c++) {
            const double d = km_d2(x, book + (int64_t)c * E, E, xs, a.cs[c]);
            if (d < low) {
                low = d;
                l = c;
            }
        }
        a.lab[i] = l;
        a.dist[i] = low > 0 ? sqrt(low) : 0.0;
    }
}

// one Lloyd step after vq (scipy _kmeans): mean distortion (np.mean, pairwise), member sums in
// row order / counts, empty codes dropped, |avg_prev - avg| > 1e-5 continues
__global__ void __launch_bounds__(1024) k_km_update(pcx_mat m, ClusterArgs a) {
    const int64_t N = m.n_rows, E = m.n_events;
    const int nc = (int)a.kst[KS_NCODES];
    __shared__ int keep[1024];  // new index of each code (-1: empty); nc <= 1024 (host-checked)
    for (int c = threadIdx.x; c < nc; c += blockDim.x) a.cnt[c] = 0;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) atomicAdd(a.cnt + a.lab[i], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        const double avg = pw_sum_dev([&](int64_t i) { return a.dist[i]; }, N) / (double)N;
        if (a.kst[KS_FIRST] != 0) {
            a.kst[KS_PREV1] = avg;
            a.kst[KS_FIRST] = 0;
        } else {
            a.kst[KS_PREV0] = a.kst[KS_PREV1];
            a.kst[KS_PREV1] = avg;
        }
        int mm = 0;
        for (int c = 0; c < nc; c++) keep[c] = a.cnt[c] > 0 ? mm++ : -1;
        a.kst[KS_NCODES] = mm;
        const double diff = fabs(a.kst[KS_PREV0] - a.kst[KS_PREV1]);
        const double it = a.kst[KS_IT] + 1;
        a.kst[KS_IT] = it;
        a.kst[KS_CONT] = (diff > 1e-5 && it < 4096) ? 1 : 0;  // 4096: the device's guard (SPEC KMEANS_MAXIT)
    }
    __syncthreads();
    for (int64_t idx = threadIdx.x; idx < (int64_t)nc * E; idx += blockDim.x) {
        const int c = (int)(idx / E);
        if (keep[c] >= 0) a.book[(int64_t)keep[c] * E + idx % E] = a.S[idx] / (double)a.cnt[c];
    }
}

// update_cluster_means: the member sum of (code c, feature k) in row order, one thread each
__global__ void __launch_bounds__(BT) k_km_sums(pcx_mat m, ClusterArgs a) {
    const int64_t N = m.n_rows, E = m.n_events;
    const int64_t n = (int64_t)a.kst[KS_NCODES] * E;
    for (int64_t idx = blockIdx.x * (int64_t)BT + threadIdx.x; idx < n; idx += (int64_t)gridDim.x * BT) {
        const int c = (int)(idx / E);
        const int64_t k = idx % E;
        double s = 0.0;
        for (int64_t i = 0; i < N; i++)
            if (a.lab[i] == c) s = s + a.X[i * E + k];
        a.S[idx] = s;
    }
}

// best restart by final mean distortion (strictly smaller wins)
__global__ void __launch_bounds__(1024) k_km_keep(pcx_mat m, ClusterArgs a) {
    __shared__ int take;
    const int64_t E = m.n_events;
    if (threadIdx.x == 0) {
        take = a.kst[KS_PREV1] < a.kst[KS_BEST];
        if (take) {
            a.kst[KS_BEST] = a.kst[KS_PREV1];
            a.kst[KS_BESTN] = a.kst[KS_NCODES];
        }
    }
    __syncthreads();
    if (!take) return;
    const int64_t n = (int64_t)a.kst[KS_NCODES] * E;
    for (int64_t idx = threadIdx.x; idx < n; idx += blockDim.x) a.best[idx] = a.book[idx];
}

__global__ void k_km_final_prep(ClusterArgs a) {
    if (threadIdx.x == 0) a.kst[KS_NCODES] = a.kst[KS_BESTN];
}

// no restart with a finite distortion (best_n == 0): the reference raises; nc = NaN
__global__ void __launch_bounds__(BT) k_km_nc_nan(pcx_mat m, ClusterArgs a) {
    if (a.kst[KS_BESTN] != 0) return;
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT)
        m.rowv[RV_N1 * m.n_rows + i] = __builtin_nan("");
}

__global__ void __launch_bounds__(BT) k_km_count(pcx_mat m, ClusterArgs a) {
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT)
        atomicAdd(a.cnt + a.lab[i], 1);
}

__global__ void __launch_bounds__(BT) k_cl_zero_cnt(pcx_mat m, ClusterArgs a) {
    for (int64_t i = blockIdx.x * (int64_t)BT + threadIdx.x; i < m.n_rows; i += (int64_t)gridDim.x * BT) a.cnt[i] = 0;
}

}  // namespace

// ------------------------------------------------------------------ stage dispatcher
const char* stage_name(int k) {
    static const char* names[M_NSTAGE] = {
        "none", "REPUTATION", "COLSTATS", "GUESS", "MEAN", "COV", "COV_REDUCE", "COV_FINISH", "POWER",
        "SCORES", "NCSUMS", "GEMV2", "DECIDE", "REPU", "SMOOTH", "OUTCOMES", "EVENTS", "SCALED_CERT", "FINAL",
        "ROWSUMS", "AGENTS", "MATRICES", "WCD", "EIG", "ZERO_LOADING", "NC_OUT", "WMEAN_OUT", "SEL_EXACT",
        "SEL_INIT", "SEL_START", "SEL_ARGMAX", "SEL_VALUE", "SEL_VALUE_FINISH", "SEL_COMPACT", "SEL_HIST",
        "SEL_STEP", "SEL_FINISH", "HARD_LIST", "HARD_GATHER", "HARD_PREP", "HARD_SORT", "HARD_WALK", "EXCHANGE",
        "H2D", "D2H", "COV_PLAN", "COV_I8", "CLUSTER", "COV_GUARD", "COV_REST", "WCD_REBUILD"};
    return (k >= 0 && k < M_NSTAGE) ? names[k] : "";
}

hipError_t tri_pack(const double* C, double* buf, int64_t E, int unpack, hipStream_t st) {
    const int64_t n = E * (E + 1) / 2;
    hipLaunchKernelGGL(k_tri_pack, dim3(grid_rows(n, BT)), dim3(BT), 0, st, (double*)C, buf, E, unpack);
    return hipGetLastError();
}

hipError_t copy2d(double* dst, int64_t dpitch, const double* src, int64_t spitch, int64_t width, int64_t rows,
                  hipStream_t st) {
    if (width <= 0 || rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_copy2d, dim3(grid_rows(width * rows, BT)), dim3(BT), 0, st, dst, dpitch, src, spitch, width,
                       rows);
    return hipGetLastError();
}

hipError_t cluster_stage(pcx_mat& m, const ClusterArgs& a, int step, hipStream_t st, std::string& err) {
    const int E = (int)m.n_events;
    const int ceb = (E + BT - 1) / BT;
    const int rg = grid_rows(m.n_rows, BT);
    const int eg = grid_rows(m.n_rows * (int64_t)E, BT);
    switch (step) {
        case CL_WTOK:
            hipLaunchKernelGGL(k_cl_wtok, dim3(rg), dim3(BT), 0, st, m, a);
            break;
        case CL_MU:  // weights -> a.mu (wpca mean) or a.outc (clusterfeck outcomes): by a.weights
            hipLaunchKernelGGL(k_cl_mu, dim3(ceb), dim3(BT), 0, st, m, a, a.weights == m.rep ? a.mu : a.outc);
            break;
        case CL_X_WCD:
            hipLaunchKernelGGL(k_cl_x, dim3(eg), dim3(BT), 0, st, m, a, 1);
            break;
        case CL_X_F:
            hipLaunchKernelGGL(k_cl_x, dim3(eg), dim3(BT), 0, st, m, a, 0);
            break;
        case CL_WHITEN:
            hipLaunchKernelGGL(k_cl_sd, dim3(ceb), dim3(BT), 0, st, m, a);
            hipLaunchKernelGGL(k_cl_div, dim3(eg), dim3(BT), 0, st, m, a);
            break;
        case CL_HIER: {
            const unsigned nt = (unsigned)((m.n_rows + CLT - 1) / CLT);
            hipLaunchKernelGGL(k_cl_iota, dim3(rg), dim3(BT), 0, st, m, a);
            hipLaunchKernelGGL(k_cl_hier, dim3(nt, nt), dim3(CLT * CLT), 0, st, m, a);
            hipLaunchKernelGGL(k_cl_roots, dim3(rg), dim3(BT), 0, st, m, a);
            hipLaunchKernelGGL(k_cl_nc, dim3(1), dim3(1024), 0, st, m, a);
            break;
        }
        case CL_FECK:
            hipLaunchKernelGGL(k_cl_feck, dim3(1), dim3(1024), 0, st, m, a);
            break;
        case KM_INIT:
            hipLaunchKernelGGL(k_km_init, dim3(grid_rows((int64_t)a.k * E, BT)), dim3(BT), 0, st, m, a);
            break;
        case KM_ITER:
            hipLaunchKernelGGL(k_km_cs, dim3((a.k + BT - 1) / BT), dim3(BT), 0, st, m, a, (const double*)a.book);
            hipLaunchKernelGGL(k_km_vq, dim3(rg), dim3(BT), 0, st, m, a, (const double*)a.book);
            hipLaunchKernelGGL(k_km_sums, dim3(grid_rows((int64_t)a.k * E, BT)), dim3(BT), 0, st, m, a);
            hipLaunchKernelGGL(k_km_update, dim3(1), dim3(1024), 0, st, m, a);
            break;
        case KM_KEEP:
            hipLaunchKernelGGL(k_km_keep, dim3(1), dim3(1024), 0, st, m, a);
            break;
        case KM_FINAL:
            hipLaunchKernelGGL(k_km_final_prep, dim3(1), dim3(64), 0, st, a);
            hipLaunchKernelGGL(k_km_cs, dim3((a.k + BT - 1) / BT), dim3(BT), 0, st, m, a, (const double*)a.best);
            hipLaunchKernelGGL(k_km_vq, dim3(rg), dim3(BT), 0, st, m, a, (const double*)a.best);
            hipLaunchKernelGGL(k_cl_zero_cnt, dim3(rg), dim3(BT), 0, st, m, a);
            hipLaunchKernelGGL(k_km_count, dim3(rg), dim3(BT), 0, st, m, a);
            hipLaunchKernelGGL(k_cl_nc, dim3(1), dim3(1024), 0, st, m, a);
            hipLaunchKernelGGL(k_km_nc_nan, dim3(rg), dim3(BT), 0, st, m, a);
            break;
        default:
            err = "cluster_stage: unknown step";
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t hard_stage(pcx_mat& m, const HardArgs& h, int stage, hipStream_t st, std::string& err) {
    if (h.n_hard <= 0) return hipSuccess;
    switch (stage) {
        case M_HARD_GATHER:
            hipLaunchKernelGGL(k_hard_gather, dim3(h.n_hard), dim3(1024), 0, st, m, h);
            break;
        case M_HARD_PREP:
            hipLaunchKernelGGL(k_hard_prep, dim3(h.n_hard), dim3(1024), 0, st, m, h);
            break;
        case M_HARD_SORT: {
            // bitonic network over n_hard contiguous segments of P (a power of two)
            const int64_t P = h.P, total = P * h.n_hard;
            const int64_t tile = P < BS_TILE ? P : BS_TILE;
            const unsigned nblk = (unsigned)(total / tile);
            hipLaunchKernelGGL(k_bsort_lds, dim3(nblk), dim3(1024), 0, st, h.keys, P, (int64_t)0);
            for (int64_t size = tile * 2; size <= P; size <<= 1) {
                for (int64_t stride = size >> 1; stride >= tile; stride >>= 1)
                    hipLaunchKernelGGL(k_bsort_global, dim3(grid_rows(total / 2, BT)), dim3(BT), 0, st, h.keys, P,
                                       total, size, stride);
                hipLaunchKernelGGL(k_bsort_lds, dim3(nblk), dim3(1024), 0, st, h.keys, P, size);
            }
            break;
        }
        case M_HARD_WALK:
            hipLaunchKernelGGL(k_hard_walk, dim3(h.n_hard), dim3(1024), 0, st, m, h);
            break;
        default:
            err = "hard_stage: unknown stage";
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// the compact column passes: general tile positions [0, gb) and grid positions [gb, E) as two
// launches of the same row chunks (blockIdx.y)
template <class KG, class KR>
static void launch_compact(KG kgen, KR kgrid, const pcx_mat& m, hipStream_t st) {
    const int64_t E = m.n_events, gb = std::min<int64_t>((int64_t)m.cov_jb * CT, E);
    if (gb > 0) hipLaunchKernelGGL(kgen, dim3((unsigned)((gb + BT - 1) / BT), m.col_blocks), dim3(BT), 0, st, m);
    if (E > gb) hipLaunchKernelGGL(kgrid, dim3((unsigned)((E - gb + BT - 1) / BT), m.col_blocks), dim3(BT), 0, st, m);
}

// the int8-MFMA weighted counts (k_outcomes_mf, k_gemv2_mf) need row chunks of at most 2^24 rows:
// their int32 digit sums are then exact
// (and only on a large grid block: at C4's 100k x 743 grid events the subset-table kernels take
// 0.15 / 0.18 ms against 0.19 / 0.20 with the digit passes' launches)
static bool wdig_fits(const pcx_mat& m) {
    if (!m.wdig) return false;
    const int64_t per = ((m.n_rows + m.col_blocks - 1) / m.col_blocks + 15) / 16 * 16;
    const int64_t ng = m.n_events - std::min<int64_t>((int64_t)m.cov_jb * CT, m.n_events);
    return per <= ((int64_t)1 << 24) && m.n_rows * ng >= ((int64_t)1 << 27);
}
// the digits of each weight vector (vector v = the v-th of ws, its largest |w| in header word slots[v])
static void wdig_prepare(const pcx_mat& m, std::initializer_list<const double*> ws, std::initializer_list<int> slots,
                         hipStream_t st) {
    const int64_t rb = std::max<int64_t>(1, (m.n_rows + BT - 1) / BT);
    int v = 0;
    auto sl = slots.begin();
    for (const double* w : ws) {
        hipLaunchKernelGGL(k_wdigits, dim3((unsigned)std::min<int64_t>(rb + 1, 4096)), dim3(BT), 0, st, m, w, v, *sl);
        v++;
        sl++;
    }
}

hipError_t mat_stage(pcx_mat& m, int stage, hipStream_t st, std::string& err) {
    const int E = (int)m.n_events;
    const int ceb = (E + BT - 1) / BT;
    const dim3 colgrid(ceb, m.col_blocks);
    const int rg = grid_rows(m.n_rows, BT);
    const int sg = (m.n_scaled + BT - 1) / BT;
    switch (stage) {
        case M_REPUTATION:
            if (m.rep_raw) hipLaunchKernelGGL(k_rep_total, dim3(1), dim3(1024), 0, st, m);
            hipLaunchKernelGGL(k_rep_local, dim3(rg), dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_spart_finish, dim3(2), dim3(BT), 0, st, m, rg, 2, (int)SC_TOK, 0);
            hipLaunchKernelGGL(k_spart_finish, dim3(1), dim3(BT), 0, st, m, rg, 1, (int)SC_BIGTOK, 2);
            hipLaunchKernelGGL(k_spart_max, dim3(1), dim3(BT), 0, st, m, rg, (int)SC_MAXTOK, 3);
            if (m.ob_order) hipLaunchKernelGGL(k_ob_sums, dim3(1), dim3(64), 0, st, m, 0);
            break;
        case M_COLSTATS:
            if (m.rep_raw)
                hipLaunchKernelGGL((m.int_dtype ? k_colstats<false, true> : k_colstats<false, false>), colgrid, dim3(BT), 0, st, m);
            else
                hipLaunchKernelGGL((m.int_dtype ? k_colstats<true, true> : k_colstats<true, false>), colgrid, dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_col_finish, dim3((E + BT / WAVE - 1) / (BT / WAVE)), dim3(BT), 0, st, m, m.col_blocks, 4, 0, 1);
            break;
        case M_GUESS:
            hipLaunchKernelGGL(k_guess, dim3(ceb), dim3(BT), 0, st, m);
            break;
        case M_MEAN:
            hipLaunchKernelGGL(k_mean, dim3(ceb), dim3(BT), 0, st, m);
            break;
        case M_COV_PLAN:
            if (!m.cov_perm || !m.cov_pos) {
                err = "M_COV_PLAN: permutation workspace missing";
                return hipErrorInvalidValue;
            }
            hipLaunchKernelGGL(k_cov_plan, dim3(1), dim3(1024), 0, st, m);
            break;
        case M_COV_I8: {
            const int nb = (int)(m.wcd_ld / CT);
            if (m.cov_jb >= nb && m.zq == 0) break;  // no grid events
            const int gb = m.cov_jb * CT;
            const int np = (int)(m.n_events - gb);  // grid positions
            if (!m.zA || !m.zB || !m.zsum || !m.Pgg || m.cov_jb < 0 || m.cov_jb > nb || m.zq < np || m.ks_gg < 1 ||
                (m.cov_mixed && m.ks_mx < 1) || m.zq % GT || m.wcd_rows % (64 * G_KS) ||
                (m.cov_mixed && (!m.zD || !m.Pmx || !m.dscale || !m.dtok)) ||
                (m.cov_gg8 && (!m.cov_mixed || !m.compact || !m.Fg || !m.zE || !m.escale || !m.Pgx || m.ks_gx < 1))) {
                err = "M_COV_I8: int8 operands missing or plan inconsistent";
                return hipErrorInvalidValue;
            }
            static std::once_flag g_once;
            static hipError_t g_err = hipSuccess;
            std::call_once(g_once, [] {
                g_err = hipFuncSetAttribute((const void*)k_gemm_i8<GEMM_I8_WAVES, GEMM_I8_NBUF>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)GEMM_I8_LDS);
            });
            if (g_err != hipSuccess) return g_err;
            const int64_t rg = m.wcd_rows / 16;
            // both products take z (zB, 2-bit packed) as the B operand; the token sums they once
            // carried as an extra position come from k_wcd (Z_j) and k_digits (S_q): a 3,073rd
            // position cost a 13th tile row and column (C5: grid 4.4 ms, mixed 15.3 ms before)
            {  // grid x grid (lower tiles): P = (tok z)^T z, |tok z z| <= 252 per row
                GemmI8 g{m.zA, m.zq, m.zB, m.zq, m.Pgg, m.zq, m.zq * m.zq, np, np, 0, 0, 1, m.ks_gg, rg, 0};
                g.tp = g.tq = (np + GT - 1) / GT;
                hipLaunchKernelGGL((k_gemm_i8<GEMM_I8_WAVES, GEMM_I8_NBUF>), dim3((unsigned)gemm_i8_items(g.tp, g.tq, g.lower, g.kslices)), dim3(GEMM_I8_WAVES * 64),
                                   GEMM_I8_LDS, st, g);
            }
            if (m.cov_mixed) {
                // general digits x grid: digits of tok w (A, PCX_NDIG per general position) times z (B);
                // stored transposed into Pmx [grid position][digit position]; |z d| <= 2 * 127 per row
                // (16 row groups a block at least: 64 left a 125k-row shard's k_digits1 with 492 blocks)
                const int ng = (int)std::min<int64_t>(4096, (rg + 15) / 16);
                // (the digit sums and, past them, the covariance guard's sums)
                if (hipMemsetAsync(m.dtok, 0, ((size_t)(PCX_NDIG + (m.gacc ? G_NSTAT : 0)) * gb + (m.gacc ? 1 : 0)) * 8, st) !=
                    hipSuccess)
                    return hipGetLastError();
                if (m.cov_gg8 && m.zE != m.zD)  // both digit strings
                    hipLaunchKernelGGL(k_digits, dim3((unsigned)((gb + DG_POS - 1) / DG_POS), (unsigned)ng), dim3(BT), 0, st, m);
                else
                    hipLaunchKernelGGL(k_digits1, dim3((unsigned)((gb + BT - 1) / BT), (unsigned)ng), dim3(BT), 0, st, m);
                GemmI8 g{m.zD, zd_ld(gb), m.zB, m.zq, m.Pmx, (int64_t)PCX_NDIG * gb, m.zq * PCX_NDIG * gb, PCX_NDIG * gb, np,
                         0, 0, 0, m.ks_mx, rg, 1};
                g.tp = (PCX_NDIG * gb + GT - 1) / GT;
                g.tq = (np + GT - 1) / GT;
                if ((int64_t)g.tp * GT > g.lda || (int64_t)g.tq * GT > g.ldb) {  // every tile's loads inside a row group
                    err = "M_COV_I8: operand row groups narrower than the tiles";
                    return hipErrorInvalidValue;
                }
                hipLaunchKernelGGL((k_gemm_i8<GEMM_I8_WAVES, GEMM_I8_NBUF>), dim3((unsigned)gemm_i8_items(g.tp, g.tq, g.lower, g.kslices)), dim3(GEMM_I8_WAVES * 64),
                                   GEMM_I8_LDS, st, g);
            }
            if (m.cov_gg8) {
                // general x general: digits of tok w (zD) x digits of w (zE), the digit pairs
                // i + j <= NDIG - 1 over the lower event tiles; |d e| <= 127^2 per row
                static std::once_flag x_once;
                static hipError_t x_err = hipSuccess;
                std::call_once(x_once, [] {
                    x_err = hipFuncSetAttribute((const void*)k_gemm_i8x<GEMM_I8X_WAVES, GEMM_I8X_NBUF>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)GEMM_I8X_LDS);
                });
                if (x_err != hipSuccess) return x_err;
                GemmX g{m.zD, m.zE, zd_ld(gb), zd_ld(gb), m.Pgx, rg, gb, (gb + GT - 1) / GT, PCX_NDIG - 1, m.ks_gx, 0,
                        (int)(m.zE == m.zD)};
                hipLaunchKernelGGL((k_gemm_i8x<GEMM_I8X_WAVES, GEMM_I8X_NBUF>), dim3((unsigned)gemm_i8x_items(g)),
                                   dim3(GEMM_I8X_WAVES * 64), GEMM_I8X_LDS, st, g);
            }
            break;
        }
        case M_WCD:
        case M_COV: {
            const int nb = (int)(m.wcd_ld / CT);
            if (!m.wcd || !m.tokp || !m.rowpart || !m.cov_perm || !m.cov_pos || m.wcd_rows % 64 ||
                m.wcd_rows < m.n_rows || m.wcd_ld % CT || m.wcd_ld < m.n_events || m.cov_jb < 0 || m.cov_jb > nb ||
                m.cov_fp_tiles != (m.cov_gg8     ? 0
                                   : m.cov_mixed ? m.cov_jb * (m.cov_jb + 1) / 2
                                                 : m.cov_jb * nb - m.cov_jb * (m.cov_jb - 1) / 2) ||
                (m.cov_jb < nb && (!m.zA || !m.zB || !m.zsum))) {
                err = "M_COV: wcd workspace missing or mis-sized (wcd_rows % 16, wcd_ld % 128) or no plan";
                return hipErrorInvalidValue;
            }
            if (stage == M_WCD) {
                const int ncb = (int)((m.wcd_ld + WCD_COLS - 1) / WCD_COLS);
                int64_t rb = std::max(1, 4096 / ncb);
                // (but keep >= 1,024 workgroups: at C4's 1,000 events -- two column blocks -- the
                // 768-row floor left 256 workgroups, one per CU: k_wcd 1.03 ms at 2.5 TB/s)
                while (rb > 1 && m.wcd_rows / rb < WCD_MIN_ROWS && (rb / 2) * ncb >= PCX_WCD_MIN_WG) rb /= 2;
                hipLaunchKernelGGL(k_wcd, dim3((unsigned)rb, ncb),
                                   dim3(BT), 0, st, m);
                if (m.zbg && m.Fg && m.cov_jb * CT >= 128) {  // the general tiles' grid events as codes
                    const int64_t groups = (m.n_rows + 15) / 16;
                    hipLaunchKernelGGL(k_zbg, dim3((unsigned)((groups + 1) / 2)), dim3(BT), 0, st, m);
                }
                break;
            }
            static std::once_flag lds_once;
            static hipError_t lds_err = hipSuccess;
            std::call_once(lds_once, [] {
                lds_err = hipFuncSetAttribute((const void*)k_syrk, hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)SY_LDS_BYTES);
            });
            if (lds_err != hipSuccess) return lds_err;
            if (m.cov_fp_tiles > 0)
                hipLaunchKernelGGL(k_syrk, dim3(m.cov_fp_tiles * m.fp_ks), dim3(256), SY_LDS_BYTES, st, m);
            break;
        }
        case M_COV_REDUCE: {  // this rank's slabs -> C in event order (one rank: normalised, flags)
            double* S = m.Mw;  // the token row's S [gb] dd (scratch)
            if (m.cov_mixed && m.cov_jb > 0)
                hipLaunchKernelGGL(k_cov_tokrow, dim3((unsigned)((m.cov_jb * CT + BT - 1) / BT)), dim3(BT), 0, st, m, S);
            if (m.world == 1) hipLaunchKernelGGL(k_info_clear, dim3(1), dim3(1), 0, st, m, (int)IN_FLAGS);
            const int nt = (int)((E + CV_T - 1) / CV_T);
            hipLaunchKernelGGL(k_cov_assemble, dim3((unsigned)(nt * (nt + 1) / 2)), dim3(CV_T * 8), 0, st, m,
                               (const double*)S, (int)(m.world == 1));
            // the guard's sums as doubles (the runner exchanges them with the covariance)
            if (m.cov_mixed && m.gacc && m.gsum && m.cov_jb > 0)
                hipLaunchKernelGGL(k_guard_stats, dim3((unsigned)((G_NSTAT * m.cov_jb * CT + BT) / BT)), dim3(BT), 0,
                                   st, m);
            break;
        }
        case M_COV_GUARD:
            if (!m.cov_mixed || !m.gsum || m.cov_jb < 1) {
                err = "M_COV_GUARD: no int8 covariance to guard";
                return hipErrorInvalidValue;
            }
            hipLaunchKernelGGL(k_cov_guard, dim3(1), dim3(1024), 0, st, m);
            break;
        case M_COV_REST: {  // every digit pair i + j >= NDIG of the general x general product (the guard)
            if (!m.cov_gg8 || !m.Pgx || m.ks_gx < 1 || m.gg_smax != 2 * PCX_NDIG - 2) {
                err = "M_COV_REST: no general x general int8 product";
                return hipErrorInvalidValue;
            }
            const int gb = m.cov_jb * CT;
            const int64_t rg = m.wcd_rows / 16;
            GemmX g{m.zD, m.zE, zd_ld(gb), zd_ld(gb), m.Pgx, rg, gb, (gb + GT - 1) / GT, 2 * PCX_NDIG - 2, m.ks_gx,
                    PCX_NDIG, (int)(m.zE == m.zD)};
            hipLaunchKernelGGL((k_gemm_i8x<GEMM_I8X_WAVES, GEMM_I8X_NBUF>), dim3((unsigned)gemm_i8x_items(g)),
                               dim3(GEMM_I8X_WAVES * 64), GEMM_I8X_LDS, st, g);
            break;
        }
        case M_WCD_REBUILD: {  // args: m.cov_gg8 still as it ran (general positions from Fg)
            if (!m.wcd || !m.zB || m.cov_jb < 1 || (m.cov_gg8 && !m.Fg) || m.wcd_rows % 16) {
                err = "M_WCD_REBUILD: operands missing";
                return hipErrorInvalidValue;
            }
            const int64_t ng = m.wcd_rows / 16;
            hipLaunchKernelGGL(k_wcd_rebuild, dim3((unsigned)std::min<int64_t>(ng, 2048), (unsigned)((E + BT - 1) / BT)),
                               dim3(BT), 0, st, m, (int)m.cov_gg8);
            break;
        }
        case M_COV_FINISH: {  // several ranks: the exchanged sum normalised, then the flags
            if (m.world == 1) break;  // (done by k_cov_assemble)
            const int64_t n = (int64_t)E * E;
            hipLaunchKernelGGL(k_cov_finish, dim3((unsigned)((n + BT - 1) / BT)), dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_info_clear, dim3(1), dim3(1), 0, st, m, (int)IN_FLAGS);
            hipLaunchKernelGGL(k_pi_check, dim3(grid_rows(n, BT)), dim3(BT), 0, st, m);
            break;
        }
        case M_SCORES:
            hipLaunchKernelGGL(k_skey_init, dim3(1), dim3(1), 0, st, m);
            if ((m.algorithm == 0 || m.algorithm == 2 || m.algorithm == 3) && !m.scores_given && m.wcd && m.rowpart &&
                m.cov_perm && m.cov_mixed)
            {
                hipLaunchKernelGGL(k_scores_prep, dim3(1), dim3(WAVE), 0, st, m);
                hipLaunchKernelGGL(k_scores_grid, dim3(grid_rows((m.n_rows + 15) / 16, BT / WAVE)), dim3(BT), 0, st, m);
            }
            else if ((m.algorithm == 0 || m.algorithm == 2 || m.algorithm == 3) && !m.scores_given && m.wcd &&
                     m.rowpart && m.cov_perm)
                hipLaunchKernelGGL(k_scores_wcd, dim3(grid_rows(m.n_rows, BT / WAVE)), dim3(BT), 0, st, m);
            else
                hipLaunchKernelGGL(k_scores, dim3(grid_rows(m.n_rows, BT / WAVE)), dim3(BT), 0, st, m);
            break;
        case M_NCSUMS:
            hipLaunchKernelGGL(k_ncsums, dim3(rg), dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_spart_finish, dim3(4), dim3(BT), 0, st, m, rg, 4, (int)SC_A1);
            if (m.ob_order) hipLaunchKernelGGL(k_ob_sums, dim3(1), dim3(64), 0, st, m, 1);
            break;
        case M_GEMV2:
            hipLaunchKernelGGL(k_nweights, dim3(rg), dim3(BT), 0, st, m);
            if (m.compact && m.Fg && m.nam && m.zB)
            {
                pcx_mat mm = m;
                if (!wdig_fits(m)) mm.wdig = nullptr;
                const int64_t gbp = std::min<int64_t>((int64_t)m.cov_jb * CT, E);
                if (mm.wdig && E > gbp) {  // the grid positions on int8 MFMA (k_gemv2_c<true> then exits)
                    wdig_prepare(mm, {m.rowv + RV_N1 * m.n_rows, m.rowv + RV_N2 * m.n_rows}, {(int)WD_N1, (int)WD_N2}, st);
                    // (from n_general, a device value > gb - 128: the waves past E exit)
                    const int64_t from = std::max<int64_t>(0, gbp - 128);
                    hipLaunchKernelGGL(k_gemv2_mf, dim3((unsigned)((E - from + 63) / 64), m.col_blocks), dim3(BT), 0, st, mm);
                }
                launch_compact(k_gemv2_c<false>, k_gemv2_c<true>, mm, st);
            }
            else
                hipLaunchKernelGGL(k_gemv2, colgrid, dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_col_finish, dim3((E + BT / WAVE - 1) / (BT / WAVE)), dim3(BT), 0, st, m, m.col_blocks, 2, 4, 0);
            break;
        case M_DECIDE:
            hipLaunchKernelGGL(k_decide_prep, dim3(ceb), dim3(BT), 0, st, m);
            if (m.rank_rule) {  // cslab is free after the covariance: int scratch of the rank counts
                int* cnt = (int*)m.cslab;
                (void)hipMemsetAsync(cnt, 0, (size_t)E * 6 * sizeof(int), st);
                hipLaunchKernelGGL(k_rank_counts, dim3(ceb, (E + RK_CH - 1) / RK_CH), dim3(BT), 0, st, m, cnt);
                hipLaunchKernelGGL(k_ranks, dim3(ceb), dim3(BT), 0, st, m, (const int*)cnt);
            }
            hipLaunchKernelGGL(k_decide, dim3(1), dim3(1024), 0, st, m);
            break;
        case M_REPU:
            hipLaunchKernelGGL(k_repu, dim3(rg), dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_spart_finish, dim3(2), dim3(BT), 0, st, m, rg, 2, (int)SC_U);
            if (m.ob_order) hipLaunchKernelGGL(k_ob_sums, dim3(1), dim3(64), 0, st, m, 2);
            break;
        case M_SMOOTH:
            hipLaunchKernelGGL(k_smooth, dim3(rg), dim3(BT), 0, st, m);
            break;
        case M_OUTCOMES:
            if (m.compact && m.Fg && m.nam && m.zB) {
                // the int8-MFMA sums when the chunks keep them int32-exact (<= 2^24 rows)
                pcx_mat mm = m;
                if (!wdig_fits(m)) mm.wdig = nullptr;
                if (mm.wdig) {
                    wdig_prepare(mm, {m.rowv + RV_SMOOTH * m.n_rows}, {(int)WD_SMOOTH}, st);
                    hipLaunchKernelGGL(k_outcomes_mf, dim3((unsigned)((E + 63) / 64), m.col_blocks), dim3(BT), 0, st, mm);
                }
                hipLaunchKernelGGL(k_outcomes_c, colgrid, dim3(BT), 0, st, mm);
            } else
                hipLaunchKernelGGL(k_outcomes, colgrid, dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_col_finish, dim3((E + BT / WAVE - 1) / (BT / WAVE)), dim3(BT), 0, st, m, m.col_blocks, 8, 6, 0);
            break;
        case M_EVENTS:
            hipLaunchKernelGGL(k_events, dim3(ceb), dim3(BT), 0, st, m);
            break;
        case M_SCALED_CERT:
            if (m.n_scaled > 0) hipLaunchKernelGGL(k_scaled_cert, dim3(m.n_scaled), dim3(BT), 0, st, m);
            break;
        case M_FINAL:
            hipLaunchKernelGGL(k_final, dim3(1), dim3(1024), 0, st, m);
            break;
        case M_ROWSUMS:
            hipLaunchKernelGGL(k_rowsums, dim3(rg), dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_spart_finish, dim3(2), dim3(BT), 0, st, m, rg, 2, (int)SC_AR);
            break;
        case M_AGENTS:
            hipLaunchKernelGGL(k_agents, dim3(rg), dim3(BT), 0, st, m);
            break;
        case M_NC_OUT:
            hipLaunchKernelGGL(k_nc_out, dim3(rg), dim3(BT), 0, st, m);
            break;
        case M_WMEAN_OUT:
            hipLaunchKernelGGL(k_wmean_out, dim3(ceb), dim3(BT), 0, st, m);
            break;
        case M_SEL_INIT:  // status, key range and the active list of the first histogram pass
            if (m.n_scaled == 0) break;
            hipLaunchKernelGGL(k_sel_setup, dim3(sg), dim3(BT), 0, st, m);
            if (m.sel_phase == 2 || m.rep_raw) {
                const int64_t wb = (m.n_rows + BT - 1) / BT;
                hipLaunchKernelGGL(k_sel_wlimbs, dim3(wb < 512 ? (wb > 0 ? wb : 1) : 512), dim3(BT), 0, st, m);
            }
            hipLaunchKernelGGL(k_sel_range, dim3(sg), dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_sel_compact, dim3(1), dim3(1024), 0, st, m);
            hipLaunchKernelGGL(k_sel_sample, dim3(m.n_scaled), dim3(BT), 0, st, m);
            break;
        case M_SEL_EXACT:
            if (m.n_scaled == 0) break;
            if (m.world != 1 || m.n_rows > SEL_EXACT_MAX) {
                err = "M_SEL_EXACT needs one rank and n_rows <= 8192";
                return hipErrorInvalidValue;
            }
            hipLaunchKernelGGL(k_sel_setup, dim3(sg), dim3(BT), 0, st, m);
            hipLaunchKernelGGL(k_sel_exact, dim3(m.n_scaled), dim3(1024), 0, st, m);
            break;
        case M_SEL_START:
            if (m.n_scaled == 0) break;
            hipLaunchKernelGGL(k_info_clear, dim3(1), dim3(1), 0, st, m, (int)IN_SEL_ARGMAX);
            hipLaunchKernelGGL(k_sel_start, dim3((unsigned)((m.n_scaled + BT / WAVE - 1) / (BT / WAVE))), dim3(BT), 0,
                               st, m);
            break;
        case M_SEL_ARGMAX:
            if (m.n_scaled == 0) break;
            hipLaunchKernelGGL(k_sel_argmax, dim3(m.n_scaled), dim3(BT), 0, st, m);
            break;
        case M_SEL_VALUE:
            if (m.n_scaled == 0) break;
            hipLaunchKernelGGL(k_sel_value, dim3(sg), dim3(BT), 0, st, m);
            break;
        case M_SEL_VALUE_FINISH:
            if (m.n_scaled == 0) break;
            hipLaunchKernelGGL(k_sel_value_finish, dim3(sg), dim3(BT), 0, st, m);
            break;
        case M_SEL_COMPACT:
            hipLaunchKernelGGL(k_sel_compact, dim3(1), dim3(1024), 0, st, m);
            break;
        case M_SEL_FINISH:
            if (m.n_scaled == 0) break;
            hipLaunchKernelGGL(k_sel_finish, dim3(sg), dim3(BT), 0, st, m);
            break;
        case M_POWER: {
            // replicated on every rank (C is identical everywhere); host loop with polling.  The
            // finite / non-zero flags of C come from M_COV_REDUCE (one rank) or M_COV_FINISH and are
            // read by the kernels themselves (pi_mode_of): a non-finite or zero covariance makes every
            // launch below return at once and the first poll see "converged"
            int iters = 0;
            int64_t maxit_flag = 0;
            {
                hipError_t e = hipSuccess;
                hipLaunchKernelGGL(k_pi_start, dim3(1), dim3(1024), 0, st, m);
                const int gb = (E + BT / WAVE - 1) / (BT / WAVE);
                const int nb = (E + CT - 1) / CT;
                const int ntri = nb * (nb + 1) / 2;
                const int64_t nn2 = (int64_t)E * E;
                // iterate on C itself until a squaring is due; M <- (M M) / max|M M| then runs
                // between the two working matrices (the same leading eigenvector, gap ratio squared)
                const double* M = m.C;
                double* Tm = m.Mw;
                // (info word 15: free -- word 8 holds the plan's general count, which the compact
                // passes after this stage read)
                unsigned long long* mxb = (unsigned long long*)&m.info[15];
                const int64_t* fl = &m.info[IN_FLAGS];
                // split-K squaring for E >= 512 when the slabs fit the covariance's (free by now);
                // smaller E keeps the single pass (the goldens' arithmetic)
                const int gks = E >= 512 ? (int)std::min<int64_t>(std::min<int64_t>(8, m.cov_kslices),
                                                                   std::max(1, 1024 / ntri))
                                         : 1;
                auto square = [&]() {
                    (void)hipMemsetAsync(mxb, 0, sizeof(unsigned long long), st);
                    if (gks > 1 && m.cslab) {
                        hipLaunchKernelGGL(k_gram_part, dim3(ntri * gks), dim3(256), 0, st, M, E, m.cslab, gks, fl);
                        const int n32 = (E + GR_T - 1) / GR_T;
                        hipLaunchKernelGGL(k_gram_reduce, dim3(n32 * (n32 + 1) / 2), dim3(256), 0, st,
                                           (const double*)m.cslab, gks, E, Tm, mxb, fl);
                    } else {
                        hipLaunchKernelGGL(k_gram, dim3(ntri), dim3(256), 0, st, M, E, Tm, mxb, fl);
                    }
                    hipLaunchKernelGGL(k_scale, dim3(grid_rows(nn2, BT)), dim3(BT), 0, st, Tm, nn2,
                                       (const unsigned long long*)mxb, fl);
                    const double* sq_out = Tm;
                    Tm = (Tm == m.Mw) ? m.Mw + nn2 : m.Mw;
                    M = sq_out;
                };
                int sq = 0;
                const int presq = E <= 1024 ? 3 : 0;  // small E: squaring is cheaper than iterations
                for (; sq < presq; sq++) square();
                // steps in batches of `poll` between host checks.  Without presquaring (E > 1024)
                // the step that brings delta to PI_TOL raises the converged flag and the batch's
                // later launches return at once; with it, whole batches run (the step count that
                // the golden cases were pinned with: two structurally symmetric events of
                // q_scaled_eq_min keep equal components, tests/parity.py)
                const bool early = presq == 0;
                const int maxit = 2048, poll = 8;
                int since = 0;
                double ps[3] = {1.0, 0.0, 0.0};  // delta, converged, steps (pv_s)
                while (iters < maxit) {
                    for (int k = 0; k < poll; k++) {
                        if (early && E % 2 == 0)
                            hipLaunchKernelGGL(k_pi_gemv4, dim3(gb), dim3(BT), 0, st, m, M, 1);
                        else
                            hipLaunchKernelGGL(k_pi_gemv, dim3(gb), dim3(BT), 0, st, m, M, (int)early);
                        hipLaunchKernelGGL(k_pi_norm, dim3(1), dim3(1024), 0, st, m, (int)early);
                    }
                    e = hipMemcpyAsync(ps, m.pvec + 3 * (E + 64), sizeof(ps), hipMemcpyDeviceToHost, st);
                    if (e == hipSuccess) e = hipStreamSynchronize(st);
                    if (e != hipSuccess) return e;
                    iters = early ? (int)ps[2] : iters + poll;
                    since += poll;
                    if (early ? ps[1] != 0.0 : ps[0] <= PI_TOL_M) break;
                    if (since >= 32 && sq < 8) {
                        square();
                        sq++;
                        since = 0;
                    }
                }
                if (!(ps[0] <= PI_TOL_M)) maxit_flag = 4;
                if (sq > 0)  // polish with C itself (after squarings)
                    for (int k = 0; k < 4; k++) {
                        hipLaunchKernelGGL(k_pi_gemv, dim3(gb), dim3(BT), 0, st, m, (const double*)m.C, 0);
                        hipLaunchKernelGGL(k_pi_norm, dim3(1), dim3(1024), 0, st, m, 0);
                    }
                iters += (sq > 0 ? 4 : 0) + sq;
            }
            hipLaunchKernelGGL(k_pi_finish, dim3(1), dim3(1024), 0, st, m, (int64_t)iters, maxit_flag);
            break;
        }
        case M_MATRICES:
            // (in place with no other matrix asked for: the scaled columns still need their rescale)
            if (m.original || m.filled || (m.orig_inplace && !m.rescaled))
                hipLaunchKernelGGL(k_matrices, colgrid, dim3(BT), 0, st, m);
            break;
        case M_EIG:
            if (m.algorithm != 2 && m.algorithm != 3) break;
            return eig_stage(m, st, err);
        case M_ZERO_LOADING:  // "absolute" / "cokurtosis": no wpca loading
            hipLaunchKernelGGL(k_zero_loading, dim3(1), dim3(256), 0, st, m);
            break;
        default:
            err = "mat_stage: unknown stage " + std::to_string(stage);
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// hard-list compaction (events with m.hard[c] != 0) into cols / modes, count -> info[IN_HARD]
hipError_t hard_list(pcx_mat& m, int32_t* cols, int32_t* modes, hipStream_t st) {
    hipLaunchKernelGGL(k_hard_list, dim3(1), dim3(1024), 0, st, m, cols, modes);
    return hipGetLastError();
}

hipError_t sel_hist(pcx_mat& m, int n_active, hipStream_t st) {
    if (n_active <= 0) return hipSuccess;
    static int ncu = 0;
    if (!ncu) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
            ncu = n;
        if (ncu <= 0) ncu = 256;
    }
    const bool cm = m.sel_phase == 1 && !m.rep_raw && m.n_rows < (1ll << 32);  // (every pass of this phase counts)
    if (n_active <= ncu) {
        if (cm)
            hipLaunchKernelGGL((k_sel_hist<1024, true>), dim3(n_active), dim3(1024), 0, st, m);
        else
            hipLaunchKernelGGL((k_sel_hist<1024, false>), dim3(n_active), dim3(1024), 0, st, m);
    } else if (cm) {  // (49 VGPRs: eight waves per SIMD, so 512 threads an event at four events a CU)
        hipLaunchKernelGGL((k_sel_hist<512, true>), dim3(n_active), dim3(512), 0, st, m);
    } else {
        // (weight mode: 107 VGPRs, four waves per SIMD; with 75 VGPRs and 384 threads an event the
        // weight passes ran 5.1 vs 4.5 ms at C5 -- more waves contend for the LDS atomics)
        hipLaunchKernelGGL((k_sel_hist<BT, false>), dim3(n_active), dim3(BT), 0, st, m);
    }
    return hipGetLastError();
}

hipError_t sel_step(pcx_mat& m, int n_active, hipStream_t st) {
    if (n_active <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sel_step, dim3((n_active + BT / WAVE - 1) / (BT / WAVE)), dim3(BT), 0, st, m, n_active);
    return hipGetLastError();
}

}  // namespace pcx
