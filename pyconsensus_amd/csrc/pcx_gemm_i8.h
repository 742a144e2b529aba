// pcx_gemm_i8.h -- the int8 covariance products of M_COV_I8 on gfx950 MFMA.
// Included by pcx_matrix.hip (the product) and tools/i8bench (the kernel's own benchmark).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// MFMA k-steps (64 rows each) per LDS ring stage of k_gemm_i8
#ifndef PCX_GEMM_KS
#define PCX_GEMM_KS 2
#endif
// balanced base-254 digits per general position (pcx_internal.h, k_digits)
#ifndef PCX_NDIG
#define PCX_NDIG 6
#endif

namespace pcx {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// XCD-aware bijective remap: consecutive logical items (the tiles of one row slice)
// land on one XCD, so their shared rows are fetched into one L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int q = nwg / 8, r = nwg % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// PCX_M_COV_I8: exact integer products on int8 MFMA (v_mfma_i32_16x16x64_i8).  The A operand
// is [row / 16][position][16] int8 blocks, so one 16-byte load is one lane's MFMA fragment (16
// rows of one position).  The B operand is z in {0, 1, 2} packed 2 bits per value:
// [row / 16][position] uint32, row r of the 16 at bit 8 (r % 4) + 2 (r / 4), so dword k of the
// fragment (rows 4k .. 4k+3, one per byte) is (P >> 2k) & 0x03030303 -- a quarter of the bytes
// through L2 and LDS, unpacked by two VALU ops per dword beside the MFMAs.  64-row stages of
// both panels stream from L2 into an LDS ring (global_load_lds); 256 x 256 output tiles; each
// k-slice's int32 tile is stored to its own slab (k_cov_assemble sums the slabs in int64),
// transposed (out[q][p]) when trans is set.  Tiles run k-slice major and XCD-grouped, so the
// WGs resident at once stream the same rows through L2.
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int GT = 256;                              // output tile edge
constexpr size_t G_PANEL = (size_t)4 * GT * 16;      // one int8 operand's 64-row stage: 16 KB
// packed B rows in LDS are XOR-swizzled: position p of row group g sits at dword p ^ (16 g), so
// the row groups one ds_read_b32 reads together (lanes 16 g + c) fall in different banks (a
// plain layout, rows a multiple of 32 dwords apart, 2-way conflicts; padding would cost the
// ring's fourth stage).  The DMA lanes fetch the swizzled positions.
constexpr int G_BSWZ = 16;
constexpr size_t G_PANEL_PK = (size_t)4 * GT * 4;    // a packed one: 4 KB
constexpr int G_KS = PCX_GEMM_KS;  // MFMA k-steps (64 rows each) per ring stage and barrier
// workgroups of a launch: one per (k-slice, tile) item
__host__ __device__ inline int64_t gemm_i8_items(int tp, int tq, int lower, int kslices) {
    return (int64_t)(lower ? tp * (tp + 1) / 2 : tp * tq) * kslices;
}

struct GemmI8 {
    const int8_t* A;
    int64_t lda;  // positions per row group
    const int8_t* B;
    int64_t ldb;
    int32_t* out;  // [kslices][slab]: row p at p * ldo (trans: row q at q * ldo)
    int64_t ldo, slab;
    int np, nq, tp, tq, lower, kslices;
    int64_t rg;  // row groups, a multiple of 4
    int trans;
};

// WAVES = 16: 4 x 4 waves of 64 x 64 (four per SIMD, 16 int32 accumulators each); WAVES = 8:
// 2 x 4 waves of 128 x 64 (two per SIMD).  NBUF stages of G_KS k-steps in the ring, one barrier
// per stage, counted vmcnt.  Address arithmetic lives on the scalar unit: the DMA sources are a
// scalar base (the stage's row group, the tile's first position) plus a fixed 32-bit lane
// offset, the ring slot rotates as a scalar and the fragment offsets are loop-invariant -- with
// 64-bit per-lane address math (~3.3 VALU per MFMA; an MFMA holds its SIMD's vector issue for
// 8 of its 16 cycles) the same loop ran 3-5 % slower.  The product launches
// <8, 3> (two waves per SIMD: half the B unpacking per MFMA of <16, 3>).
template <int WAVES, int NBUF>
__global__ void __launch_bounds__(WAVES * 64, 1) k_gemm_i8(GemmI8 g) {
    static_assert(WAVES == 16 || WAVES == 8, "4 x 4 or 2 x 4 waves");
    constexpr int KS = G_KS;
    constexpr int WR = WAVES == 16 ? 4 : 2, TM = GT / WR, AF = TM / 16;
    constexpr int LPP = 16 / WAVES;  // DMA pieces per wave per operand per k-step
    constexpr size_t STAGE = KS * (G_PANEL + G_PANEL_PK);
    static_assert(NBUF >= 2 && NBUF * STAGE <= 163840, "int8 GEMM ring (160 KB of LDS)");
    constexpr int LOADS = 2 * KS * LPP;  // vector-memory ops per wave per stage (A chunks + packed B pieces)
    extern __shared__ __attribute__((aligned(16))) char glds[];
    // lower: only the tp (tp + 1) / 2 tiles on and below the diagonal are items (with the upper
    // tiles in the grid as empty workgroups, the XCDs' shares of real items differed by up to a
    // third: C5's grid block 5.3 ms at 13 k-slices)
    const int ntiles = g.lower ? g.tp * (g.tp + 1) / 2 : g.tp * g.tq;
    const int item = xcd_remap(blockIdx.x, gridDim.x);
    const int ks = item / ntiles, tl = item % ntiles;
    int ip, iq;
    if (g.lower) {  // tl = ip (ip + 1) / 2 + iq, iq <= ip
        ip = (int)((__builtin_sqrtf(8.0f * (float)tl + 1.0f) - 1.0f) * 0.5f);
        while (ip * (ip + 1) / 2 > tl) ip--;
        while ((ip + 1) * (ip + 2) / 2 <= tl) ip++;
        iq = tl - ip * (ip + 1) / 2;
    } else {
        ip = tl / g.tq;
        iq = tl % g.tq;
    }
    const int64_t nst = g.rg / (4 * KS);  // (rg is a multiple of 4 KS)
    const int64_t per = (nst + g.kslices - 1) / g.kslices;
    const int64_t s0 = ks * per < nst ? ks * per : nst;
    const int64_t s1 = s0 + per < nst ? s0 + per : nst;  // (an empty slice stores zeros)
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar
    const int wr = wv >> 2, wc = wv & 3;
    const int lc = lane & 15, lg = lane >> 4;
    // DMA: piece ch = wv + j WAVES of each 64-row k-step = (row group ch & 3, positions
    // (ch >> 2) * 64 .. + 63), for A (1 KB) and for the packed B (256 B)
    const int8_t* const abase = g.A + (int64_t)ip * GT * 16;
    const char* const bbase = reinterpret_cast<const char*>(g.B) + (int64_t)iq * GT * 4;
    const int64_t astep = 4 * g.lda * 16, bstep = 4 * g.ldb * 4;  // bytes per k-step
    uint32_t aoff[LPP], boff[LPP], adst[LPP], bdst[LPP];
#pragma unroll
    for (int j = 0; j < LPP; j++) {
        const int ch = wv + j * WAVES, mg = ch & 3, mh = ch >> 2;
        aoff[j] = (uint32_t)(((int64_t)mg * g.lda + mh * 64 + lane) * 16);
        boff[j] = (uint32_t)(((int64_t)mg * g.ldb + ((mh * 64 + lane) ^ (G_BSWZ * mg))) * 4);
        adst[j] = (uint32_t)((mg * GT + mh * 64) * 16);
        bdst[j] = (uint32_t)(KS * G_PANEL + (mg * GT + mh * 64) * 4);
    }
    auto issue = [&](int64_t st, int buf) {
        char* sb = glds + (size_t)buf * STAGE;
#pragma unroll
        for (int kk = 0; kk < KS; kk++) {
            const int64_t k = (s0 + st) * KS + kk;
#pragma unroll
            for (int j = 0; j < LPP; j++) {
                __builtin_amdgcn_global_load_lds((const void*)(abase + k * astep + aoff[j]),
                                                 (lds_ptr_t)(sb + kk * G_PANEL + adst[j]), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void*)(bbase + k * bstep + boff[j]),
                                                 (lds_ptr_t)(sb + kk * G_PANEL_PK + bdst[j]), 4, 0, 0);
            }
        }
    };
    // fragment offsets inside a stage (bytes), loop-invariant
    const uint32_t afr = (uint32_t)((lg * GT + wr * TM + lc) * 16);
    uint32_t bfr[4];
#pragma unroll
    for (int b = 0; b < 4; b++)
        bfr[b] = (uint32_t)(KS * G_PANEL + (lg * GT + wc * 64 + lc + ((b * 16) ^ (G_BSWZ * lg))) * 4);
    struct Frag {  // one k-step's fragments: AF A blocks, four packed B dwords
        v4i a[AF];
        uint32_t b[4];
    };
    auto read = [&](int buf, int kk, Frag& f) {
        const char* sb = glds + (size_t)buf * STAGE;
#pragma unroll
        for (int a = 0; a < AF; a++) f.a[a] = *reinterpret_cast<const v4i*>(sb + kk * G_PANEL + afr + a * 256);
#pragma unroll
        for (int b = 0; b < 4; b++) f.b[b] = *reinterpret_cast<const uint32_t*>(sb + kk * G_PANEL_PK + bfr[b]);
    };
    v4i acc[AF][4];
#pragma unroll
    for (int a = 0; a < AF; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = v4i{0, 0, 0, 0};
    auto mma = [&](const Frag& f) {
        constexpr uint32_t M2 = 0x03030303u;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t P = f.b[b];
            const v4i bf = v4i{(int)(P & M2), (int)((P >> 2) & M2), (int)((P >> 4) & M2), (int)((P >> 6) & M2)};
#pragma unroll
            for (int a = 0; a < AF; a++) acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[a], bf, acc[a][b], 0, 0, 0);
        }
    };
    // The fragment reads are software-pipelined across the ring's barrier (round 5; reading a
    // k-step's fragments and then running its MFMAs left every SIMD's MFMA pipe empty after each
    // barrier while all waves read LDS at once): k-step 1's fragments are read under k-step 0's
    // MFMAs, and k-step 1's MFMAs wait until after the barrier that publishes the next stage, whose
    // first fragments are then read under them.  Every wave has its fragments of stage t in registers
    // when it reaches that barrier, so stage t's slot takes stage t + NBUF right after it (all NBUF
    // slots filled up front: NBUF - 1 stages stay in flight, as before).  C5 mixed block 14.06 ->
    // 13.40 ms, grid block 4.00 -> 3.71 ms with 8 waves (tools/i8bench).
    static_assert(KS == 2, "the pipelined loop alternates two k-steps per stage");
    const int64_t n = s1 - s0;
    if (n > 0) {
#pragma unroll
        for (int k = 0; k < NBUF; k++)
            if (k < n) issue(k, k);
        if (NBUF - 1 < n)
            wait_vmcnt<LOADS * (NBUF - 1)>();
        else
            wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        Frag F, G;  // a stage's first k-step in F, its second in G
        read(0, 0, F);
        int buf = 0;
        for (int64_t t = 0; t + 1 < n; t++) {  // (the last stage peeled: no join before its mma(G))
            read(buf, 1, G);
            mma(F);
            if (t + NBUF - 1 < n)
                wait_vmcnt<LOADS * (NBUF - 2)>();  // stage t + 1 landed (this wave's pieces)
            else
                wait_vmcnt<0>();
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) as a builtin (an asm one is opaque to
                                                 // the compiler, which then waited for F's reads too
                                                 // before mma(G) below)
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (t + NBUF < n) issue(t + NBUF, buf);
            buf = buf + 1 == NBUF ? 0 : buf + 1;
            read(buf, 0, F);
            __builtin_amdgcn_sched_barrier(0);
            mma(G);
        }
        read(buf, 1, G);
        mma(F);
        mma(G);
    }
    // D layout (i32 16x16): col = lane & 15, row = 4 * (lane >> 4) + r
    const int p0 = ip * GT + wr * TM + 4 * lg, q0 = iq * GT + wc * 64 + lc;
    int32_t* out = g.out + (int64_t)ks * g.slab;
#pragma unroll
    for (int a = 0; a < AF; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int pa = p0 + a * 16, q = q0 + b * 16;
            if (g.trans) {  // out[q][p .. p + 3]: one 16-byte store per lane
                if (q < g.nq && pa + 3 < g.np && (g.ldo & 3) == 0) {
                    *(v4i*)(out + (int64_t)q * g.ldo + pa) = acc[a][b];
                } else {
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (pa + r < g.np && q < g.nq) out[(int64_t)q * g.ldo + pa + r] = acc[a][b][r];
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int p = pa + r;
                    if (p < g.np && q < g.nq && (!g.lower || q <= p)) out[(int64_t)p * g.ldo + q] = acc[a][b][r];
                }
            }
        }
}

// General x general pairs on int8 (k_gemm_i8x): both operands are PCX_NDIG balanced base-254 digit
// slices in the A layout above -- A the digits of tok w (zD), B those of w (zE), digit i of general
// position q at position i gb + q -- and the product of digit i of p with digit j of q is weighted
// 254^-(i + j + 2).  Only the digit pairs with i + j <= smax matter at fp64's level and only the
// lower event tiles (p >= q) are needed.  Items run k-slice major, then by output tile, then by
// digit pair, so the workgroups resident on one XCD at a time share their digit panels in its L2;
// each writes its whole 256 x 256 int32 tile to its own slab,
// out[ks][i][j][tile (a, b)][256][256] (row: the position of p in the tile, column: that of q).
struct GemmX {
    const int8_t* A;  // [rg][lda][16]
    const int8_t* B;  // [rg][ldb][16]
    int64_t lda, ldb;
    int32_t* out;
    int64_t rg;  // row groups, a multiple of 4 KS
    int gb;      // positions per digit slice, a multiple of 256
    int nt;      // gb / 256 event tiles per side
    int smax, kslices;
    int smin;  // the pairs smin <= i + j <= smax (0: from the first; the covariance guard's second launch
               // takes the rest, PCX_NDIG .. 2 PCX_NDIG - 2, pcx_matrix.hip k_cov_guard)
    int sym;   // A == B (one digit string, every token 2^k): on a diagonal tile (a == b) the pair (i, j)
               // with i > j is the transpose of (j, i) -- those items exit at once, the reader transposes
};
// digit j range of digit i among the pairs smin <= i + j <= smax (empty: j1 < j0)
__host__ __device__ inline int gemm_i8x_j0(int i, int smin) { return smin - i > 0 ? smin - i : 0; }
__host__ __device__ inline int gemm_i8x_j1(int i, int smax) { return smax - i < PCX_NDIG - 1 ? smax - i : PCX_NDIG - 1; }
__host__ __device__ inline int gemm_i8x_pairs(int smax, int smin = 0) {  // digit pairs (i, j), i, j < NDIG
    int n = 0;
    for (int i = 0; i < PCX_NDIG; i++) {
        const int nj = gemm_i8x_j1(i, smax) - gemm_i8x_j0(i, smin) + 1;
        n += nj > 0 ? nj : 0;
    }
    return n;
}
__host__ __device__ inline int64_t gemm_i8x_items(const GemmX& g) {
    return (int64_t)g.kslices * gemm_i8x_pairs(g.smax, g.smin) * (g.nt * (g.nt + 1) / 2);
}
// slab of (k-slice, i, j, lower tile)
__host__ __device__ inline int64_t gemm_i8x_slab(int ks, int i, int j, int tl, int nt) {
    return (((int64_t)ks * PCX_NDIG + i) * PCX_NDIG + j) * (nt * (nt + 1) / 2) + tl;
}

// 16-byte fragments of both operands straight from the LDS ring (no unpacking); the fragment reads
// are software-pipelined across the ring's barrier: a stage's last k-step keeps its MFMAs until after
// the barrier that publishes the next stage, whose first fragments are then read under them (every
// wave has its fragments of the stage in registers before it arrives, so that stage's slot is
// refilled right after the barrier: stage t + NBUF into stage t's slot).  WAVES = 8: 2 x 4 waves of
// 128 x 64; 16: 4 x 4 of 64 x 64.
template <int WAVES, int NBUF>
__global__ void __launch_bounds__(WAVES * 64, 1) k_gemm_i8x(GemmX g) {
    static_assert(WAVES == 16 || WAVES == 8, "4 x 4 or 2 x 4 waves");
    constexpr int KS = 2, WR = WAVES == 16 ? 4 : 2, TM = GT / WR, AF = TM / 16;
    constexpr int LPP = 16 / WAVES;       // DMA pieces per wave per operand per k-step
    constexpr size_t STAGE = KS * 2 * G_PANEL;
    static_assert(NBUF >= 2 && NBUF * STAGE <= 163840, "int8 GEMM ring (160 KB of LDS)");
    constexpr int LOADS = 2 * KS * LPP;  // vector-memory ops per wave per stage
    extern __shared__ __attribute__((aligned(16))) char glds[];
    const int ntri = g.nt * (g.nt + 1) / 2, npair = gemm_i8x_pairs(g.smax, g.smin);
    const int item = xcd_remap(blockIdx.x, gridDim.x);
    const int ks = item / (npair * ntri);
    // tile major: every digit pair of one output tile, then the next tile (a, b + 1) -- the items
    // resident on one XCD share both operands' digit panels (11.85 vs 12.09 ms at C5 against
    // ordering by A panel, digit i then tile a, then (j, b))
    int r = item % (npair * ntri), i = 0;
    const int tl = r / npair;
    r %= npair;
    for (;; i++) {  // digit i: the digits j0 .. j1 of the pair range
        const int nj = gemm_i8x_j1(i, g.smax) - gemm_i8x_j0(i, g.smin) + 1;
        if (r < nj) break;
        r -= nj > 0 ? nj : 0;
    }
    const int j = gemm_i8x_j0(i, g.smin) + r;
    int ta = (int)((__builtin_sqrtf(8.0f * (float)tl + 1.0f) - 1.0f) * 0.5f);  // tl = ta (ta + 1) / 2 + tb
    while (ta * (ta + 1) / 2 > tl) ta--;
    while ((ta + 1) * (ta + 2) / 2 <= tl) ta++;
    const int tb = tl - ta * (ta + 1) / 2;
    if (g.sym && ta == tb && i > j) return;  // (the workgroup as a whole, before any barrier)
    const int64_t nst = g.rg / (4 * KS);
    const int64_t per = (nst + g.kslices - 1) / g.kslices;
    const int64_t s0 = ks * per < nst ? ks * per : nst;
    const int64_t s1 = s0 + per < nst ? s0 + per : nst;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wv >> 2, wc = wv & 3;
    const int lc = lane & 15, lg = lane >> 4;
    const int8_t* const abase = g.A + ((int64_t)i * g.gb + (int64_t)ta * GT) * 16;
    const int8_t* const bbase = g.B + ((int64_t)j * g.gb + (int64_t)tb * GT) * 16;
    const int64_t astep = 4 * g.lda * 16, bstep = 4 * g.ldb * 16;  // bytes per k-step
    uint32_t aoff[LPP], boff[LPP], dst[LPP];
#pragma unroll
    for (int u = 0; u < LPP; u++) {
        const int ch = wv + u * WAVES, mg = ch & 3, mh = ch >> 2;
        aoff[u] = (uint32_t)(((int64_t)mg * g.lda + mh * 64 + lane) * 16);
        boff[u] = (uint32_t)(((int64_t)mg * g.ldb + mh * 64 + lane) * 16);
        dst[u] = (uint32_t)((mg * GT + mh * 64) * 16);
    }
    auto issue = [&](int64_t st, int buf) {
        char* sb = glds + (size_t)buf * STAGE;
#pragma unroll
        for (int kk = 0; kk < KS; kk++) {
            const int64_t k = (s0 + st) * KS + kk;
#pragma unroll
            for (int u = 0; u < LPP; u++) {
                __builtin_amdgcn_global_load_lds((const void*)(abase + k * astep + aoff[u]),
                                                 (lds_ptr_t)(sb + kk * G_PANEL + dst[u]), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void*)(bbase + k * bstep + boff[u]),
                                                 (lds_ptr_t)(sb + (KS + kk) * G_PANEL + dst[u]), 16, 0, 0);
            }
        }
    };
    const uint32_t afr = (uint32_t)((lg * GT + wr * TM + lc) * 16);
    const uint32_t bfr = (uint32_t)(KS * G_PANEL + (lg * GT + wc * 64 + lc) * 16);
    struct Frag {
        v4i a[AF], b[4];
    };
    auto read = [&](int buf, int kk, Frag& f) {
        const char* sb = glds + (size_t)buf * STAGE + kk * G_PANEL;
#pragma unroll
        for (int a = 0; a < AF; a++) f.a[a] = *reinterpret_cast<const v4i*>(sb + afr + a * 256);
#pragma unroll
        for (int b = 0; b < 4; b++) f.b[b] = *reinterpret_cast<const v4i*>(sb + bfr + b * 256);
    };
    v4i acc[AF][4];
#pragma unroll
    for (int a = 0; a < AF; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = v4i{0, 0, 0, 0};
    auto mma = [&](const Frag& f) {
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int a = 0; a < AF; a++) acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f.a[a], f.b[b], acc[a][b], 0, 0, 0);
    };
    const int64_t n = s1 - s0;
    if (n > 0) {
#pragma unroll
        for (int k = 0; k < NBUF; k++)
            if (k < n) issue(k, k);
        if (NBUF - 1 < n)
            wait_vmcnt<LOADS * (NBUF - 1)>();
        else
            wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // stage t + 1 published: every wave's pieces landed and every wave's fragments of stage t are in
        // registers (the lgkmcnt wait is a builtin, so the compiler's own wait before the next MFMAs
        // knows they have landed); stage t's slot then takes stage t + NBUF
        auto publish = [&](int64_t t, int slot) {
            if (t + NBUF - 1 < n)
                wait_vmcnt<LOADS * (NBUF - 2)>();  // stage t + 1 landed (this wave's pieces)
            else
                wait_vmcnt<0>();
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (t + NBUF < n) issue(t + NBUF, slot);
        };
        Frag F, G;
        read(0, 0, F);
        int buf = 0;
        // a stage's first k-step in F, its second in G.  (One k-step per stage in a four-stage ring,
        // alternating stages between F and G: 11.84 vs 12.02 ms at C5, not kept.)
        for (int64_t t = 0; t + 1 < n; t++) {  // (the last stage peeled: no join before its mma(G))
            read(buf, 1, G);
            mma(F);
            publish(t, buf);
            buf = buf + 1 == NBUF ? 0 : buf + 1;
            read(buf, 0, F);
            __builtin_amdgcn_sched_barrier(0);
            mma(G);
        }
        read(buf, 1, G);
        mma(F);
        mma(G);
    }
    // D layout (i32 16x16): col = lane & 15, row = 4 * (lane >> 4) + r
    int32_t* out = g.out + gemm_i8x_slab(ks, i, j, tl, g.nt) * (GT * GT);
#pragma unroll
    for (int a = 0; a < AF; a++)
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int e = 0; e < 4; e++)
                out[(wr * TM + a * 16 + 4 * lg + e) * GT + wc * 64 + b * 16 + lc] = acc[a][b][e];
}
constexpr int GEMM_I8X_WAVES = 8, GEMM_I8X_NBUF = 2;
constexpr size_t GEMM_I8X_LDS = (size_t)GEMM_I8X_NBUF * 2 * 2 * G_PANEL;  // 128 KB

// the product's configuration (pcx_matrix.hip M_COV_I8)
constexpr int GEMM_I8_WAVES = 8, GEMM_I8_NBUF = 3;
constexpr size_t GEMM_I8_LDS = (size_t)GEMM_I8_NBUF * G_KS * (G_PANEL + G_PANEL_PK);  // 120 KB
static_assert(GEMM_I8_LDS <= 163840, "int8 GEMM ring (160 KB of LDS)");

}  // namespace pcx
