// pcx_gemm_i8.h -- the int8 covariance products of M_COV_I8 on gfx950 MFMA.
// Included by pcx_matrix.hip (the product) and tools/i8bench (the kernel's own benchmark).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// MFMA k-steps (64 rows each) per LDS ring stage of k_gemm_i8
#ifndef PCX_GEMM_KS
#define PCX_GEMM_KS 2
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
// rows of one position).  The B operand is either the same (BPACK = false) or z in {0, 1, 2}
// packed 2 bits per value (BPACK): [row / 16][position] uint32, row r of the 16 at bit
// 8 (r % 4) + 2 (r / 4), so dword k of the fragment (rows 4k .. 4k+3, one per byte) is
// (P >> 2k) & 0x03030303 -- a quarter of the bytes through L2 and LDS, unpacked by two VALU
// ops per dword beside the MFMAs.  The kernel streams 64-row stages of both panels from L2
// into LDS (global_load_lds) and is bound by that stream: at 256 x 256 tiles (the largest the
// register file holds) a 16 KB + 16 KB stage feeds 1,024 MFMA cycles per SIMD, more than L2
// delivers per CU; a packed B panel cuts the stage to 20 KB.  256 x 256 output tiles, 16 waves
// of 64 x 64 (16 int32 accumulators each, four waves per SIMD); a G_NBUF-stage ring (one
// barrier per stage, counted vmcnt); each k-slice's int32 tile is stored to its own slab
// (k_cov_reduce sums the slabs in int64), transposed (out[q][p]) when trans is set.  Tiles run
// k-slice major and XCD-grouped, so the WGs resident at once stream the same rows through L2.
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
template <bool BPACK>
struct GRing {
    static constexpr int KS = G_KS;
    static constexpr size_t BPANEL = BPACK ? G_PANEL_PK : G_PANEL;
    static constexpr int NBUF = KS == 1 ? (BPACK ? 6 : 4) : (BPACK ? 3 : 2);  // LDS ring depth
    static constexpr size_t STAGE = KS * (G_PANEL + BPANEL);
    static constexpr size_t BYTES = NBUF * STAGE;  // <= 128 KB
};
static_assert(GRing<true>::BYTES <= 163840, "int8 GEMM ring (160 KB of LDS)");  // (only the packed-B form is launched)

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

// WAVES = 16: 4 x 4 waves of 64 x 64 (four waves per SIMD); WAVES = 8: 2 x 4 waves of 128 x 64
// (two per SIMD, 8 A + 4 B fragment reads per 32 MFMAs instead of 4 + 4 per 16: a quarter less
// LDS read traffic per MFMA).  Same items, slabs and integer results.
template <int WAVES, bool BPACK>
__global__ void __launch_bounds__(WAVES * 64, 1) k_gemm_i8(GemmI8 g) {
    static_assert(!BPACK || WAVES == 16, "packed B: one dword load per wave per k-step");
    using RG = GRing<BPACK>;
    constexpr int KS = RG::KS;
    constexpr int WR = WAVES == 16 ? 4 : 2;  // wave rows (p); 4 wave columns (q)
    constexpr int TM = GT / WR, AF = TM / 16;
    constexpr int LPP = 16 / WAVES;  // 1 KB loads per wave per int8 panel per k-step (16 KB panels)
    constexpr int LOADS = KS * (LPP + (BPACK ? 1 : LPP));  // vector-memory ops per wave per stage
    extern __shared__ __attribute__((aligned(16))) char glds[];
    const int ntiles = g.tp * g.tq;
    const int item = xcd_remap(blockIdx.x, gridDim.x);
    const int ks = item / ntiles, t = item % ntiles;
    const int ip = t / g.tq, iq = t % g.tq;
    if (g.lower && iq > ip) return;  // above the diagonal (square tiles)
    const int64_t nst = g.rg / (4 * KS);  // (rg is a multiple of 4 KS)
    const int64_t per = (nst + g.kslices - 1) / g.kslices;
    const int64_t s0 = ks * per < nst ? ks * per : nst;
    const int64_t s1 = s0 + per < nst ? s0 + per : nst;  // (an empty slice stores zeros)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wr = wv >> 2, wc = wv & 3;
    const int lc = lane & 15, lg = lane >> 4;
    auto issue = [&](int64_t st, int buf) {
        char* sbase = glds + (size_t)buf * RG::STAGE;
#pragma unroll
        for (int kk = 0; kk < KS; kk++) {
#pragma unroll
            for (int j = 0; j < LPP; j++) {  // chunk ch = (row group mg, quarter mh) of the int8 panels
                const int ch = wv + j * WAVES, mg = ch & 3, mh = ch >> 2;
                char* base = sbase + kk * G_PANEL + ((size_t)mg * GT + mh * 64) * 16;
                const int64_t grp = (st * KS + kk) * 4 + mg;
                const int8_t* Ab = g.A + ((int64_t)ip * GT + mh * 64 + lane) * 16;
                __builtin_amdgcn_global_load_lds((const void*)(Ab + grp * g.lda * 16), (lds_ptr_t)base, 16, 0, 0);
                if constexpr (!BPACK) {
                    const int8_t* Bb = g.B + ((int64_t)iq * GT + mh * 64 + lane) * 16;
                    __builtin_amdgcn_global_load_lds((const void*)(Bb + grp * g.ldb * 16),
                                                     (lds_ptr_t)(base - kk * G_PANEL + KS * G_PANEL + kk * RG::BPANEL),
                                                     16, 0, 0);
                }
            }
            if constexpr (BPACK) {  // packed panel [mg][256 positions] uint32: 256 B per wave
                const int mg = wv & 3, mh = wv >> 2;
                const uint32_t* Bb = reinterpret_cast<const uint32_t*>(g.B) + ((st * KS + kk) * 4 + mg) * g.ldb +
                                     (int64_t)iq * GT + ((mh * 64 + lane) ^ (G_BSWZ * mg));
                __builtin_amdgcn_global_load_lds(
                    (const void*)Bb, (lds_ptr_t)(sbase + KS * G_PANEL + kk * RG::BPANEL + ((size_t)mg * GT + mh * 64) * 4),
                    4, 0, 0);
            }
        }
    };
    v4i acc[AF][4];
#pragma unroll
    for (int a = 0; a < AF; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = v4i{0, 0, 0, 0};
    const int64_t n = s1 - s0;
#pragma unroll
    for (int k = 0; k < RG::NBUF - 1; k++)
        if (k < n) issue(s0 + k, k);
    for (int64_t t = 0; t < n; t++) {
        const int buf = (int)(t % RG::NBUF);
        if (t + RG::NBUF - 2 < n)
            wait_vmcnt<LOADS * (RG::NBUF - 2)>();  // stage t landed, t+1 .. t+NBUF-2 may be in flight
        else
            wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t + RG::NBUF - 1 < n) issue(s0 + t + RG::NBUF - 1, (int)((t + RG::NBUF - 1) % RG::NBUF));
        const char* sb = glds + (size_t)buf * RG::STAGE;
#pragma unroll
        for (int kk = 0; kk < KS; kk++) {
            const v4i* As = (const v4i*)(sb + kk * G_PANEL) + lg * GT + wr * TM + lc;
            v4i af[AF], bf[4];
#pragma unroll
            for (int a = 0; a < AF; a++) af[a] = As[a * 16];
            if constexpr (BPACK) {
                const uint32_t* Bs = (const uint32_t*)(sb + KS * G_PANEL + kk * RG::BPANEL) + lg * GT + wc * 64 + lc;
                constexpr uint32_t M2 = 0x03030303u;
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const uint32_t P = Bs[(b * 16) ^ (G_BSWZ * lg)];
                    bf[b] = v4i{(int)(P & M2), (int)((P >> 2) & M2), (int)((P >> 4) & M2), (int)((P >> 6) & M2)};
                }
            } else {
                const v4i* Bs = (const v4i*)(sb + KS * G_PANEL + kk * RG::BPANEL) + lg * GT + wc * 64 + lc;
#pragma unroll
                for (int b = 0; b < 4; b++) bf[b] = Bs[b * 16];
            }
#pragma unroll
            for (int a = 0; a < AF; a++)
#pragma unroll
                for (int b = 0; b < 4; b++)
                    acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        asm volatile("" ::: "memory");
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

// k_gemm_i8u: the same products (packed B) with B unpacked ONCE per 64-row stage instead of
// beside every MFMA.  Each thread loads packed dwords (16 rows of one position) two stages
// ahead into registers, unpacks them (7 VALU per dword) and stores the 16-byte fragments into an
// LDS panel laid out like A's, [row group][256 positions][16 B]; the waves then read their B
// fragments with one ds_read_b128 each, like A.  (k_gemm_i8 unpacks each B dword in every one
// of the WR waves that share it, beside the MFMAs: ~1.75 VALU per MFMA of the ~3.6 that, with
// the loop's 64-bit address arithmetic, held the MFMA pipe near 60 % -- an MFMA holds its
// SIMD's vector issue for 8 of its 16 cycles.)  A streams by LDS-DMA into an NA-stage ring; the
// DMA and the B loads address through a scalar base plus a fixed 32-bit lane offset.  One
// barrier per stage: after it every wave has finished the previous stage's MFMAs (so the
// unpacked panel they read is free to refill) and this stage's panel, stored before the
// barrier, is visible.  WAVES = 16: 4 x 4 waves of 64 x 64; 8: 2 x 4 waves of 128 x 64.
template <int NA>
struct GRingU {
    static constexpr size_t BYTES = (size_t)(NA + 2) * G_PANEL;  // A ring + two unpacked B panels
};

template <int WAVES, int NA>
__global__ void __launch_bounds__(WAVES * 64, 1) k_gemm_i8u(GemmI8 g) {
    static_assert(WAVES == 16 || WAVES == 8, "4 x 4 or 2 x 4 waves");
    static_assert(NA >= 2 && GRingU<NA>::BYTES <= 163840, "A ring depth");
    constexpr int NT = WAVES * 64;
    constexpr int WR = WAVES == 16 ? 4 : 2;  // wave rows (p); 4 wave columns (q)
    constexpr int TM = GT / WR, AF = TM / 16;
    constexpr int LPP = 16 / WAVES;        // 1 KB A chunks per wave per stage
    constexpr int BPT = 4 * GT / NT;       // packed B dwords per thread per stage
    extern __shared__ __attribute__((aligned(16))) char glds[];
    char* const aring = glds;
    char* const ubuf = glds + (size_t)NA * G_PANEL;
    const int ntiles = g.tp * g.tq;
    const int item = xcd_remap(blockIdx.x, gridDim.x);
    const int ks = item / ntiles, tl = item % ntiles;
    const int ip = tl / g.tq, iq = tl % g.tq;
    if (g.lower && iq > ip) return;  // above the diagonal (square tiles)
    const int64_t nst = g.rg / 4;    // 64-row stages (rg is a multiple of 4)
    const int64_t per = (nst + g.kslices - 1) / g.kslices;
    const int64_t s0 = ks * per < nst ? ks * per : nst;
    const int64_t s1 = s0 + per < nst ? s0 + per : nst;  // (an empty slice stores zeros)
    const int64_t n = s1 - s0;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 2, wc = wv & 3;
    const int lc = lane & 15, lg = lane >> 4;
    // A: chunk ch = (row group mg = ch & 3, quarter mh = ch >> 2) of the stage's [4][256][16] panel
    const int8_t* const abase = g.A + ((int64_t)ip * GT) * 16;  // + stage * 4 lda 16 (scalar)
    uint32_t aoff[LPP], adst[LPP];
#pragma unroll
    for (int j = 0; j < LPP; j++) {
        const int ch = wv + j * WAVES, mg = ch & 3, mh = ch >> 2;
        aoff[j] = (uint32_t)(((int64_t)mg * g.lda + mh * 64 + lane) * 16);
        adst[j] = (uint32_t)(((size_t)mg * GT + mh * 64) * 16);
    }
    // B: packed dword u = tid + k NT of the stage = (row group u >> 8, position u & 255)
    const uint32_t* const bbase = reinterpret_cast<const uint32_t*>(g.B) + (int64_t)iq * GT;  // + stage * 4 ldb
    uint32_t boff[BPT];
#pragma unroll
    for (int k = 0; k < BPT; k++) {
        const int u = tid + k * NT;
        boff[k] = (uint32_t)((u >> 8) * g.ldb + (u & 255));
    }
    auto issue_a = [&](int64_t st) {
        const int8_t* src = abase + (s0 + st) * 4 * g.lda * 16;
        char* dst = aring + (size_t)(st % NA) * G_PANEL;
#pragma unroll
        for (int j = 0; j < LPP; j++)
            __builtin_amdgcn_global_load_lds((const void*)(src + aoff[j]), (lds_ptr_t)(dst + adst[j]), 16, 0, 0);
    };
    uint32_t bq[2][BPT];  // packed B of the two stages in flight: stage st in slot st & 1 (static below)
    auto issue_b = [&](int64_t st, uint32_t(&q)[BPT]) {
        const uint32_t* src = bbase + (s0 + st) * 4 * g.ldb;
#pragma unroll
        for (int k = 0; k < BPT; k++) q[k] = src[boff[k]];
    };
    auto unpack_b = [&](int64_t st, const uint32_t(&q)[BPT]) {  // -> unpacked panel st & 1
        v4i* dst = reinterpret_cast<v4i*>(ubuf + (size_t)(st & 1) * G_PANEL);
        constexpr uint32_t M2 = 0x03030303u;
#pragma unroll
        for (int k = 0; k < BPT; k++) {
            const uint32_t P = q[k];
            dst[tid + k * NT] = v4i{(int)(P & M2), (int)((P >> 2) & M2), (int)((P >> 4) & M2), (int)((P >> 6) & M2)};
        }
    };
    v4i acc[AF][4];
#pragma unroll
    for (int a = 0; a < AF; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = v4i{0, 0, 0, 0};
    // prologue: A stages 0 .. NA-2 in flight; B stage 0 unpacked, stages 1 and 2 in flight
    if (n > 0) {
#pragma unroll
        for (int k = 0; k < NA - 1; k++)
            if (k < n) issue_a(k);
        issue_b(0, bq[0]);
        wait_vmcnt<0>();
        unpack_b(0, bq[0]);
        if (1 < n) issue_b(1, bq[1]);
        if (2 < n) issue_b(2, bq[0]);
    }
    // per stage t the loads issue as A(t + NA - 1) (LPP ops), then B(t + 3) (BPT ops); stage t
    // needs A(t) and B(t + 1) landed.  In steady state the loads issued after them number at
    // least min(BPT + (NA - 2) OPS, OPS), and loads return in order
    constexpr int OPS = LPP + BPT;
    constexpr int WA = BPT + (NA - 2) * OPS;
    constexpr int WSTEADY = WA < OPS ? WA : OPS;
    constexpr int TLO = NA - 1 > 2 ? NA - 1 : 2, THI = NA - 2 > 2 ? NA - 2 : 2;
    auto body = [&](int64_t t, uint32_t(&q)[BPT]) {  // q: the slot of stage t + 1 (then of t + 3)
        if (t >= TLO && t + THI < n)
            wait_vmcnt<WSTEADY>();
        else
            wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t + NA - 1 < n) issue_a(t + NA - 1);
        if (t + 1 < n) unpack_b(t + 1, q);
        if (t + 3 < n) issue_b(t + 3, q);
        const v4i* As = reinterpret_cast<const v4i*>(aring + (size_t)(t % NA) * G_PANEL) + lg * GT + wr * TM + lc;
        const v4i* Us = reinterpret_cast<const v4i*>(ubuf + (size_t)(t & 1) * G_PANEL) + lg * GT + wc * 64 + lc;
        v4i af[AF], bf[4];
#pragma unroll
        for (int b = 0; b < 4; b++) bf[b] = Us[b * 16];
#pragma unroll
        for (int a = 0; a < AF; a++) af[a] = As[a * 16];
#pragma unroll
        for (int a = 0; a < AF; a++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[a], bf[b], acc[a][b], 0, 0, 0);
        asm volatile("" ::: "memory");
    };
    int64_t t = 0;
    for (; t + 1 < n; t += 2) {
        body(t, bq[1]);      // stage t + 1 sits in slot 1 (t even)
        body(t + 1, bq[0]);  // stage t + 2 in slot 0
    }
    if (t < n) body(t, bq[1]);
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
}  // namespace pcx
