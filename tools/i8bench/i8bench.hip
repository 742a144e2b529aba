// i8bench.hip -- standalone benchmark of the M_COV_I8 int8 products (pyconsensus_amd/csrc/pcx_gemm_i8.h)
// at the C5 shapes (1M rows: 62,504 groups of 16), every configuration checked against the
// product's (k_gemm_i8<GEMM_I8_WAVES, GEMM_I8_NBUF>) as the int64 sum of its k-slice slabs, and all of them
// against a CPU reference on a small case.
//   mixed: A = PCX_NDIG int8 digits x 1,024 general positions, B = z of 3,072 grid events
//          (packed 2 bits), stored transposed;
//   grid:  A = tok z (int8, 3,072 positions), B = z packed, lower tiles;
//   gg (shape argument "gg"): the general x general digit pairs (k_gemm_i8x), both operands digits.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/i8bench/i8bench.hip -o tools/i8bench/i8bench
// usage: i8bench [reps=5] [rows=1000064] [variant substring] [shape substring]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../pyconsensus_amd/csrc/pcx_gemm_i8.h"

#ifndef PCX_NDIG
#define PCX_NDIG 6  // (pcx_internal.h)
#endif

using namespace pcx;

static int64_t zd_ld(int64_t gb) { return ((int64_t)PCX_NDIG * gb + 255) / 256 * 256 + 256; }  // (pcx_internal.h)

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ void k_fill_a(int8_t* A, int64_t n, int lim, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        A[i] = (int8_t)((int)(mix(seed + i) % (uint64_t)(2 * lim + 1)) - lim);
}

__global__ void k_fill_b(uint32_t* B, int64_t n, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t r = mix(seed + i);
        uint32_t P = 0;
        for (int f = 0; f < 16; f++) {
            P |= (uint32_t)(r % 3) << (2 * f);
            r /= 3;
        }
        B[i] = P;
    }
}

// sum of the k-slice slabs (int64), n entries each
__global__ void k_slabsum(const int32_t* P, int ks, int64_t slab, int64_t n, long long* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        long long s = 0;
        for (int k = 0; k < ks; k++) s += P[(int64_t)k * slab + i];
        out[i] = s;
    }
}

__global__ void k_cmp(const long long* a, const long long* b, int64_t n, unsigned long long* bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (a[i] != b[i]) atomicAdd(bad, 1ull);
}

struct Shape {
    const char* name;
    int64_t lda, ldb;
    int np, nq, lower, trans;
};

static int ks_for(int64_t tiles, int64_t nst, int ncu) {  // the runner's choice (pcx_runner.cpp)
    int64_t best = 1;
    double best_cost = 1e300;
    for (int64_t k = 1; k <= std::min<int64_t>(32, nst); k++) {
        const double cost = (double)((tiles * k + ncu - 1) / ncu) / (double)k;
        if (cost < best_cost * (1.0 - 1e-9)) {
            best_cost = cost;
            best = k;
        }
    }
    return (int)best;
}

typedef void (*kfun)(GemmI8);
struct Variant {
    const char* name;
    kfun f;
    int threads;
    size_t lds;
};

// ---- general x general digit pairs (k_gemm_i8x): A = digits of tok w, B = digits of w, both [rg][ld][16]
static int run_gg(int reps, int64_t rows, const std::vector<int>& ks_list) {
    constexpr int ND = PCX_NDIG;
    auto make = [](int smax, GemmX& g) { g.smax = smax; };
    CK(hipFuncSetAttribute((const void*)k_gemm_i8x<8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GEMM_I8X_LDS));
    CK(hipFuncSetAttribute((const void*)k_gemm_i8x<16, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GEMM_I8X_LDS));
    {  // small check against the CPU: gb 512 (two event tiles), 32 row groups, 3 k-slices
        const int64_t srg = 32, gb = 512, ld = zd_ld(gb);
        std::vector<int8_t> hA(srg * ld * 16), hB(srg * ld * 16);
        for (size_t i = 0; i < hA.size(); i++) {
            hA[i] = (int8_t)((int)((i * 2654435761u) % 255) - 127);
            hB[i] = (int8_t)((int)((i * 40503u + 7u) % 255) - 127);
        }
        GemmX g{};
        make(ND, g);
        g.lda = g.ldb = ld;
        g.rg = srg;
        g.gb = (int)gb;
        g.nt = (int)(gb / GT);
        g.kslices = 3;
        const int ntri = g.nt * (g.nt + 1) / 2;
        const size_t outn = (size_t)g.kslices * ND * ND * ntri * GT * GT;
        int8_t *dA, *dB;
        int32_t* dP;
        CK(hipMalloc(&dA, hA.size()));
        CK(hipMalloc(&dB, hB.size()));
        CK(hipMalloc(&dP, outn * 4));
        CK(hipMemcpy(dA, hA.data(), hA.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dB, hB.data(), hB.size(), hipMemcpyHostToDevice));
        g.A = dA;
        g.B = dB;
        g.out = dP;
        for (int wv : {8, 16}) {
            CK(hipMemset(dP, 0, outn * 4));
            if (wv == 8)
                hipLaunchKernelGGL((k_gemm_i8x<8, 2>), dim3((unsigned)gemm_i8x_items(g)), dim3(512), GEMM_I8X_LDS, 0, g);
            else
                hipLaunchKernelGGL((k_gemm_i8x<16, 2>), dim3((unsigned)gemm_i8x_items(g)), dim3(1024), GEMM_I8X_LDS, 0, g);
            CK(hipGetLastError());
            std::vector<int32_t> got(outn);
            CK(hipMemcpy(got.data(), dP, outn * 4, hipMemcpyDeviceToHost));
            size_t bad = 0, n = 0;
            const int64_t spg = 8;  // row groups per stage (two k-steps)
            const int64_t nst = srg / spg, per = (nst + g.kslices - 1) / g.kslices;
            for (int ks = 0; ks < g.kslices; ks++)
                for (int pr = 0; pr < ND * ND; pr++)
                    for (int ta = 0; ta < g.nt; ta++)
                        for (int tb = 0; tb <= ta; tb++) {
                            const int tl = ta * (ta + 1) / 2 + tb, pi = pr / ND, pj = pr % ND;
                            if (pi + pj > g.smax) continue;
                            const int64_t g0 = std::min(nst, ks * per) * spg, g1 = std::min(nst, ks * per + per) * spg;
                            for (int r = 0; r < GT; r += 7)
                                for (int c = 0; c < GT; c += 5) {
                                    long long ref = 0;
                                    const int64_t pa = pi * gb + ta * GT + r, pb = pj * gb + tb * GT + c;
                                    for (int64_t grp = g0; grp < g1; grp++)
                                        for (int k = 0; k < 16; k++)
                                            ref += (long long)hA[(grp * ld + pa) * 16 + k] * hB[(grp * ld + pb) * 16 + k];
                                    const size_t o = (size_t)gemm_i8x_slab(ks, pi, pj, tl, g.nt) * GT * GT + (size_t)r * GT + c;
                                    bad += got[o] != ref;
                                    n++;
                                }
                        }
            printf("small check k_gemm_i8x<%d,2>  %s (%zu of %zu differ)\n", wv, bad ? "FAIL" : "ok", bad, n);
            if (bad) return 2;
        }
        CK(hipFree(dA));
        CK(hipFree(dB));
        CK(hipFree(dP));
    }
    const int64_t rg = rows / 16, gb = 1024, ld = zd_ld(gb);
    int8_t *dA, *dB;
    CK(hipMalloc(&dA, (size_t)rg * ld * 16));
    CK(hipMalloc(&dB, (size_t)rg * ld * 16));
    hipLaunchKernelGGL(k_fill_a, dim3(4096), dim3(256), 0, 0, dA, rg * ld * 16, 127, 21ull);
    hipLaunchKernelGGL(k_fill_a, dim3(4096), dim3(256), 0, 0, dB, rg * ld * 16, 127, 23ull);
    std::vector<int> kl = ks_list.empty() ? std::vector<int>{8, 12, 16} : ks_list;
    for (int smax : {ND - 1})
        for (int wv : {8})  // (16 waves spill: 32 VGPRs)
            for (int ks : kl) {
                GemmX g{};
                make(smax, g);
                g.A = dA;
                g.B = dB;
                g.lda = g.ldb = ld;
                g.rg = rg;
                g.gb = (int)gb;
                g.nt = (int)(gb / GT);
                g.kslices = ks;
                const size_t outn = (size_t)g.kslices * ND * ND * (g.nt * (g.nt + 1) / 2) * GT * GT;
                CK(hipMalloc(&g.out, outn * 4));
                auto launch = [&] {
                    if (wv == 8)
                        hipLaunchKernelGGL((k_gemm_i8x<8, 2>), dim3((unsigned)gemm_i8x_items(g)), dim3(512), GEMM_I8X_LDS, 0, g);
                    else
                        hipLaunchKernelGGL((k_gemm_i8x<16, 2>), dim3((unsigned)gemm_i8x_items(g)), dim3(1024), GEMM_I8X_LDS, 0, g);
                };
                launch();
                CK(hipGetLastError());
                CK(hipDeviceSynchronize());
                hipEvent_t e0, e1;
                CK(hipEventCreate(&e0));
                CK(hipEventCreate(&e1));
                std::vector<float> ms;
                for (int r = 0; r < reps; r++) {
                    CK(hipEventRecord(e0, 0));
                    launch();
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float t = 0;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    ms.push_back(t);
                }
                std::sort(ms.begin(), ms.end());
                const double ops = 2.0 * (double)rg * 16 * (double)gemm_i8x_pairs(smax) * (g.nt * (g.nt + 1) / 2) * GT * GT;
                printf("gg     k_gemm_i8x<%d,2> pairs %d ks %2d  %8.3f ms (min %8.3f)  %7.1f TOP/s\n", wv, gemm_i8x_pairs(smax), ks,
                       ms[ms.size() / 2], ms[0], ops / (ms[ms.size() / 2] * 1e-3) / 1e12);
                fflush(stdout);
                CK(hipFree(g.out));
            }
    CK(hipFree(dA));
    CK(hipFree(dB));
    return 0;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const int64_t rows = argc > 2 ? atoll(argv[2]) : 1000064;
    const char* vsel = argc > 3 ? argv[3] : "";
    const char* ssel = argc > 4 ? argv[4] : "";
    // optional: comma-separated k-slice counts to sweep (product configuration only)
    std::vector<int> ks_list;
    if (argc > 5)
        for (const char* p = argv[5]; *p;) {
            ks_list.push_back(atoi(p));
            while (*p && *p != ',') p++;
            if (*p == ',') p++;
        }
    if (!strcmp(ssel, "gg")) return run_gg(reps, rows, ks_list);
    const int64_t rg = rows / 16;
    int ncu = 256;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<Variant> vs = {
        {"k_gemm_i8<8,3> (product)", k_gemm_i8<GEMM_I8_WAVES, GEMM_I8_NBUF>, GEMM_I8_WAVES * 64, GEMM_I8_LDS},
        {"k_gemm_i8<16,3>", k_gemm_i8<16, 3>, 1024, 3 * PCX_GEMM_KS * (G_PANEL + G_PANEL_PK)},
        {"k_gemm_i8<8,4>", k_gemm_i8<8, 4>, 512, 4 * PCX_GEMM_KS * (G_PANEL + G_PANEL_PK)},
    };
    for (auto& v : vs) CK(hipFuncSetAttribute((const void*)v.f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.lds));

    // ---- small-case CPU check of the product kernel and the variants
    {
        const int64_t srg = 16, lda = 512, ldb = 512;
        const int np = 300, nq = 260;
        std::vector<int8_t> hA(srg * lda * 16);
        std::vector<uint32_t> hB(srg * ldb);
        for (size_t i = 0; i < hA.size(); i++) hA[i] = (int8_t)((int)((i * 2654435761u) % 255) - 127);
        for (size_t i = 0; i < hB.size(); i++) {
            uint32_t P = 0, r = (uint32_t)(i * 40503u + 17u);
            for (int f = 0; f < 16; f++) {
                P |= (r % 3) << (2 * f);
                r = r / 3 + (uint32_t)i * 7u + (uint32_t)f;
            }
            hB[i] = P;
        }
        std::vector<long long> ref((size_t)nq * np, 0);
        for (int64_t g = 0; g < srg; g++)
            for (int r = 0; r < 16; r++)
                for (int q = 0; q < nq; q++) {
                    const int z = (hB[g * ldb + q] >> (8 * (r & 3) + 2 * (r >> 2))) & 3;
                    if (!z) continue;
                    for (int p = 0; p < np; p++) ref[(size_t)q * np + p] += (long long)z * hA[(g * lda + p) * 16 + r];
                }
        int8_t* dA;
        uint32_t* dB;
        int32_t* dP;
        long long* dS;
        CK(hipMalloc(&dA, hA.size() + 4096 * 16));
        CK(hipMalloc(&dB, hB.size() * 4 + 4096));
        CK(hipMalloc(&dP, (size_t)4 * nq * np * 4));
        CK(hipMalloc(&dS, (size_t)nq * np * 8));
        CK(hipMemcpy(dA, hA.data(), hA.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dB, hB.data(), hB.size() * 4, hipMemcpyHostToDevice));
        for (auto& v : vs) {
            GemmI8 g{dA, lda, (const int8_t*)dB, ldb, dP, np, (int64_t)nq * np, np, nq, 0, 0, 0, 2, srg, 1};
            g.tp = (np + GT - 1) / GT;
            g.tq = (nq + GT - 1) / GT;
            CK(hipMemset(dP, 0, (size_t)4 * nq * np * 4));
            hipLaunchKernelGGL(v.f, dim3((unsigned)gemm_i8_items(g.tp, g.tq, g.lower, g.kslices)), dim3(v.threads), v.lds, 0, g);
            CK(hipGetLastError());
            hipLaunchKernelGGL(k_slabsum, dim3(256), dim3(256), 0, 0, dP, g.kslices, g.slab, (int64_t)nq * np, dS);
            std::vector<long long> got((size_t)nq * np);
            CK(hipMemcpy(got.data(), dS, got.size() * 8, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < got.size(); i++) bad += got[i] != ref[i];
            printf("small check %-24s %s (%zu of %zu differ)\n", v.name, bad ? "FAIL" : "ok", bad, got.size());
            if (bad) return 2;
        }
        CK(hipFree(dA));
        CK(hipFree(dB));
        CK(hipFree(dP));
        CK(hipFree(dS));
    }

    const Shape shapes[] = {
        {"mixed", PCX_NDIG * 1024, 3072, PCX_NDIG * 1024, 3072, 0, 1},
        {"grid", 3072, 3072, 3072, 3072, 1, 0},
    };
    for (const Shape& sh : shapes) {
        if (!strstr(sh.name, ssel)) continue;
        int8_t* dA;
        uint32_t* dB;
        CK(hipMalloc(&dA, (size_t)rg * sh.lda * 16));
        CK(hipMalloc(&dB, (size_t)rg * sh.ldb * 4));
        hipLaunchKernelGGL(k_fill_a, dim3(4096), dim3(256), 0, 0, dA, rg * sh.lda * 16, sh.trans ? 127 : 63, 11ull);
        hipLaunchKernelGGL(k_fill_b, dim3(4096), dim3(256), 0, 0, dB, rg * sh.ldb, 977ull);
        const int tp = (sh.np + GT - 1) / GT, tq = (sh.nq + GT - 1) / GT;
        const int64_t tiles = sh.lower ? (int64_t)tp * (tp + 1) / 2 : (int64_t)tp * tq;
        const int64_t outn = sh.trans ? (int64_t)sh.nq * sh.np : (int64_t)sh.np * sh.nq;
        long long *dRef, *dSum;
        unsigned long long* dBad;
        CK(hipMalloc(&dRef, outn * 8));
        CK(hipMalloc(&dSum, outn * 8));
        CK(hipMalloc(&dBad, 8));
        const double ops = 2.0 * (double)rg * 16 * sh.np * (double)sh.nq * (sh.lower ? 0.5 : 1.0);
        const size_t nrun = ks_list.empty() ? vs.size() : 1 + ks_list.size();
        for (size_t ri = 0; ri < nrun; ri++) {
            const size_t vi = ks_list.empty() ? ri : 0;
            const Variant& v = vs[vi];
            if (ri > 0 && ks_list.empty() && !strstr(v.name, vsel)) continue;
            const int ks = (ri > 0 && !ks_list.empty()) ? ks_list[ri - 1] : ks_for(tiles, rg / (4 * PCX_GEMM_KS), ncu);
            int32_t* dP;
            CK(hipMalloc(&dP, (size_t)ks * outn * 4));
            CK(hipMemset(dP, 0, (size_t)ks * outn * 4));
            GemmI8 g{dA, sh.lda, (const int8_t*)dB, sh.ldb, dP, sh.trans ? sh.np : sh.nq, outn, sh.np, sh.nq, tp, tq,
                     sh.lower, ks, rg, sh.trans};
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            hipLaunchKernelGGL(v.f, dim3((unsigned)gemm_i8_items(tp, tq, sh.lower, ks)), dim3(v.threads), v.lds, 0, g);  // warm
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            std::vector<float> ms;
            for (int r = 0; r < reps; r++) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(v.f, dim3((unsigned)gemm_i8_items(tp, tq, sh.lower, ks)), dim3(v.threads), v.lds, 0, g);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t = 0;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            hipLaunchKernelGGL(k_slabsum, dim3(4096), dim3(256), 0, 0, dP, ks, outn, outn, ri == 0 ? dRef : dSum);
            unsigned long long bad = 0;
            if (ri > 0) {
                CK(hipMemset(dBad, 0, 8));
                hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, dRef, dSum, outn, dBad);
                CK(hipMemcpy(&bad, dBad, 8, hipMemcpyDeviceToHost));
            }
            CK(hipDeviceSynchronize());
            printf("%-6s %-24s ks %2d  %8.3f ms (min %8.3f)  %7.1f TOP/s  %s\n", sh.name, v.name, ks, ms[ms.size() / 2],
                   ms[0], ops / (ms[ms.size() / 2] * 1e-3) / 1e12, ri == 0 ? "reference" : (bad ? "MISMATCH" : "equal"));
            fflush(stdout);
            CK(hipFree(dP));
            if (bad) return 3;
        }
        CK(hipFree(dA));
        CK(hipFree(dB));
        CK(hipFree(dRef));
        CK(hipFree(dSum));
        CK(hipFree(dBad));
    }
    return 0;
}
