// i8bench.hip -- standalone benchmark of the M_COV_I8 int8 products (pyconsensus_amd/csrc/pcx_gemm_i8.h)
// at the C5 shapes (1M rows: 62,504 groups of 16), every configuration checked against the
// product's (k_gemm_i8<16, GEMM_I8_NBUF>) as the int64 sum of its k-slice slabs, and all of them
// against a CPU reference on a small case.
//   mixed: A = PCX_NDIG int8 digits x 1,024 general positions, B = z of 3,072 grid events
//          (packed 2 bits), stored transposed;
//   grid:  A = tok z (int8, 3,072 positions), B = z packed, lower tiles.
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
    const int64_t rg = rows / 16;
    int ncu = 256;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<Variant> vs = {
        {"k_gemm_i8<16,3> (product)", k_gemm_i8<16, 3>, 1024, 3 * PCX_GEMM_KS * (G_PANEL + G_PANEL_PK)},
        {"k_gemm_i8<16,4>", k_gemm_i8<16, 4>, 1024, 4 * PCX_GEMM_KS * (G_PANEL + G_PANEL_PK)},
        {"k_gemm_i8<8,3>", k_gemm_i8<8, 3>, 512, 3 * PCX_GEMM_KS * (G_PANEL + G_PANEL_PK)},
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
