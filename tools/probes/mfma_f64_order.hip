// Probe: is v_mfma_f64_16x16x4_f64 accumulated over K in chunks of 4 bit-identical to a
// sequential fma chain acc = fma(a_k, b_k, acc), k = 0..K-1?  (Decides whether the
// batched kernel's SPEC covariance order can run on MFMA unchanged.)
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/probes/mfma_f64_order.hip -o tools/probes/mfma_f64_order
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>
typedef double d4 __attribute__((ext_vector_type(4)));

// A [16][K] (row m, k), B [K][16]; K multiple of 4
__global__ void k_mfma(const double* A, const double* B, int K, double* D) {
    const int l = threadIdx.x;
    d4 acc = {0, 0, 0, 0};
    for (int k0 = 0; k0 < K; k0 += 4) {
        const double a = A[(l & 15) * K + k0 + (l >> 4)];
        const double b = B[(k0 + (l >> 4)) * 16 + (l & 15)];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; r++) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

__global__ void k_chain(const double* A, const double* B, int K, double* D) {
    const int m = threadIdx.x >> 4, n = threadIdx.x & 15;
    if (threadIdx.x >= 256) return;
    double acc = 0.0;
    for (int k = 0; k < K; k++) acc = fma(A[m * K + k], B[k * 16 + n], acc);
    D[m * 16 + n] = acc;
}

__global__ void k_chain_mul_add(const double* A, const double* B, int K, double* D) {
    const int m = threadIdx.x >> 4, n = threadIdx.x & 15;
    double acc = 0.0;
    for (int k = 0; k < K; k++) acc = acc + A[m * K + k] * B[k * 16 + n];
    D[m * 16 + n] = acc;
}

int main() {
    const int K = 52;
    int mism_fma = 0, mism_ma = 0, tot = 0;
    srand(7);
    for (int trial = 0; trial < 200; trial++) {
        std::vector<double> A(16 * K), B(K * 16);
        for (auto& x : A) x = (rand() / (double)RAND_MAX - 0.5) * (trial % 3 == 0 ? 1e8 : 1.0) + (trial % 5 == 0 ? 1.0 : 0.0);
        for (auto& x : B) x = (rand() / (double)RAND_MAX - 0.5) * (trial % 7 == 0 ? 1e-8 : 1.0);
        double *dA, *dB, *d1, *d2, *d3;
        hipMalloc(&dA, A.size() * 8); hipMalloc(&dB, B.size() * 8);
        hipMalloc(&d1, 256 * 8); hipMalloc(&d2, 256 * 8); hipMalloc(&d3, 256 * 8);
        hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, dA, dB, K, d1);
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(256), 0, 0, dA, dB, K, d2);
        hipLaunchKernelGGL(k_chain_mul_add, dim3(1), dim3(256), 0, 0, dA, dB, K, d3);
        std::vector<double> h1(256), h2(256), h3(256);
        hipMemcpy(h1.data(), d1, 2048, hipMemcpyDeviceToHost);
        hipMemcpy(h2.data(), d2, 2048, hipMemcpyDeviceToHost);
        hipMemcpy(h3.data(), d3, 2048, hipMemcpyDeviceToHost);
        for (int i = 0; i < 256; i++) {
            mism_fma += memcmp(&h1[i], &h2[i], 8) != 0;
            mism_ma += memcmp(&h1[i], &h3[i], 8) != 0;
            tot++;
        }
        hipFree(dA); hipFree(dB); hipFree(d1); hipFree(d2); hipFree(d3);
    }
    printf("{\"probe\":\"mfma_f64_order\",\"entries\":%d,\"mismatch_vs_fma_chain\":%d,\"mismatch_vs_mul_add_chain\":%d}\n",
           tot, mism_fma, mism_ma);
    return 0;
}
