#include <hip/hip_runtime.h>
__global__ void k(unsigned* o) {
  unsigned v = threadIdx.x * 7 + 1;
  auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  auto q = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  o[threadIdx.x] = r[0]; o[64 + threadIdx.x] = r[1]; o[128 + threadIdx.x] = q[0]; o[192 + threadIdx.x] = q[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 256 * 4); hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[256]; hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  for (int t = 0; t < 4; t++) { printf("r%d:", t); for (int l = 0; l < 64; l++) printf(" %u", (h[t * 64 + l] - 1) / 7); printf("\n"); }
  return 0;
}
