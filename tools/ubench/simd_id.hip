// Which SIMD each wave of a 1024-thread workgroup lands on (HW_ID.SIMD_ID, bits 5:4 on gfx9):
// checks the round-robin placement the sampler's ISO variant assumes (fps_cull.h).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void simd_ids(int* out) {
  const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID, all bits
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = (int)((hw >> 4) & 3);
}
int main() {
  int* d = nullptr;
  hipMalloc(&d, 8 * 16 * sizeof(int));
  hipLaunchKernelGGL(simd_ids, dim3(8), dim3(1024), 0, 0, d);
  int h[8 * 16];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int b = 0; b < 8; ++b) {
    printf("wg %d:", b);
    for (int w = 0; w < 16; ++w) printf(" %d", h[b * 16 + w]);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
