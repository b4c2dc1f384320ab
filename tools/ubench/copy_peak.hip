// Copy-peak sweep (bench.py's copy peak, csrc/copy.hip): float4 copy kernels over 1 GiB --
// unroll 1/2/4/8, plain or non-temporal loads / stores, 4/8/16 workgroups per CU of 256
// threads -- HIP events, best of 5, read + write bytes. Build: hipcc --offload-arch=gfx950 -O3
using v4f = float __attribute__((ext_vector_type(4)));
#include <hip/hip_runtime.h>
#include <cstdio>

template <int U, bool NT>
__global__ __launch_bounds__(256) void cp(const v4f* __restrict__ s, v4f* __restrict__ d, size_t n) {
  const size_t tile = 256 * U, stride = (size_t)gridDim.x * tile;
  size_t i = (size_t)blockIdx.x * tile + threadIdx.x;
  for (; i + (U - 1) * 256 < n; i += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(&s[i + u * 256]) : s[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], &d[i + u * 256]);
      else d[i + u * 256] = v[u];
    }
  }
  for (; i < n; i += 256) d[i] = s[i];
}

template <int U, bool NT>
void run(const v4f* s, v4f* d, size_t n, int cus) {
  for (int wpc : {4, 8, 16}) {
    const unsigned g = cus * wpc;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e9f;
    for (int r = 0; r < 6; ++r) {
      hipEventRecord(a);
      hipLaunchKernelGGL((cp<U, NT>), dim3(g), dim3(256), 0, 0, s, d, n);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r) best = ms < best ? ms : best;
    }
    printf("{\"unroll\": %d, \"nt\": %d, \"wg_per_cu\": %d, \"GBps\": %.1f}\n", U, NT ? 1 : 0, wpc,
           2.0 * n * 16 / (best * 1e-3) / 1e9);
    hipEventDestroy(a);
    hipEventDestroy(b);
  }
}

int main() {
  const size_t bytes = 1ull << 30, n = bytes / 16;
  v4f *s, *d;
  if (hipMalloc(&s, bytes) || hipMalloc(&d, bytes)) return 1;
  hipMemset(s, 1, bytes);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  run<1, false>(s, d, n, cus);
  run<2, false>(s, d, n, cus);
  run<4, false>(s, d, n, cus);
  run<8, false>(s, d, n, cus);
  run<4, true>(s, d, n, cus);
  run<8, true>(s, d, n, cus);
  hipFree(s);
  hipFree(d);
  return 0;
}
