// Microbenchmark (diagnostic tool, not product): cycles per iteration of the FPS iteration
// tail pieces, one workgroup, NW waves. Build: make -C tools/ubench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../pointcloud-segmentation-attention_amd/csrc/common.h"

using namespace pn2;

template <int MODE>
__global__ void tail2_kernel(int iters, unsigned long long* out, float* sink, int* gidx) {
  __shared__ uint2 red[2][16];
  __shared__ float sxyz[3 * 8192];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, NW = blockDim.x >> 6;
  for (int e = t; e < 3 * 8192; e += blockDim.x) sxyz[e] = (float)e;
  __syncthreads();
  float cx = 0.f, acc = 0.f;
  uint32_t hi = (uint32_t)(t * 2654435761u) >> 8;
  int ring = 0;
  unsigned long long t0 = clock64();
  for (int j = 1; j <= iters; ++j) {
    const uint32_t wm = wave_max_u32(hi ^ (uint32_t)j);
    if (lane == 0) red[j & 1][w] = make_uint2(wm, wm ^ 77u);
    __syncthreads();
    const bool in = lane < NW;
    const uint2 r = in ? red[j & 1][lane] : make_uint2(0u, 0u);
    const uint32_t km = (uint32_t)__builtin_amdgcn_readlane((int)row16_max_u32(r.x), 0);
    const uint64_t ball = __ballot(in && r.x == km);
    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)r.y, __ffsll((unsigned long long)ball) - 1) & 8191u;
    if constexpr (MODE >= 1) cx = sxyz[3 * k] + sxyz[3 * k + 1];
    if constexpr (MODE == 2 || MODE == 3) {
      const int sl = j & 63;
      ring = lane == sl ? (int)k : ring;
      if constexpr (MODE == 3) if (sl == 63 && w == 0) gidx[(j & ~63) + lane] = ring;
    }
    if constexpr (MODE == 4) if (t == 0) gidx[j] = (int)k;
    hi ^= k + __float_as_uint(cx);
    acc += cx;
  }
  unsigned long long t1 = clock64();
  if (t == 0) out[0] = (t1 - t0);
  if (acc == 12345.f) sink[t] = acc + ring;
}

template <int MODE>
__global__ void tail_kernel(int iters, unsigned long long* out, float* sink) {
  __shared__ unsigned long long s_key[3];
  __shared__ float sxyz[3 * 8192];
  const int t = threadIdx.x, lane = t & 63;
  for (int e = t; e < 3 * 8192; e += blockDim.x) sxyz[e] = (float)e;
  if (t < 3) s_key[t] = 0ull;
  __syncthreads();
  float cx = 0.f, acc = 0.f;
  uint32_t hi = (uint32_t)(t * 2654435761u) >> 8;
  unsigned long long t0 = clock64();
  for (int j = 1; j <= iters; ++j) {
    if constexpr (MODE >= 2) hi = wave_max_u32(hi ^ (uint32_t)j);
    if constexpr (MODE >= 1) {
      if (MODE == 1 ? lane == 0 : (hi & 63) == (uint32_t)lane) atomicMax(&s_key[j % 3], (unsigned long long)hi + j);
    }
    __syncthreads();
    if constexpr (MODE >= 1) {
      if (t == 0) s_key[(j + 2) % 3] = 0ull;
      const uint32_t k = uniform_u32((uint32_t)s_key[j % 3]) & 8191u;
      if constexpr (MODE >= 3) cx = sxyz[3 * k] + sxyz[3 * k + 1];
      hi ^= k;
    }
    acc += cx;
  }
  unsigned long long t1 = clock64();
  if (t == 0) out[0] = (t1 - t0);
  if (acc == 12345.f) sink[t] = acc;
}

extern "C" int ubench_tail(int mode, int nthreads, int iters, unsigned long long* out_dev, float* sink) {
  switch (mode) {
    case 0: hipLaunchKernelGGL(tail_kernel<0>, dim3(1), dim3(nthreads), 0, 0, iters, out_dev, sink); break;
    case 1: hipLaunchKernelGGL(tail_kernel<1>, dim3(1), dim3(nthreads), 0, 0, iters, out_dev, sink); break;
    case 2: hipLaunchKernelGGL(tail_kernel<2>, dim3(1), dim3(nthreads), 0, 0, iters, out_dev, sink); break;
    case 3: hipLaunchKernelGGL(tail_kernel<3>, dim3(1), dim3(nthreads), 0, 0, iters, out_dev, sink); break;
    default: return -22;
  }
  return (int)hipDeviceSynchronize();
}

extern "C" int ubench_tail2(int mode, int nthreads, int iters, unsigned long long* out_dev, float* sink, int* gidx) {
  switch (mode) {
    case 0: hipLaunchKernelGGL(tail2_kernel<0>, dim3(1), dim3(nthreads), 0, 0, iters, out_dev, sink, gidx); break;
    case 1: hipLaunchKernelGGL(tail2_kernel<1>, dim3(1), dim3(nthreads), 0, 0, iters, out_dev, sink, gidx); break;
    case 2: hipLaunchKernelGGL(tail2_kernel<2>, dim3(1), dim3(nthreads), 0, 0, iters, out_dev, sink, gidx); break;
    case 3: hipLaunchKernelGGL(tail2_kernel<3>, dim3(1), dim3(nthreads), 0, 0, iters, out_dev, sink, gidx); break;
    case 4: hipLaunchKernelGGL(tail2_kernel<4>, dim3(1), dim3(nthreads), 0, 0, iters, out_dev, sink, gidx); break;
    default: return -22;
  }
  return (int)hipDeviceSynchronize();
}

// calibration: cycles between back-to-back s_memtime stamps
__global__ void stamp_kernel(unsigned long long* out) {
  unsigned long long a, b;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(a)::"memory");
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(b)::"memory");
  unsigned long long c = clock64(), d = clock64();
  if (threadIdx.x == 0) { out[0] = b - a; out[1] = d - c; }
}
extern "C" int ubench_stamp(unsigned long long* out_dev) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, 0, out_dev);
  return (int)hipDeviceSynchronize();
}
