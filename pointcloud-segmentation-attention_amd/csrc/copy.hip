// The HBM copy peak that bench.py quotes the roofline fractions against beside the 8 TB/s
// nominal (MI355X_MICROARCH.md: 6.29 TB/s for a float4 copy): every thread
// moves four 16-byte elements per trip, all four loads issued before the first store, over a
// grid of 16 workgroups per CU (tools/ubench/copy_peak.hip: 6.03 TB/s, the best of unroll
// 1-8, plain or non-temporal, 4-16 workgroups per CU). A measurement utility only: no operator uses it.
#include "common.h"

namespace pn2 {
namespace {

constexpr int kCopyBlock = 256;
constexpr int kCopyUnroll = 4;
using v4f = float __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kCopyBlock) void copy_f4_kernel(const v4f* __restrict__ src,
                                                             v4f* __restrict__ dst, size_t n4) {
  constexpr size_t kTile = (size_t)kCopyBlock * kCopyUnroll;
  const size_t stride = (size_t)gridDim.x * kTile;
  size_t i = (size_t)blockIdx.x * kTile + threadIdx.x;
  for (; i + (kCopyUnroll - 1) * kCopyBlock < n4; i += stride) {
    v4f v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) v[u] = __builtin_nontemporal_load(&src[i + u * kCopyBlock]);
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) __builtin_nontemporal_store(v[u], &dst[i + u * kCopyBlock]);
  }
  for (; i < n4; i += kCopyBlock) dst[i] = src[i];  // the last partial tile
}

}  // namespace
}  // namespace pn2

extern "C" int pn2_copy_f4(const void* src, void* dst, size_t bytes, int cus,
                           pn2_stream_t stream) {
  if (bytes == 0) return PN2_OK;
  if (!src || !dst || cus <= 0 || (bytes & 15) || ((((uintptr_t)src) | ((uintptr_t)dst)) & 15))
    return PN2_EINVAL;
  const size_t n4 = bytes / 16;
  const size_t tiles = (n4 + pn2::kCopyBlock * pn2::kCopyUnroll - 1) /
                       (pn2::kCopyBlock * pn2::kCopyUnroll);
  const unsigned grid = (unsigned)std::min<size_t>(tiles, (size_t)cus * 16);
  hipLaunchKernelGGL(pn2::copy_f4_kernel, dim3(grid), dim3(pn2::kCopyBlock), 0,
                     (hipStream_t)stream, (const pn2::v4f*)src, (pn2::v4f*)dst, n4);
  PN2_RETURN_LAUNCH();
}
