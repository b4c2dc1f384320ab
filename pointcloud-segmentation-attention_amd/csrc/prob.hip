// prob_sample: sampling by a categorical distribution per batch row, gfx950.
//
// Replaces ProbSample (tf_sampling.py:14-23 -> ProbSampleGpuOp tf_sampling.cpp:66-92 ->
// probsampleLauncher tf_sampling_g.cu:197-201): an inclusive prefix sum of the weights, then
// for every uniform draw r the first index whose prefix sum reaches r * total. The output is
// an index, so it must match the reference bit for bit, and that fixes the fp32 addition order
// of the prefix sum (cumsumKernel :7-88), which this kernel reproduces:
//  - the row in chunks of 8,192; per chunk 4-element prefixes (v2+v1, v4+v3, v3+v2, v4+v2),
//    a trailing partial quad summed left to right;
//  - the quad totals scanned by the same up/down tree (pairs ((2k+2)<<u)-1 += ((2k+1)<<u)-1,
//    then ((2k+3)<<u)-1 += ((2k+2)<<u)-1), one level per barrier;
//  - each quad += the previous quad's inclusive total, + the running sum of earlier chunks,
//    which is carried with Kahan compensation.
// Layout: one 1024-thread workgroup per row, the chunk and its quad totals in LDS (the
// totals padded one float per 32 against bank conflicts; the order of additions does not
// depend on the block size or the padding). The search is one thread per draw.
#include "common.h"

namespace pn2 {
namespace {

constexpr int kScanBlock = 1024;
constexpr int kChunk = 8192;  // the reference's BlockSize * 4
constexpr int kQuads = kChunk / 4;
constexpr int kPad = 5;

PN2_DEV int padded(int i) { return i + (i >> kPad); }

__global__ __launch_bounds__(kScanBlock) void prob_cumsum_kernel(const float* __restrict__ w,
                                                                  int n, float* __restrict__ cum) {
  __shared__ float quad[kChunk];
  __shared__ float tot[kQuads + (kQuads >> kPad)];
  const float* x = w + (size_t)blockIdx.x * n;
  float* y = cum + (size_t)blockIdx.x * n;
  float run = 0.f, comp = 0.f;
  for (int j = 0; j < n; j += kChunk) {
    const int len = min(n - j, kChunk);
    const int nq = (len + 3) >> 2;
    for (int q = threadIdx.x; q < nq; q += kScanBlock) {
      const int k = 4 * q;
      if (k + 3 < len) {
        const float v1 = x[j + k];
        const float v2 = x[j + k + 1] + v1;
        const float v34 = x[j + k + 3] + x[j + k + 2];
        const float v3 = x[j + k + 2] + v2;
        const float v4 = v34 + v2;
        quad[k] = v1;
        quad[k + 1] = v2;
        quad[k + 2] = v3;
        quad[k + 3] = v4;
        tot[padded(q)] = v4;
      } else {  // the row's last, partial quad
        float v = 0.f;
        for (int e = 0; e < 4; ++e) {
          if (k + e < len) v = v + x[j + k + e];
          quad[k + e] = v;
        }
        tot[padded(q)] = v;
      }
    }
    int u = 0;
    for (; (2 << u) <= nq; ++u) {
      __syncthreads();
      for (int k = threadIdx.x; k < (nq >> (u + 1)); k += kScanBlock) {
        const int a = padded((((k << 1) + 2) << u) - 1), c = padded((((k << 1) + 1) << u) - 1);
        tot[a] = tot[a] + tot[c];
      }
    }
    for (--u; u >= 0; --u) {
      __syncthreads();
      for (int k = threadIdx.x; k < ((nq - (1 << u)) >> (u + 1)); k += kScanBlock) {
        const int a = padded((((k << 1) + 3) << u) - 1), c = padded((((k << 1) + 2) << u) - 1);
        tot[a] = tot[a] + tot[c];
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < nq; q += kScanBlock) {
      const float p = q ? tot[padded(q - 1)] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * q + e;
        if (k < len) y[j + k] = (q ? quad[k] + p : quad[k]) + run;
      }
    }
    const float t = tot[padded(nq - 1)] + comp;
    const float r2 = run + t;
    comp = t - (r2 - run);
    run = r2;
    __syncthreads();  // the next chunk overwrites quad and tot
  }
}

__global__ __launch_bounds__(256) void prob_search_kernel(const float* __restrict__ cum,
                                                          const float* __restrict__ r, int B,
                                                          int n, int m, int base,
                                                          int32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  for (int b = blockIdx.y; b < B; b += gridDim.y) {
    const float* d = cum + (size_t)b * n;
    const float q = r[(size_t)b * m + i] * d[n - 1];
    int pos = n - 1;
    for (int k = base; k >= 1; k >>= 1)
      if (pos >= k && d[pos - k] >= q) pos -= k;
    out[(size_t)b * m + i] = pos;
  }
}

}  // namespace
}  // namespace pn2

extern "C" {

size_t pn2_prob_sample_workspace_size(int B, int N) {
  return (B > 0 && N > 0) ? (size_t)B * N * sizeof(float) : 0;
}

int pn2_prob_sample(const float* inp, const float* inpr, int B, int N, int M, float* workspace,
                    size_t workspace_bytes, int32_t* out, pn2_stream_t stream) {
  if (B < 0 || N < 0 || M < 0) return PN2_EINVAL;
  if (B == 0 || M == 0) return PN2_OK;
  // n = 0 reads cum[-1] in the reference (binarysearchKernel :95); rejected here
  if (N == 0 || !inp || !inpr || !out || !workspace) return PN2_EINVAL;
  if (workspace_bytes < pn2_prob_sample_workspace_size(B, N)) return PN2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pn2::prob_cumsum_kernel, dim3((unsigned)B), dim3(pn2::kScanBlock), 0, s, inp,
                     N, workspace);
  {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  int base = 1;
  while (base < N) base <<= 1;
  const unsigned gy = (unsigned)(B < 65535 ? B : 65535);
  hipLaunchKernelGGL(pn2::prob_search_kernel, dim3((unsigned)((M + 255) / 256), gy), dim3(256), 0,
                     s, workspace, inpr, B, N, M, base, out);
  PN2_RETURN_LAUNCH();
}

}  // extern "C"
