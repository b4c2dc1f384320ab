// Ball-query radius grouping for gfx950.
//
// Replaces QueryBallPointGpuOp / query_ball_point_gpu
// (pointnet2_tensorflow/tf_ops/grouping/tf_grouping.cpp:66-106, tf_grouping_g.cu:3-36) whose
// CPU twin is grouping/test/query_ball_point.cpp:19-47.
//
// Semantics kept bit-exact:
//  * membership: max(sqrtf(d2), 1e-20f) < radius, d2 = ((dx*dx+dy*dy)+dz*dz) fp32 (:24-25).
//    sqrt_rn is monotone, so that predicate equals  d2 < T  for one fp32 threshold T that the
//    host finds by bisection over float bit patterns (pn2_ball_threshold) — no sqrt on device;
//  * hits are the FIRST nsample points in index order (:15-17); slots after the last hit
//    repeat the first hit (:26-29); pts_cnt = hits found, capped at nsample (:34).
//
// Design: one wavefront per query. The query's cloud is staged once per workgroup into LDS
// as SoA x[],y[],z[] (conflict-free ds_read_b32 per lane); the wave tests 64 consecutive
// points per step (4 steps unrolled for memory-level parallelism), compacts hits IN ORDER with
// __ballot + popcount of the lower lanes, and leaves the scan as soon as nsample hits are in
// (a wave-uniform exit). Many queries per cloud are split across workgroups so every CU is
// busy (the reference runs one 256-thread block per cloud).
#include <math.h>
#include <string.h>

#include "common.h"

namespace pn2 {
namespace {

constexpr int kUnroll = 4;  // 64-point steps per scan iteration

template <int BLOCK, int CAP>  // CAP = LDS capacity in points (0 = read xyz1 from global)
__global__ __launch_bounds__(BLOCK) void ball_query_kernel(const float* __restrict__ xyz1,
                                                           const float* __restrict__ xyz2, int N,
                                                           int M, float thresh, int ns, int qpb,
                                                           int32_t* __restrict__ idx,
                                                           int32_t* __restrict__ pts_cnt) {
  constexpr int NW = BLOCK / kWave;
  __shared__ float sx[CAP > 0 ? CAP : 1], sy[CAP > 0 ? CAP : 1], sz[CAP > 0 ? CAP : 1];
  const int b = blockIdx.y;
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const float* __restrict__ P = xyz1 + (size_t)b * N * 3;
  if constexpr (CAP > 0) {
    for (int e = t; e < N; e += BLOCK) {
      sx[e] = P[3 * e + 0];
      sy[e] = P[3 * e + 1];
      sz[e] = P[3 * e + 2];
    }
    __syncthreads();
  }
  const uint64_t lower = (lane == 0) ? 0ull : (~0ull >> (64 - lane));  // lanes below this one
  const int q_end = min(M, (int)(blockIdx.x + 1) * qpb);
  for (int q = blockIdx.x * qpb + w; q < q_end; q += NW) {
    const float* Q = xyz2 + ((size_t)b * M + q) * 3;
    const float qx = Q[0], qy = Q[1], qz = Q[2];
    int32_t* __restrict__ row = idx + ((size_t)b * M + q) * ns;
    int cnt = 0, first = 0;
    for (int base = 0; base < N && cnt < ns; base += kWave * kUnroll) {
      bool hit[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int k = base + u * kWave + lane;
        hit[u] = false;
        if (k < N) {
          float x, y, z;
          if constexpr (CAP > 0) { x = sx[k]; y = sy[k]; z = sz[k]; }
          else { x = P[3 * k]; y = P[3 * k + 1]; z = P[3 * k + 2]; }
          hit[u] = sqdist(qx, qy, qz, x, y, z) < thresh;  // tf_grouping_g.cu:24-25
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const uint64_t mask = __ballot(hit[u]);
        if (mask != 0ull && cnt < ns) {
          if (cnt == 0) first = base + u * kWave + (__ffsll((unsigned long long)mask) - 1);
          const int pos = cnt + __popcll(mask & lower);
          if (hit[u] && pos < ns) row[pos] = base + u * kWave + lane;
          cnt += __popcll(mask);
        }
      }
    }
    if (cnt > ns) cnt = ns;
    for (int p = cnt + lane; p < ns; p += kWave) row[p] = first;  // :26-29 (0 when no hit)
    if (lane == 0) pts_cnt[(size_t)b * M + q] = cnt;
  }
}

template <int BLOCK, int CAP>
void launch_bq(const float* xyz1, const float* xyz2, int B, int N, int M, float T, int ns,
               int32_t* idx, int32_t* cnt, hipStream_t s) {
  constexpr int NW = BLOCK / kWave;
  // ~2 workgroups per CU over the whole batch, at least one query per wave
  const long long queries = (long long)B * M;
  long long qpb = (queries + 511) / 512;
  qpb = ((qpb + NW - 1) / NW) * NW;
  if (qpb < NW) qpb = NW;
  const unsigned gx = (unsigned)((M + qpb - 1) / qpb);
  hipLaunchKernelGGL((ball_query_kernel<BLOCK, CAP>), dim3(gx, B), dim3(BLOCK), 0, s, xyz1, xyz2,
                     N, M, T, ns, (int)qpb, idx, cnt);
}

}  // namespace
}  // namespace pn2

extern "C" {

float pn2_ball_threshold(float radius) {
  // smallest fp32 d2 >= 0 with max(sqrtf(d2),1e-20f) >= radius; hit <=> d2 < T.
  if (!(radius > 1e-20f)) return 0.0f;  // nothing is ever inside (and NaN radius)
  uint32_t lo = 0u, hi = 0x7F800000u;   // [+0, +inf]; sqrtf(+inf) = inf >= radius
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    float f;
    memcpy(&f, &mid, 4);
    const float s = sqrtf(f);
    const float d = s > 1e-20f ? s : 1e-20f;
    if (d >= radius) hi = mid; else lo = mid + 1;
  }
  float T;
  memcpy(&T, &lo, 4);
  return T;
}

int pn2_ball_query(const float* xyz1, const float* xyz2, int B, int N, int M, float radius,
                   int nsample, int32_t* idx, int32_t* pts_cnt, pn2_stream_t stream) {
  if (!(radius > 0.0f) || nsample <= 0 || B < 0 || N < 0 || M < 0) return PN2_EINVAL;
  if ((long long)B * M == 0) return PN2_OK;
  if (!xyz2 || !idx || !pts_cnt || (N > 0 && !xyz1)) return PN2_EINVAL;
  if (B > 65535) return PN2_EINVAL;
  const float T = pn2_ball_threshold(radius);
  hipStream_t s = (hipStream_t)stream;
  if (N <= 1024) pn2::launch_bq<256, 1024>(xyz1, xyz2, B, N, M, T, nsample, idx, pts_cnt, s);
  else if (N <= 4096) pn2::launch_bq<512, 4096>(xyz1, xyz2, B, N, M, T, nsample, idx, pts_cnt, s);
  else if (N <= 8192) pn2::launch_bq<1024, 8192>(xyz1, xyz2, B, N, M, T, nsample, idx, pts_cnt, s);
  else pn2::launch_bq<1024, 0>(xyz1, xyz2, B, N, M, T, nsample, idx, pts_cnt, s);
  PN2_RETURN_LAUNCH();
}

}  // extern "C"
