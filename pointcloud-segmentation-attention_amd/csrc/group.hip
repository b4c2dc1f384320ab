// group_point (+grad) and the fused group + centre + concat of sample_and_group, gfx950.
//
// Replaces GroupPointGpuOp / group_point_gpu (tf_grouping.cpp:139-171, tf_grouping_g.cu:40-57),
// GroupPointGradGpuOp / group_point_grad_gpu (tf_grouping.cpp:174-208, tf_grouping_g.cu:61-78)
// and the TF graph glue of pointnet_util.py:39-56 (SSG: group xyz, subtract new_xyz, group
// points, concat [xyz, points]) and :186-193 (MSG: concat [points, xyz]).
//
// Design: the output (B*M*nsample rows of Cout floats) is written as one flat, fully
// coalesced stream — consecutive lanes write consecutive floats of consecutive rows — while the
// reads gather whole source rows (contiguous channels) that stay L2-resident per cloud. The
// reference instead runs one thread per query that walks nsample*C scalars (stride-C stores,
// <<<B,256>>>), plus two more TF launches for the subtraction and the concat.
// The centring is one fp32 subtraction, so the fused output is bit-identical to
// group_point(xyz) - tile(new_xyz) (pointnet_util.py:40).
#include "common.h"

namespace pn2 {
namespace {

enum Layout : int {
  kPointsOnly = 0,  // out = points[idx]                       (Cout = C)
  kXyzOnly = 1,     // out = xyz[idx] - new_xyz                (Cout = 3)
  kXyzFirst = 2,    // out = [xyz[idx] - new_xyz, points[idx]] (Cout = 3 + C)
  kXyzLast = 3,     // out = [points[idx], xyz[idx] - new_xyz] (Cout = C + 3)
};

constexpr int kBlock = 256;
// measured with tools/bench_group.py (profiles/r2/bench_group_r2.log)
constexpr int kTileElems = 2048;  // output floats per workgroup tile
constexpr int kGcU = 4;           // elements whose gathers a thread has in flight before its stores

// Tile = `rows` consecutive output rows (rows*Cout <= max(kTileElems, Cout)).
__global__ __launch_bounds__(kBlock) void group_concat_kernel(
    const float* __restrict__ xyz, const float* __restrict__ points,
    const float* __restrict__ new_xyz, const int32_t* __restrict__ idx, int N, int C, int M,
    int ns, int Cout, int layout, int rows, FastDiv div_cout, FastDiv div_ns, FastDiv div_m,
    uint32_t total_rows, int tiles, float* __restrict__ grouped_xyz, float* __restrict__ out) {
  // the tile's neighbour indices are staged in LDS first (one coalesced load per row), and a
  // thread then issues the gathers of kU elements before it stores any: one element at a time
  // made each element two dependent memory trips (idx, then the gather), latency-bound
  constexpr int kU = kGcU;
  __shared__ int s_idx[kTileElems];
  // XCD-aware order (common.h): each XCD takes a contiguous range of tiles, so the rows of a
  // cloud's xyz / points are fetched into one L2, not into all eight
  const int tile = xcd_block((int)blockIdx.x, tiles);
  if (tile >= tiles) return;  // padding blocks leave before the barrier
  const uint32_t r0 = (uint32_t)tile * (uint32_t)rows;
  const int nrows = (int)min((uint32_t)rows, total_rows - r0);
  const int elems = nrows * Cout;
  for (int rl = threadIdx.x; rl < nrows; rl += kBlock) s_idx[rl] = idx[r0 + rl];
  __syncthreads();
  for (int e0 = threadIdx.x; e0 < elems; e0 += kBlock * kU) {
    float a[kU], d[kU];
    int cxs[kU];
    uint32_t rs[kU];
    int cs[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int e = e0 + u * kBlock < elems ? e0 + u * kBlock : e0;  // (skipped below)
      const uint32_t rl = fdiv((uint32_t)e, div_cout);
      const int c = e - (int)rl * Cout;
      const uint32_t r = r0 + rl;          // row = (b*M + j)*ns + k
      const uint32_t g = fdiv(r, div_ns);  // group = b*M + j
      const uint32_t b = fdiv(g, div_m);
      const int i = s_idx[rl];
      int cx = -1;  // xyz channel, or -1 for a feature channel
      int cp = c;   // feature channel
      if (layout == kXyzOnly) cx = c;
      else if (layout == kXyzFirst) { if (c < 3) cx = c; else cp = c - 3; }
      else if (layout == kXyzLast) { if (c >= C) cx = c - C; }
      const float* pa = cx >= 0 ? xyz + ((size_t)b * N + i) * 3 + cx
                                : points + ((size_t)b * N + i) * C + cp;
      a[u] = *pa;
      d[u] = 0.0f;
      if (cx >= 0) d[u] = new_xyz[(size_t)g * 3 + cx];  // (feature lanes issue no load)
      cxs[u] = cx;
      rs[u] = r;
      cs[u] = c;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (e0 + u * kBlock >= elems) break;
      float v = a[u];
      if (cxs[u] >= 0) {
        v = a[u] - d[u];  // pointnet_util.py:40
        if (grouped_xyz) grouped_xyz[(size_t)rs[u] * 3 + cxs[u]] = v;
      }
      out[(size_t)rs[u] * Cout + cs[u]] = v;
    }
  }
}

__global__ __launch_bounds__(kBlock) void group_grad_kernel(const float* __restrict__ grad_out,
                                                            const int32_t* __restrict__ idx,
                                                            int N, int C, int rows, FastDiv div_c,
                                                            FastDiv div_ns, FastDiv div_m,
                                                            uint32_t total_rows,
                                                            float* __restrict__ grad_points) {
  const uint32_t r0 = blockIdx.x * (uint32_t)rows;
  const int nrows = (int)min((uint32_t)rows, total_rows - r0);
  const int elems = nrows * C;
  for (int e = threadIdx.x; e < elems; e += kBlock) {
    const uint32_t rl = fdiv((uint32_t)e, div_c);
    const int c = e - (int)rl * C;
    const uint32_t r = r0 + rl;
    const uint32_t b = fdiv(fdiv(r, div_ns), div_m);
    atomicAdd(&grad_points[((size_t)b * N + idx[r]) * C + c], grad_out[(size_t)r * C + c]);
  }
}

// Largest batch chunk whose 32-bit row arithmetic with magic-number division stays exact
// (common.h FastDiv): rows*ns < 2^32 and groups*M < 2^32 inside one launch.
int batch_chunk(int B, int M, int ns, int rows, int cols) {
  const long long lim = 1LL << 32;
  if ((long long)rows * cols * cols >= lim) return 0;
  const long long rows_b = (long long)M * ns;  // output rows per cloud
  const long long a = rows_b * ns, g = (long long)M * M;
  long long ch = B;
  if (a > 0) ch = ch < (lim - 1) / a ? ch : (lim - 1) / a;
  if (g > 0) ch = ch < (lim - 1) / g ? ch : (lim - 1) / g;
  if (rows_b > 0 && ch * rows_b >= (1LL << 31)) ch = ((1LL << 31) - 1) / rows_b;
  return (int)ch;
}

int launch_group(const float* xyz, const float* points, const float* new_xyz, const int32_t* idx,
                 int B, int N, int C, int M, int ns, int layout, float* grouped_xyz, float* out,
                 hipStream_t s) {
  int Cout = C;
  if (layout == kXyzOnly) Cout = 3;
  else if (layout == kXyzFirst || layout == kXyzLast) Cout = C + 3;
  if ((long long)B * M * ns == 0 || Cout == 0) return PN2_OK;
  const int rows = Cout >= kTileElems ? 1 : kTileElems / Cout;
  const int chunk = batch_chunk(B, M, ns, rows, Cout);
  if (chunk <= 0) return PN2_EINVAL;
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nb = B - b0 < chunk ? B - b0 : chunk;
    const long long total_rows = (long long)nb * M * ns;
    const long long tiles = (total_rows + rows - 1) / rows;
    hipLaunchKernelGGL(group_concat_kernel, dim3(xcd_grid(tiles)), dim3(kBlock), 0, s,
                       xyz ? xyz + (size_t)b0 * N * 3 : nullptr,
                       points ? points + (size_t)b0 * N * C : nullptr,
                       new_xyz ? new_xyz + (size_t)b0 * M * 3 : nullptr,
                       idx + (size_t)b0 * M * ns, N, C, M, ns, Cout, layout, rows,
                       make_fastdiv((uint32_t)Cout), make_fastdiv((uint32_t)ns),
                       make_fastdiv((uint32_t)M), (uint32_t)total_rows, (int)tiles,
                       grouped_xyz ? grouped_xyz + (size_t)b0 * M * ns * 3 : nullptr,
                       out + (size_t)b0 * M * ns * Cout);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return PN2_OK;
}

}  // namespace
}  // namespace pn2

extern "C" {

int pn2_group_point(const float* points, const int32_t* idx, int B, int N, int C, int M,
                    int nsample, float* out, pn2_stream_t stream) {
  if (B < 0 || N < 0 || C < 0 || M < 0 || nsample < 0) return PN2_EINVAL;
  if ((long long)B * M * nsample * C == 0) return PN2_OK;
  if (!points || !idx || !out) return PN2_EINVAL;
  return pn2::launch_group(nullptr, points, nullptr, idx, B, N, C, M, nsample, pn2::kPointsOnly,
                           nullptr, out, (hipStream_t)stream);
}

int pn2_group_point_grad(const float* grad_out, const int32_t* idx, int B, int N, int C, int M,
                         int nsample, float* grad_points, pn2_stream_t stream) {
  if (B < 0 || N < 0 || C < 0 || M < 0 || nsample < 0) return PN2_EINVAL;
  const size_t bytes = (size_t)B * N * C * sizeof(float);
  if (bytes) {
    if (!grad_points) return PN2_EINVAL;
    hipError_t e = hipMemsetAsync(grad_points, 0, bytes, (hipStream_t)stream);
    if (e != hipSuccess) return (int)e;
  }
  if ((long long)B * M * nsample == 0 || C == 0) return PN2_OK;
  if (!grad_out || !idx) return PN2_EINVAL;
  const int rows = C >= pn2::kTileElems ? 1 : pn2::kTileElems / C;
  const int chunk = pn2::batch_chunk(B, M, nsample, rows, C);
  if (chunk <= 0) return PN2_EINVAL;
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nb = B - b0 < chunk ? B - b0 : chunk;
    const long long total_rows = (long long)nb * M * nsample;
    const long long tiles = (total_rows + rows - 1) / rows;
    hipLaunchKernelGGL(pn2::group_grad_kernel, dim3((unsigned)tiles), dim3(pn2::kBlock), 0,
                       (hipStream_t)stream, grad_out + (size_t)b0 * M * nsample * C,
                       idx + (size_t)b0 * M * nsample, N, C, rows, pn2::make_fastdiv((uint32_t)C),
                       pn2::make_fastdiv((uint32_t)nsample), pn2::make_fastdiv((uint32_t)M),
                       (uint32_t)total_rows, grad_points + (size_t)b0 * N * C);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return PN2_OK;
}

int pn2_group_concat(const float* xyz, const float* points, const float* new_xyz,
                     const int32_t* idx, int B, int N, int C, int M, int nsample, int flags,
                     float* grouped_xyz, float* new_points, pn2_stream_t stream) {
  if (B < 0 || N < 0 || C < 0 || M < 0 || nsample < 0) return PN2_EINVAL;
  if ((long long)B * M * nsample == 0) return PN2_OK;
  if (!xyz || !new_xyz || !idx || !new_points) return PN2_EINVAL;
  int layout;
  if (!points) layout = pn2::kXyzOnly;  // pointnet_util.py:55-56
  else if (!(flags & PN2_USE_XYZ)) layout = pn2::kPointsOnly;
  else layout = (flags & PN2_XYZ_LAST) ? pn2::kXyzLast : pn2::kXyzFirst;
  hipStream_t s = (hipStream_t)stream;
  if (layout == pn2::kPointsOnly && grouped_xyz) {
    // grouped_xyz is still an output of sample_and_group (pointnet_util.py:58)
    int rc = pn2::launch_group(xyz, nullptr, new_xyz, idx, B, N, 0, M, nsample, pn2::kXyzOnly,
                               nullptr, grouped_xyz, s);
    if (rc) return rc;
  }
  return pn2::launch_group(xyz, points, new_xyz, idx, B, N, C, M, nsample, layout,
                           layout == pn2::kPointsOnly ? nullptr : grouped_xyz, new_points, s);
}

int pn2_sample_and_group(const float* xyz, const float* points, int B, int N, int C,
                         int npoint, float radius, int nsample, int flags, int32_t* fps_idx,
                         float* new_xyz, int32_t* idx, int32_t* pts_cnt, float* grouped_xyz,
                         float* new_points, pn2_stream_t stream) {
  int rc = pn2_fps_gather(xyz, B, N, npoint, fps_idx, new_xyz, stream);  // pointnet_util.py:34
  if (rc) return rc;
  rc = pn2_ball_query(xyz, new_xyz, B, N, npoint, radius, nsample, idx, pts_cnt, stream);  // :38
  if (rc) return rc;
  return pn2_group_concat(xyz, points, new_xyz, idx, B, N, C, npoint, nsample, flags,
                          grouped_xyz, new_points, stream);  // :39-56
}

}  // extern "C"
