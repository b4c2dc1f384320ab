// Uniform spatial grid over the points of each cloud (built by pn2_grid_build, grid.hip),
// shared by the grid ball query (grid.hip) and the grid three_nn (interp.hip).
//
// Per cloud, grid_stride(N) bytes: header {bbox min, 1/cell edge, dims}, the exclusive cell
// offsets (kGridCap + 1 ints), then the N points sorted by cell as float4 (x, y, z, bits(k)),
// k = the point's index in the input. Cells are ordered x fastest, so the cells x0..x1 of one
// (y, z) row are one contiguous range of the sorted points.
#pragma once
#include <math.h>

#include "common.h"

namespace pn2 {

constexpr int kGridCap = 32768;  // cells per cloud: the build's counting sort lives in LDS
// an automatic-edge grid (cell_edge <= 0) has at most max(N, kAutoMinCells) cells
constexpr int kAutoMinCells = 64;

struct GridHdr {
  float ox, oy, oz, inv;  // bbox min, 1 / cell edge (0: one cell)
  int nx, ny, nz, ncell;
};
constexpr size_t kGridOffBytes =
    ((sizeof(GridHdr) + (size_t)(kGridCap + 1) * 4) + 15) & ~(size_t)15;

__host__ __device__ inline size_t grid_stride(int N) { return kGridOffBytes + (size_t)N * 16; }

struct GridView {
  GridHdr h;
  const int* off;
  const float4* pts;
};
PN2_DEV GridView grid_view(const void* grid, int b, int N) {
  const char* G = (const char*)grid + (size_t)b * grid_stride(N);
  GridView v;
  v.h = *(const GridHdr*)G;
  v.off = (const int*)(G + sizeof(GridHdr));
  v.pts = (const float4*)(G + kGridOffBytes);
  return v;
}

// Monotone cell coordinate of v (NaN -> 0): clamp in float, then convert. Points and query
// ranges use the same function, so containment in real arithmetic carries over.
PN2_DEV int cell_coord(float v, float o, float inv, int n) {
  float f = floorf((v - o) * inv);
  f = fminf(fmaxf(f, 0.0f), (float)(n - 1));
  return (int)f;
}

constexpr float kAutoPointsPerCell = 2.0f;

// min / max over the wave (every lane gets it): DPP within rows of 16, then the gfx950
// permlane swaps across rows -- no LDS crossbar round trip per step (ds_bpermute shuffles)
template <bool MAX>
PN2_DEV float wave_minmax_f(float v) {
  auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : fminf(a, b); };
#define PN2_MM_DPP(C) v = op(v, __int_as_float(__builtin_amdgcn_update_dpp( \
                             __float_as_int(v), __float_as_int(v), C, 0xF, 0xF, false)))
  PN2_MM_DPP(kDppXor1);
  PN2_MM_DPP(kDppXor2);
  PN2_MM_DPP(kDppHalfMirror);
  PN2_MM_DPP(kDppMirror);
#undef PN2_MM_DPP
  {
    auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = op(__uint_as_float(x[0]), __uint_as_float(x[1]));
  }
  {
    auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = op(__uint_as_float(x[0]), __uint_as_float(x[1]));
  }
  return v;
}
PN2_DEV float wave_min_f(float v) { return wave_minmax_f<false>(v); }
PN2_DEV float wave_max_f(float v) { return wave_minmax_f<true>(v); }
// inclusive prefix sum over the wave: DPP row shifts (1, 2, 4, 8 within each 16-lane row; a
// lane without a source adds 0), then row_bcast:15 / :31 carry each row's total into the rows
// above -- six VALU steps, where the __shfl_up form was six dependent LDS-crossbar round trips
// (every lane of the wave active; SA1's grid query 22.0 -> 21.0 us, tools/bench_side.py)
PN2_DEV int wave_incl_scan(int v, int lane) {
  (void)lane;
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15, rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31, rows 2, 3
  return v;
}

// The grid's header for bbox [lo, hi] of N points (an empty / NaN-only axis as lo = hi = 0).
// One thread computes it: pn2_grid_build's workgroup, or each workgroup of the fused FP
// search (interp.hip), which builds a cloud's grid of known points in its own LDS.
// ppc: the automatic edge's points per cell (then at most max(N * 2 / ppc, 64) cells).
PN2_DEV GridHdr grid_dims(const float lo[3], const float hi[3], int N, float edge,
                          float ppc = kAutoPointsPerCell) {
  GridHdr h;
  // cell edge: the caller's, or ~kAutoPointsPerCell points per cell of the bbox volume
  // (then also at most max(N, 64) cells, which bounds the grid's size for LDS staging);
  // grown by 1.25x until the cells fit kGridCap;
  // degenerate extents (inf / NaN coordinates) fall back to one cell (inv = 0)
  // (the automatic edge's cube root in fp32: any edge gives exact search results, and the
  // double-precision cbrt held the building workgroup at its barrier)
  float c = edge;
  if (!(c > 0.0f)) {
    const float ext = fmaxf(fmaxf(hi[0] - lo[0], hi[1] - lo[1]), hi[2] - lo[2]);
    const float cells = fmaxf((float)N / ppc, 1.0f);
    c = cbrtf((hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]) / cells);
    if (!(c > 0.0f)) c = ext / cbrtf(cells);
    if (!(c > 0.0f) || !(c < INFINITY)) c = 1.0f;  // all points identical: one cell
  }
  int n[3] = {1, 1, 1};
  bool ok = false;
  for (int it = 0; it < 400 && !ok; ++it) {
    double cells = 1.0, d[3];
    for (int a = 0; a < 3; ++a) {
      d[a] = floor((double)(hi[a] - lo[a]) / (double)c) + 1.0;
      cells *= d[a];
    }
    if (cells <= (double)kGridCap &&
        (edge > 0.0f || cells <= fmax(ceil((double)N * kAutoPointsPerCell / ppc), (double)kAutoMinCells))) {
      for (int a = 0; a < 3; ++a) n[a] = (int)d[a];
      ok = true;
    } else {
      c *= 1.25f;
    }
  }
  if (!ok) { n[0] = n[1] = n[2] = 1; c = INFINITY; }
  h.ox = lo[0]; h.oy = lo[1]; h.oz = lo[2];
  h.inv = ok ? 1.0f / c : 0.0f;
  h.nx = n[0]; h.ny = n[1]; h.nz = n[2];
  h.ncell = n[0] * n[1] * n[2];
  return h;
}

// The automatic-edge grid of M points P (xyz AoS, global memory, written by this workgroup
// before a barrier), built by a whole workgroup of BLOCK threads into the grid G of one cloud
// (grid_stride(M) bytes, pn2_grid_build's layout and header: the same cells as
// pn2_grid_build(P, ..., cell_edge = 0)). The order inside a cell is the order of the atomics
// -- the searches that read a grid do not depend on it. LDS: scnt >= max(M, kAutoMinCells)
// words, red [BLOCK / 64][8] floats, wsum [BLOCK / 64] ints, one header. Every thread calls
// it, t = its thread index.
template <int BLOCK>
PN2_DEV void block_grid_build(const float* __restrict__ P, int M, char* __restrict__ G,
                              uint32_t* scnt, float (*red)[8], int* wsum, GridHdr* shh, int t) {
  constexpr int NW = BLOCK / kWave;
  const int lane = t & (kWave - 1), w = t / kWave;
  int* __restrict__ off = (int*)(G + sizeof(GridHdr));
  float4* __restrict__ pts = (float4*)(G + kGridOffBytes);
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int k = t; k < M; k += BLOCK) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float v = P[3 * k + a];
      mn[a] = fminf(mn[a], v);
      mx[a] = fmaxf(mx[a], v);
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    mn[a] = wave_min_f(mn[a]);
    mx[a] = wave_max_f(mx[a]);
  }
  if (lane == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) { red[w][a] = mn[a]; red[w][4 + a] = mx[a]; }
  }
  __syncthreads();
  if (t == 0) {
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
      lo[a] = red[0][a];
      hi[a] = red[0][4 + a];
      for (int i = 1; i < NW; ++i) { lo[a] = fminf(lo[a], red[i][a]); hi[a] = fmaxf(hi[a], red[i][4 + a]); }
      if (!(hi[a] >= lo[a])) { lo[a] = 0.0f; hi[a] = 0.0f; }  // NaN-only axis
    }
    *shh = grid_dims(lo, hi, M, 0.0f);
    *(GridHdr*)G = *shh;
  }
  __syncthreads();
  const GridHdr h = *shh;
  for (int c = t; c < h.ncell; c += BLOCK) scnt[c] = 0u;
  __syncthreads();
  auto cell_at = [&](int k) {
    const int ix = cell_coord(P[3 * k + 0], h.ox, h.inv, h.nx);
    const int iy = cell_coord(P[3 * k + 1], h.oy, h.inv, h.ny);
    const int iz = cell_coord(P[3 * k + 2], h.oz, h.inv, h.nz);
    return (iz * h.ny + iy) * h.nx + ix;
  };
  for (int k = t; k < M; k += BLOCK) atomicAdd(&scnt[cell_at(k)], 1u);
  __syncthreads();
  {  // exclusive scan of the counts: a contiguous run of cells per thread
    const int per = (h.ncell + BLOCK - 1) / BLOCK;
    const int s0 = min(t * per, h.ncell), s1 = min(s0 + per, h.ncell);
    int sum = 0;
    for (int c = s0; c < s1; ++c) sum += (int)scnt[c];
    const int incl = wave_incl_scan(sum, lane);
    if (lane == kWave - 1) wsum[w] = incl;
    __syncthreads();
    int base = incl - sum;
    for (int i = 0; i < w; ++i) base += wsum[i];
    for (int c = s0; c < s1; ++c) {
      const int n = (int)scnt[c];
      scnt[c] = (uint32_t)base;
      off[c] = base;
      base += n;
    }
    if (t == 0) off[h.ncell] = M;
  }
  __syncthreads();
  for (int k = t; k < M; k += BLOCK) {
    const int pos = (int)atomicAdd(&scnt[cell_at(k)], 1u);
    pts[pos] = make_float4(P[3 * k + 0], P[3 * k + 1], P[3 * k + 2], __int_as_float(k));
  }
}

}  // namespace pn2
