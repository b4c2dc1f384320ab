// Uniform spatial grid over the points of each cloud (built by pn2_grid_build, grid.hip),
// shared by the grid ball query (grid.hip) and the grid three_nn (interp.hip).
//
// Per cloud, grid_stride(N) bytes: header {bbox min, 1/cell edge, dims}, the exclusive cell
// offsets (kGridCap + 1 ints), then the N points sorted by cell as float4 (x, y, z, bits(k)),
// k = the point's index in the input. Cells are ordered x fastest, so the cells x0..x1 of one
// (y, z) row are one contiguous range of the sorted points.
#pragma once
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

}  // namespace pn2
