// Feature propagation for gfx950: three_nn, IDW weights, three_interpolate (+grad), and the
// fused pointnet_fp_module geometry.
//
// Replaces ThreeNNOp / threenn_cpu (tf_interpolate.cpp:157-187, :60-103), ThreeInterpolateOp /
// threeinterpolate_cpu (:191-222, :107-127), ThreeInterpolateGradOp (:225-262, :131-153) and
// the TF graph ops of pointnet_util.py:218-226. In the reference these run on the HOST CPU
// (DEVICE_CPU kernels only, tf_interpolate.cpp:187,222,262), so every FP layer of a GPU
// training step pays a device→host→device round trip; here they stay in HBM.
//
// three_nn semantics kept bit-exact: d2 = ((dx*dx+dy*dy)+dz*dz) in fp32 (:73, stored to a
// double without changing its value), strict '<' insertion into best1..3 (:74-89) so equal
// distances keep the lower known index, unfilled slots stay idx 0 / dist +inf (= (float)1e40).
// three_interpolate: ((p1*w1)+(p2*w2))+(p3*w3) in fp32 without FMA (:119).
//
// Design: a workgroup owns 64 unknown points of one cloud; the known cloud is staged in LDS
// as float4 tiles. Each unknown point is searched by a QUAD of lanes (lane q of the quad scans
// known points k = q mod 4: 4 distinct broadcast addresses per ds_read_b128, conflict-free),
// so a 256-thread workgroup keeps 4 waves busy per 64 points and FP4 (8192 unknowns per cloud)
// runs 8 waves per SIMD. Each lane keeps its best three sorted by (d2, k) — which is exactly
// the order the reference's stable strict-'<' insertion produces — and the quad merges its four
// lists with two xor-shuffle steps. The fused FP kernel then parks each row's (idx, weight)
// triple in LDS and writes the [interp, points1] rows; for short layers (FP1-FP3) the channel
// range is split over extra workgroups (grid.z) so that the chip is full, and the copy is
// float4-vectorised when the channel counts allow.
#include <algorithm>
#include <type_traits>

#include "grid.h"

namespace pn2 {
namespace {

constexpr int kNNBlock = 256;
constexpr int kNNGroup = 4;                       // lanes per unknown point (a quad)
constexpr int kNNRows = kNNBlock / kNNGroup;      // unknown points per workgroup
constexpr int kNNTile = 2048;                     // known points per LDS tile (32 KiB float4)

struct Best3 {
  float d1, d2, d3;
  int i1, i2, i3;
};

PN2_DEV void best3_init(Best3& b) {
  b.d1 = b.d2 = b.d3 = __builtin_inff();
  b.i1 = b.i2 = b.i3 = 0;
}

// tf_interpolate.cpp:74-89 as selects (same result: the if/else-if chain is a stable insert)
PN2_DEV void best3_insert(Best3& b, float d, int k) {
  const bool c1 = d < b.d1, c2 = d < b.d2, c3 = d < b.d3;
  b.d3 = c2 ? b.d2 : (c3 ? d : b.d3);
  b.i3 = c2 ? b.i2 : (c3 ? k : b.i3);
  b.d2 = c1 ? b.d1 : (c2 ? d : b.d2);
  b.i2 = c1 ? b.i1 : (c2 ? k : b.i2);
  b.d1 = c1 ? d : b.d1;
  b.i1 = c1 ? k : b.i1;
}

// (d, k) lexicographic insert: merging two lists that are each sorted by (d, k)
PN2_DEV bool lex_lt(float d, int k, float bd, int bk) { return d < bd || (d == bd && k < bk); }
PN2_DEV void best3_insert_lex(Best3& b, float d, int k) {
  const bool c1 = lex_lt(d, k, b.d1, b.i1), c2 = lex_lt(d, k, b.d2, b.i2),
             c3 = lex_lt(d, k, b.d3, b.i3);
  b.d3 = c2 ? b.d2 : (c3 ? d : b.d3);
  b.i3 = c2 ? b.i2 : (c3 ? k : b.i3);
  b.d2 = c1 ? b.d1 : (c2 ? d : b.d2);
  b.i2 = c1 ? b.i1 : (c2 ? k : b.i2);
  b.d1 = c1 ? d : b.d1;
  b.i1 = c1 ? k : b.i1;
}

PN2_DEV void best3_merge_xor(Best3& b, int mask) {
  const float d1 = __shfl_xor(b.d1, mask, kWave), d2 = __shfl_xor(b.d2, mask, kWave),
              d3 = __shfl_xor(b.d3, mask, kWave);
  const int i1 = __shfl_xor(b.i1, mask, kWave), i2 = __shfl_xor(b.i2, mask, kWave),
            i3 = __shfl_xor(b.i3, mask, kWave);
  best3_insert_lex(b, d1, i1);
  best3_insert_lex(b, d2, i2);
  best3_insert_lex(b, d3, i3);
}

// The (d, k)-lexicographic top 3 as three 64-bit keys (bits(d) << 32 | k): for d >= +0 (a
// sum of squares; NaN keys sort above +inf, so a NaN distance never enters, as with the float
// compares) the unsigned key order IS the lexicographic order, so an insert is three
// v_cmp_lt_u64 and the selects, where the float form took three compares and two mask
// operations per test (the grid walk's inner loop, round 6).
struct Best3K {
  uint64_t k1, k2, k3;
};
PN2_DEV uint64_t nn_key(float d, int k) {
  return ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)k;
}
PN2_DEV void best3k_init(Best3K& b) { b.k1 = b.k2 = b.k3 = nn_key(__builtin_inff(), 0); }
PN2_DEV void best3k_insert(Best3K& b, uint64_t key) {
  const bool c1 = key < b.k1, c2 = key < b.k2, c3 = key < b.k3;
  b.k3 = c2 ? b.k2 : (c3 ? key : b.k3);
  b.k2 = c1 ? b.k1 : (c2 ? key : b.k2);
  b.k1 = c1 ? key : b.k1;
}
// the quad partner's key (lane ^ 1 or lane ^ 2): DPP quad permutes, no LDS crossbar trip (a
// quad's lanes are active together, so the partner's registers are always there)
template <int CTRL>
PN2_DEV uint64_t quad_xor_u64(uint64_t v) {
  const uint32_t lo = dpp_u32<CTRL>((uint32_t)v);
  const uint32_t hi = dpp_u32<CTRL>((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
template <int CTRL>
PN2_DEV void best3k_merge_quad(Best3K& b) {
  const uint64_t o1 = quad_xor_u64<CTRL>(b.k1), o2 = quad_xor_u64<CTRL>(b.k2),
                 o3 = quad_xor_u64<CTRL>(b.k3);
  best3k_insert(b, o1);
  best3k_insert(b, o2);
  best3k_insert(b, o3);
}
PN2_DEV Best3 best3_of(const Best3K& b) {
  Best3 r;
  r.d1 = __uint_as_float((uint32_t)(b.k1 >> 32));
  r.d2 = __uint_as_float((uint32_t)(b.k2 >> 32));
  r.d3 = __uint_as_float((uint32_t)(b.k3 >> 32));
  r.i1 = (int)(uint32_t)b.k1;
  r.i2 = (int)(uint32_t)b.k2;
  r.i3 = (int)(uint32_t)b.k3;
  return r;
}

// Top-3 search of one unknown point (x1,y1,z1) by the 4 lanes of a quad over the m known
// points of one cloud. Every thread of the block must call it (tiles are staged with
// barriers). On return every lane of the quad holds the quad's result.
PN2_DEV void scan_known(const float* __restrict__ K, int m, float x1, float y1, float z1,
                        float4* sk, Best3& best, int tile = kNNTile) {
  const int q = threadIdx.x & (kNNGroup - 1);
  for (int t0 = 0; t0 < m; t0 += tile) {
    const int cnt = min(tile, m - t0);
    __syncthreads();  // previous tile fully consumed
    for (int e = threadIdx.x; e < cnt; e += kNNBlock) {
      const float* p = K + 3 * (size_t)(t0 + e);
      sk[e] = make_float4(p[0], p[1], p[2], 0.0f);
    }
    __syncthreads();
#pragma unroll 8
    for (int e = q; e < cnt; e += kNNGroup) {
      const float4 p = sk[e];
      best3_insert(best, sqdist(p.x, p.y, p.z, x1, y1, z1), t0 + e);  // (x2-x1), x2 known
    }
  }
  best3_merge_xor(best, 1);
  best3_merge_xor(best, 2);
}

// weight = (1/d)/sum(1/d), d = max(dist, 1e-10)  (pointnet_util.py:219-222)
PN2_DEV void idw(float d1, float d2, float d3, float& w1, float& w2, float& w3) {
  const float r1 = 1.0f / fmaxf(d1, 1e-10f);
  const float r2 = 1.0f / fmaxf(d2, 1e-10f);
  const float r3 = 1.0f / fmaxf(d3, 1e-10f);
  const float norm = (r1 + r2) + r3;
  w1 = r1 / norm;
  w2 = r2 / norm;
  w3 = r3 / norm;
}

__global__ __launch_bounds__(kNNBlock) void three_nn_kernel(const float* __restrict__ xyz1,
                                                            const float* __restrict__ xyz2, int n,
                                                            int m, float* __restrict__ dist,
                                                            int32_t* __restrict__ idx) {
  __shared__ float4 sk[kNNTile];
  const int b = blockIdx.y;
  const int j = blockIdx.x * kNNRows + threadIdx.x / kNNGroup;
  const bool valid = j < n;
  const float* U = xyz1 + ((size_t)b * n + (valid ? j : 0)) * 3;
  Best3 best;
  best3_init(best);
  scan_known(xyz2 + (size_t)b * m * 3, m, U[0], U[1], U[2], sk, best);
  if (valid && (threadIdx.x & (kNNGroup - 1)) == 0) {
    float* D = dist + ((size_t)b * n + j) * 3;
    int32_t* I = idx + ((size_t)b * n + j) * 3;
    D[0] = best.d1; D[1] = best.d2; D[2] = best.d3;
    I[0] = best.i1; I[1] = best.i2; I[2] = best.i3;
  }
}

// three_nn over a spatial grid of the KNOWN points (grid.h): the same (d, k)-lexicographic
// top 3 as the scan, visiting cells in cubic shells of Chebyshev radius s around the unknown
// point's cell until the third-best distance is below the squared gap to every unvisited cell
// (with a relative and an absolute slack far above fp32 rounding), or the shells cover the
// grid. Cells hold points in arbitrary order, which the lexicographic insert makes
// irrelevant. One lane per unknown point; when `ugrid` (a grid over the UNKNOWN points) is
// given, lane i takes the i-th unknown in cell order, so the lanes of a wave share cells.
// LDS: the known grid (sorted points + offsets) is staged once per workgroup when it fits.
//
// QUAD: four lanes per unknown point (the scan path's quad). The single-lane walk is
// latency-bound: at FP4 a launch is only 2048 waves (two per SIMD) and each lane's walk is a
// chain of dependent LDS reads and inserts (69 candidates per unknown on average), so the
// SIMDs mostly wait. With a quad, lane q of the quad takes every fourth point of each visited
// range (its own top 3 over its share), a launch has four times the waves, and each lane's
// chain is a quarter as long. At the end of every shell the quad merges its four lists (two
// xor exchanges, the (d, k)-lexicographic insert) into a copy that every lane of the quad
// holds, and tests the certificate on it -- the same test for all four lanes, so the quad
// leaves the walk together; the merged copy is the result.

// squared-gap certificate: every point outside the cell box [xl..xh] x [yl..yh] x [zl..zh]
// (faces on the grid boundary excepted: nothing lies beyond them) is farther from p than
// sqrt(d3), with slack for the rounding of the cell assignment and of the face coordinates
PN2_DEV bool box_certifies(const GridHdr& h, float px, float py, float pz, int xl, int xh,
                           int yl, int yh, int zl, int zh, float d3) {
  if (!(d3 < __builtin_inff())) return false;
  const float edge = 1.0f / h.inv;
  float gap = __builtin_inff();
  auto face = [&](float d, float pc, float o, int c) {
    const float fc = o + (float)c * edge;
    gap = fminf(gap, d - 1e-5f * (fabsf(pc) + fabsf(o) + fabsf(fc) + (float)c * edge) - 1e-30f);
  };
  if (xl > 0) face(px - (h.ox + (float)xl * edge), px, h.ox, xl);
  if (xh < h.nx - 1) face((h.ox + (float)(xh + 1) * edge) - px, px, h.ox, xh + 1);
  if (yl > 0) face(py - (h.oy + (float)yl * edge), py, h.oy, yl);
  if (yh < h.ny - 1) face((h.oy + (float)(yh + 1) * edge) - py, py, h.oy, yh + 1);
  if (zl > 0) face(pz - (h.oz + (float)zl * edge), pz, h.oz, zl);
  if (zh < h.nz - 1) face((h.oz + (float)(zh + 1) * edge) - pz, pz, h.oz, zh + 1);
  return gap > 0.0f && d3 < gap * gap * 0.9999f;
}

// a cell's gap along one axis from p (p's own cell: 0), less the certificate's slack (0 at
// least): every point the grid assigns to cell c of that axis is at least this far from p
// along it. Cells below p's are bounded by their upper face, cells above by their lower one
// (never a clamped grid boundary: c < cp <= n - 1 and c > cp >= 0).
PN2_DEV float axis_gap(float p, float o, float edge, int c, int cp) {
  if (c == cp) return 0.0f;
  const int f = c > cp ? c : c + 1;  // the face between p and cell c
  const float fc = o + (float)f * edge;
  const float d = c > cp ? fc - p : p - fc;
  return fmaxf(d - 1e-5f * (fabsf(p) + fabsf(o) + fabsf(fc) + (float)f * edge) - 1e-30f, 0.0f);
}
// cells whose squared gap exceeds d3 (the certificate's 0.9999 slack for the distance's fp32
// rounding) hold only points strictly farther than the third best: they cannot enter the top 3
PN2_DEV bool gap_excludes(float g2, float d3) { return d3 < g2 * 0.9999f; }

constexpr int kNNFirst = 1;  // the walk's first pass: the cube of shells 0..kNNFirst
// (Measured and not kept, profiles/r5/round2: the cube's rows a z slab at a time with the
// slab's offsets and first points loaded together -- FP4 42.5 -> 44.3 us; the walk is not
// bound by its dependent LDS round trips.)

// The three nearest known points of (px, py, pz) over a grid's sorted points (pts, off: in
// LDS or global memory), lexicographic in (d, k): cubic shells of cells around the point's
// cell until the certificate holds; G lanes (lane q of them) split each row's points and
// merge their lists at the shell's end, so all G return the same result. (Measured slower and
// removed: the G lanes dealing a shell's rows round-robin, 33 -> 49 us at FP4, profiles/r4/rows.)
template <int G, typename Off>
PN2_DEV Best3 grid_nn3(const GridHdr& h, const float4* __restrict__ pts,
                       const Off* __restrict__ off, float px, float py, float pz, int q) {
  Best3K best;
  best3k_init(best);
  auto merged = [&]() {  // the lanes' top 3 (every lane of the G gets the same)
    Best3K mb = best;
    if constexpr (G == 4) {
      best3k_merge_quad<kDppXor1>(mb);
      best3k_merge_quad<kDppXor2>(mb);
    }
    return best3_of(mb);
  };
  const int cx = cell_coord(px, h.ox, h.inv, h.nx);
  const int cy = cell_coord(py, h.oy, h.inv, h.ny);
  const int cz = cell_coord(pz, h.oz, h.inv, h.nz);
  Best3 res;
  // the first pass takes shells 0 and 1 together (the 3x3x3 block: nine full rows): the own
  // cell alone (~2 points) almost never certifies, so its merge and test were wasted
  for (int s = kNNFirst;; ++s) {
    const int xl = cx - s, xh = cx + s, yl = cy - s, yh = cy + s, zl = cz - s, zh = cz + s;
    const int x0 = max(xl, 0), x1 = min(xh, h.nx - 1);
    const bool block = s == kNNFirst;  // every row of the cube, not just its shell
    auto visit = [&](int lo, int hi) {  // sorted points [lo, hi), this lane's share
      for (int e = lo + q; e < hi; e += G) {
        const float4 p = pts[e];
        best3k_insert(best, nn_key(sqdist(p.x, p.y, p.z, px, py, pz), __float_as_int(p.w)));
      }
    };
    if (block) {
      // (Measured and not kept, profiles/r6/nn: every row's offsets read before any point and
      // two points a lane per trip -- 21.4 -> 24.2 us for the search, 70 VGPRs.)
      for (int z = max(zl, 0); z <= min(zh, h.nz - 1); ++z)
        for (int y = max(yl, 0); y <= min(yh, h.ny - 1); ++y) {
          const int row = (z * h.ny + y) * h.nx;
          visit(off[row + x0], off[row + x1 + 1]);  // a row of the block: all of x0..x1
        }
    } else {
      // shells past the first: only the cells that can still hold a point within the merged
      // third-best distance of the shells before (most of a shell is farther: skipped whole
      // z slabs and rows, face rows narrowed to their x cells within reach). The quad's lanes
      // hold the same merged list, so they take the same cells. A skipped cell is farther
      // than the final third best too (it only shrinks), so the certificate below is unchanged.
      // (Measured, tools/bench_nn.py, profiles/r6/nn: neutral at FP4's automatic edge -- 42.4
      // vs 42.6 us fused, the 27-cell first pass nearly always certifies -- and 42.5 -> 39 us
      // for the grid search over a 0.15 edge, where later shells are common.)
      const float d3 = res.d3, edge = 1.0f / h.inv;
#pragma nounroll
      for (int z = max(zl, 0); z <= min(zh, h.nz - 1); ++z) {
        const float gz = axis_gap(pz, h.oz, edge, z, cz), gz2 = gz * gz;
        if (gap_excludes(gz2, d3)) continue;
#pragma nounroll
        for (int y = max(yl, 0); y <= min(yh, h.ny - 1); ++y) {
          const float gy = axis_gap(py, h.oy, edge, y, cy), gyz = gz2 + gy * gy;
          if (gap_excludes(gyz, d3)) continue;
          const int row = (z * h.ny + y) * h.nx;
          // the row's cells in reach: a face row's x0..x1 narrowed from both ends, an inner
          // row's two shell cells xl and xh (each tested on its own)
          const bool face = z == zl || z == zh || y == yl || y == yh;
          int xa = face ? x0 : xl, xb = face ? x1 : xh;
#pragma nounroll
          while (xa <= xb) {
            const float g = axis_gap(px, h.ox, edge, xa, cx);
            if (xa >= 0 && xa < h.nx && !gap_excludes(gyz + g * g, d3)) break;
            xa = face || xa != xl ? xa + 1 : xh;
          }
#pragma nounroll
          while (xb > xa) {
            const float g = axis_gap(px, h.ox, edge, xb, cx);
            if (xb >= 0 && xb < h.nx && !gap_excludes(gyz + g * g, d3)) break;
            xb = face || xb != xh ? xb - 1 : xl;
          }
          if (xa > xb) continue;
          if (face || xa == xb) {
            visit(off[row + xa], off[row + xb + 1]);
          } else {  // both shell cells of an inner row
            visit(off[row + xa], off[row + xa + 1]);
            visit(off[row + xb], off[row + xb + 1]);
          }
        }
      }
    }
    res = merged();
    if (xl <= 0 && yl <= 0 && zl <= 0 && xh >= h.nx - 1 && yh >= h.ny - 1 && zh >= h.nz - 1)
      break;  // every cell visited
    if (box_certifies(h, px, py, pz, xl, xh, yl, yh, zl, zh, res.d3)) break;
  }
  return res;
}

// grid_nn3 for one G-lane group of a wave; a group without an unknown (valid = false) returns
// an empty list. (A wave-box first pass -- every group scans its wave's bounding box, then
// certifies -- was measured slower and removed: FP4 search 34 -> 44 us, profiles/r4/box.)
template <int G, typename Off>
PN2_DEV Best3 grid_nn3_wave(const GridHdr& h, const float4* __restrict__ pts,
                            const Off* __restrict__ off, float px, float py, float pz, int q,
                            bool valid) {
  if (valid) return grid_nn3<G, Off>(h, pts, off, px, py, pz, q);
  Best3 none;
  best3_init(none);
  return none;
}


// G lanes per unknown point (1, or 4 = a quad); BLOCK / G unknowns per row block, K row
// blocks of one cloud per workgroup
template <int BLOCK, bool LDS, int G, int K>
__global__ __launch_bounds__(BLOCK) void three_nn_grid_kernel(
    const void* __restrict__ kgrid, int m, const void* __restrict__ ugrid,
    const float* __restrict__ xyz1, int n, int B, float* __restrict__ dist,
    int32_t* __restrict__ idx) {
  static_assert(G == 1 || G == 4, "one lane or a quad per unknown");
  constexpr int QPB = BLOCK / G;  // unknowns per row block
  extern __shared__ float4 s_pts[];  // LDS: m sorted known points, then ncell+1 offsets
  // logical block (cloud b, block x of K row blocks), XCD-aware: the blocks of a cloud share
  // one L2
  const int R = (n + QPB * K - 1) / (QPB * K);
  const int Lg = xcd_block(blockIdx.x, R * B);
  if (Lg >= R * B) return;
  const int b = Lg / R;
  const int q = (int)threadIdx.x & (G - 1);
  const GridView g = grid_view(kgrid, b, m);
  const GridHdr& h = g.h;
  const float4* __restrict__ pts = g.pts;
  const int* __restrict__ off = g.off;
  // the whole known grid of this cloud, once per workgroup, when its cell count is within
  // what the launch sized the LDS for (automatic-edge grids always are)
  if (LDS && h.ncell <= max(m, kAutoMinCells)) {
    int* s_off = (int*)(s_pts + m);
    for (int e = threadIdx.x; e < m; e += BLOCK) s_pts[e] = g.pts[e];
    for (int e = threadIdx.x; e <= h.ncell; e += BLOCK) s_off[e] = g.off[e];
    __syncthreads();
    pts = s_pts;
    off = s_off;
  }
  const float4* __restrict__ upts = ugrid ? grid_view(ugrid, b, n).pts : nullptr;
  for (int kb = 0; kb < K; ++kb) {  // no barriers below; a quad's lanes share i
    const int i0 = ((Lg - b * R) * K + kb) * QPB;
    if (i0 >= n) break;  // (workgroup-uniform)
    const int i = i0 + (int)threadIdx.x / G;
    const bool valid = i < n;
    const int ic = valid ? i : n - 1;
    float px, py, pz;
    int u;
    if (upts) {
      const float4 U = upts[ic];
      px = U.x; py = U.y; pz = U.z;
      u = __float_as_int(U.w);
    } else {
      const float* U = xyz1 + ((size_t)b * n + ic) * 3;
      px = U[0]; py = U[1]; pz = U[2];
      u = ic;
    }
    const Best3 res = grid_nn3_wave<G, int>(h, pts, off, px, py, pz, q, valid);
    if (valid && q == 0) {
      float* D = dist + ((size_t)b * n + u) * 3;
      int32_t* I = idx + ((size_t)b * n + u) * 3;
      D[0] = res.d1; D[1] = res.d2; D[2] = res.d3;
      I[0] = res.i1; I[1] = res.i2; I[2] = res.i3;
    }
  }
}

__global__ void idw_kernel(const float* __restrict__ dist, int total, float* __restrict__ weight) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const float* d = dist + 3 * (size_t)i;
  float w1, w2, w3;
  idw(d[0], d[1], d[2], w1, w2, w3);
  weight[3 * (size_t)i + 0] = w1;
  weight[3 * (size_t)i + 1] = w2;
  weight[3 * (size_t)i + 2] = w3;
}

constexpr int kBlock = 256;
constexpr int kTileElems = 2048;

// out (B,n,C): flat coalesced stream, `rows` rows per workgroup
__global__ __launch_bounds__(kBlock) void three_interp_kernel(
    const float* __restrict__ points, const int32_t* __restrict__ idx,
    const float* __restrict__ weight, int m, int C, int n, int rows, FastDiv div_c,
    FastDiv div_n, uint32_t total_rows, float* __restrict__ out) {
  const uint32_t r0 = blockIdx.x * (uint32_t)rows;
  const int nrows = (int)min((uint32_t)rows, total_rows - r0);
  const int elems = nrows * C;
  for (int e = threadIdx.x; e < elems; e += kBlock) {
    const uint32_t rl = fdiv((uint32_t)e, div_c);
    const int c = e - (int)rl * C;
    const uint32_t r = r0 + rl;  // r = b*n + j
    const uint32_t b = fdiv(r, div_n);
    const int32_t* I = idx + 3 * (size_t)r;
    const float* W = weight + 3 * (size_t)r;
    const float* P = points + (size_t)b * m * C + c;
    float v = P[(size_t)I[0] * C] * W[0];
    v = v + P[(size_t)I[1] * C] * W[1];
    v = v + P[(size_t)I[2] * C] * W[2];
    out[(size_t)r * C + c] = v;
  }
}

__global__ __launch_bounds__(kBlock) void three_interp_grad_kernel(
    const float* __restrict__ grad_out, const int32_t* __restrict__ idx,
    const float* __restrict__ weight, int m, int C, int rows, FastDiv div_c, FastDiv div_n,
    uint32_t total_rows, float* __restrict__ grad_points) {
  const uint32_t r0 = blockIdx.x * (uint32_t)rows;
  const int nrows = (int)min((uint32_t)rows, total_rows - r0);
  const int elems = nrows * C;
  for (int e = threadIdx.x; e < elems; e += kBlock) {
    const uint32_t rl = fdiv((uint32_t)e, div_c);
    const int c = e - (int)rl * C;
    const uint32_t r = r0 + rl;
    const uint32_t b = fdiv(r, div_n);
    const int32_t* I = idx + 3 * (size_t)r;
    const float* W = weight + 3 * (size_t)r;
    float* G = grad_points + (size_t)b * m * C + c;
    const float g = grad_out[(size_t)r * C + c];
    atomicAdd(G + (size_t)I[0] * C, g * W[0]);  // tf_interpolate.cpp:143-145
    atomicAdd(G + (size_t)I[1] * C, g * W[1]);
    atomicAdd(G + (size_t)I[2] * C, g * W[2]);
  }
}

// pointnet_fp_module geometry (fp_fused_kernel below). One FP layer's arguments (a launch may carry several, fp_fused_layers_kernel).
struct FpLayer {
  const float* xyz1;
  const float* xyz2;
  const float* pdist;
  const int32_t* pidx;
  const void* ugrid;
  const float* points1;
  const float* points2;
  float* out;
  int C1, C2, n, m, cw, B, Z;
  FastDiv div_cw;
};

// One output row's three neighbours (I.x..z), IDW weights (W.x..z) and row index r.
struct FpRow {
  int4 I;
  float4 W;
  int r;
};

// The output rows j0 .. j0 + 63 of cloud b, column slice zb, from the rows' three neighbours
// and IDW weights (row(rl) -> FpRow for the workgroup's row rl): interpolated columns
// ((p1*w1)+(p2*w2))+(p3*w3), then the points1 concat.
template <int V2, int V1, int UN, int FB = kNNBlock, typename RowFn>
PN2_DEV void fp_write_rows(const FpLayer& p, int b, int zb, int j0, RowFn row) {
  const float* __restrict__ points1 = p.points1;
  const float* __restrict__ points2 = p.points2;
  float* __restrict__ out = p.out;
  const int C1 = p.C1, C2 = p.C2, n = p.n, m = p.m, cw = p.cw;
  const FastDiv div_cw = p.div_cw;
  const int Cout = C2 + C1;             // floats
  // columns: c2v interpolated ones of V2 floats, then c1v concat ones of V1 floats
  const int c2v = C2 / V2, coutv = c2v + C1 / V1;
  const int cb = zb * cw;               // first column of this workgroup
  const int ce = min(coutv, cb + cw);
  if (ce <= cb) return;
  // element e -> (row e / cw, column cb + e % cw); the last channel slice can be narrower
  // than cw (coutv % zsplit != 0), its surplus columns are skipped
  const int nrows = min(FB / kNNGroup, n - j0);
  const int elems = nrows * cw;
  using V2T = typename std::conditional<V2 == 4, float4, float>::type;
  using V1T = typename std::conditional<
      V1 == 4, float4, typename std::conditional<V1 == 2, float2, float>::type>::type;
  const V2T* P2 = reinterpret_cast<const V2T*>(points2 + (size_t)b * m * C2);
  const float* P1 = points1 + (size_t)b * n * C1;
  float* O = out + (size_t)b * n * Cout;
  // U elements per thread in flight: every element's loads are issued before any element is
  // combined, so a thread waits for one memory round trip per U elements (one per element
  // made this loop latency-bound: 34 dependent trips per thread at Cout = 137).
  constexpr int U = UN;
  for (int e0 = threadIdx.x; e0 < elems; e0 += FB * U) {
    V2T a[U], bb[U], cc[U];
    V1T q[U];  // (both branches set every array: arrays set on one branch went to scratch)
    float4 W[U];
    bool cat[U], ok[U];
    size_t o[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * FB;
      const int rl = (int)fdiv((uint32_t)(e < elems ? e : e0), div_cw);
      int c = cb + ((e < elems ? e : e0) - rl * cw);
      ok[u] = e < elems && c < ce;
      c = min(c, ce - 1);  // (a skipped element still loads from inside the rows)
      const FpRow rw = row(rl);
      const int r = rw.r;
      cat[u] = c >= c2v;
      W[u] = rw.W;
      if constexpr (V1 == V2) {
        // one width: no branch; a concat element loads its points1 value three times (same
        // address) and is selected as is
        const int4 I = rw.I;
        const V2T* P1v = reinterpret_cast<const V2T*>(P1);
        const V2T* pa = cat[u] ? P1v + (size_t)r * (C1 / V1) + (c - c2v) : P2 + (size_t)I.x * c2v + c;
        const V2T* pb = cat[u] ? pa : P2 + (size_t)I.y * c2v + c;
        const V2T* pc = cat[u] ? pa : P2 + (size_t)I.z * c2v + c;
        a[u] = *pa;
        bb[u] = *pb;
        cc[u] = *pc;
        q[u] = V1T{};
        o[u] = (size_t)r * Cout + (size_t)c * V2;  // (C2 + (c - c2v) V1 = c V2 here)
      } else if (!cat[u]) {
        q[u] = V1T{};
        const int4 I = rw.I;
        a[u] = P2[(size_t)I.x * c2v + c];
        bb[u] = P2[(size_t)I.y * c2v + c];
        cc[u] = P2[(size_t)I.z * c2v + c];
        o[u] = (size_t)r * Cout + (size_t)c * V2;
      } else {  // concat [interpolated, points1] (pointnet_util.py:226)
        q[u] = *reinterpret_cast<const V1T*>(P1 + (size_t)r * C1 + (size_t)(c - c2v) * V1);
        a[u] = bb[u] = cc[u] = V2T{};
        o[u] = (size_t)r * Cout + C2 + (size_t)(c - c2v) * V1;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      if constexpr (V1 == V2) {
        // three_interpolate (tf_interpolate.cpp:119): ((p1*w1)+(p2*w2))+(p3*w3), or the copy
        // (selected per component: a select of whole float4 values went through scratch)
        const bool k = cat[u];
        if constexpr (V2 == 4) {
          float4 v;
          v.x = k ? a[u].x : (a[u].x * W[u].x + bb[u].x * W[u].y) + cc[u].x * W[u].z;
          v.y = k ? a[u].y : (a[u].y * W[u].x + bb[u].y * W[u].y) + cc[u].y * W[u].z;
          v.z = k ? a[u].z : (a[u].z * W[u].x + bb[u].z * W[u].y) + cc[u].z * W[u].z;
          v.w = k ? a[u].w : (a[u].w * W[u].x + bb[u].w * W[u].y) + cc[u].w * W[u].z;
          *reinterpret_cast<float4*>(O + o[u]) = v;
        } else {
          O[o[u]] = k ? a[u] : (a[u] * W[u].x + bb[u] * W[u].y) + cc[u] * W[u].z;
        }
        continue;
      }
      if (cat[u]) {
        *reinterpret_cast<V1T*>(O + o[u]) = q[u];
        continue;
      }
      // three_interpolate (tf_interpolate.cpp:119): ((p1*w1)+(p2*w2))+(p3*w3)
      if constexpr (V2 == 4) {
        float4 v;
        v.x = (a[u].x * W[u].x + bb[u].x * W[u].y) + cc[u].x * W[u].z;
        v.y = (a[u].y * W[u].x + bb[u].y * W[u].y) + cc[u].y * W[u].z;
        v.z = (a[u].z * W[u].x + bb[u].z * W[u].y) + cc[u].z * W[u].z;
        v.w = (a[u].w * W[u].x + bb[u].w * W[u].y) + cc[u].w * W[u].z;
        if (V1 == 4 || (o[u] & 3) == 0) {  // 16 B aligned (always when C1 % 4 == 0)
          *reinterpret_cast<float4*>(O + o[u]) = v;
        } else if (V1 == 2) {  // an even row width (C1 % 2 == 0): 8 B aligned, two float2
          *reinterpret_cast<float2*>(O + o[u]) = make_float2(v.x, v.y);
          *reinterpret_cast<float2*>(O + o[u] + 2) = make_float2(v.z, v.w);
        } else {  // a row of odd width C2 + C1 starts off 16 B: four dword stores
          O[o[u]] = v.x;
          O[o[u] + 1] = v.y;
          O[o[u] + 2] = v.z;
          O[o[u] + 3] = v.w;
        }
      } else {
        O[o[u]] = (a[u] * W[u].x + bb[u] * W[u].y) + cc[u] * W[u].z;
      }
    }
  }
}

// sk: the known-point tile (dynamic LDS of `tile` float4, sized by the launch to its largest m
// up to kNNTile: a 32 KB static tile held FP1-3's workgroups to 4 per CU for m <= 256)
template <int V2, int V1, bool PRE, int UN>
PN2_DEV void fp_fused_body(const FpLayer& p, int Lg, float4* sk, int tile) {
  __shared__ int4 s_idx[kNNRows];
  __shared__ float4 s_w[kNNRows];
  __shared__ int s_row[PRE ? kNNRows : 1];
  const float* __restrict__ xyz1 = p.xyz1;
  const float* __restrict__ xyz2 = p.xyz2;
  const float* __restrict__ pdist = p.pdist;
  const int32_t* __restrict__ pidx = p.pidx;
  const void* __restrict__ ugrid = p.ugrid;
  const int n = p.n, m = p.m, Z = p.Z;
  const int R = (n + kNNRows - 1) / kNNRows;
  const int b = Lg / (R * Z);
  const int zb = (Lg - b * R * Z) / R;
  const int j0 = (Lg - b * R * Z - zb * R) * kNNRows;
  if constexpr (PRE) {
    int jj = j0 + (int)threadIdx.x;
    if (threadIdx.x < kNNRows && jj < n) {
      if (ugrid) jj = __float_as_int(grid_view(ugrid, b, n).pts[jj].w);
      s_row[threadIdx.x] = jj;
      const float* D = pdist + ((size_t)b * n + jj) * 3;
      const int32_t* I = pidx + ((size_t)b * n + jj) * 3;
      float w1, w2, w3;
      idw(D[0], D[1], D[2], w1, w2, w3);
      s_idx[threadIdx.x] = make_int4(I[0], I[1], I[2], 0);
      s_w[threadIdx.x] = make_float4(w1, w2, w3, 0.0f);
    }
  } else {
    const int jl = threadIdx.x / kNNGroup;
    const int j = j0 + jl;
    const bool valid = j < n;
    const float* U = xyz1 + ((size_t)b * n + (valid ? j : 0)) * 3;
    Best3 best;
    best3_init(best);
    scan_known(xyz2 + (size_t)b * m * 3, m, U[0], U[1], U[2], sk, best, tile);
    if ((threadIdx.x & (kNNGroup - 1)) == 0) {
      float w1, w2, w3;
      idw(best.d1, best.d2, best.d3, w1, w2, w3);
      s_idx[jl] = make_int4(best.i1, best.i2, best.i3, 0);
      s_w[jl] = make_float4(w1, w2, w3, 0.0f);
    }
  }
  __syncthreads();
  fp_write_rows<V2, V1, UN>(p, b, zb, j0, [&](int rl) {
    if constexpr (PRE) return FpRow{s_idx[rl], s_w[rl], s_row[rl]};
    else return FpRow{s_idx[rl], s_w[rl], j0 + rl};
  });
}

// Workgroup (x, b, z) of one layer: unknown points [64x, 64x+64) of cloud b, columns
// [z*cw, (z+1)*cw) of the Cout = C2 + C1 concat row (V2- / V1-float columns). PRE: the three
// neighbours come from a previous three_nn (pdist, pidx) instead of the scan; with `ugrid` (a
// grid over the unknown points) the workgroup's 64 rows are 64 consecutive points in cell
// order, so their neighbours' feature rows are shared through the caches. Logical blocks are
// XCD-aware: the blocks of a cloud share one L2, which then holds its points2 rows once.
template <int V2, int V1, bool PRE, int UN>
__global__ __launch_bounds__(kNNBlock) void fp_fused_kernel(FpLayer p, int tile) {
  extern __shared__ float4 sk[];
  const int total = (p.n + kNNRows - 1) / kNNRows * p.B * p.Z;
  const int Lg = xcd_block(blockIdx.x, total);
  if (Lg >= total) return;
  fp_fused_body<V2, V1, PRE, UN>(p, Lg, sk, tile);
}

// pointnet_fp_module geometry over a grid of the KNOWN points that every workgroup builds in
// its own LDS (FP4: the m = 1024 FPS centres of an 8192-point cloud). One launch does what
// pn2_grid_build + pn2_three_nn_grid + pn2_fp_apply did in three, each waiting for the one
// before: per workgroup (cloud b, unknowns j0 .. j0 + 63 in `ugrid` order, all columns),
//   1. the bbox of the cloud's known points and the grid's header (grid_dims, the automatic
//      edge of pn2_grid_build: ~2 points per cell, at most max(m, 64) cells);
//   2. a counting sort of the known points into cells, in LDS (the order inside a cell is
//      the order of the atomics -- the (d, k)-lexicographic search does not depend on it);
//   3. the quad search (grid_nn3_wave) of each unknown, its IDW weights, optionally dist / idx;
//   4. the rows (fp_write_rows).
// A cloud's 128 workgroups each redo steps 1-2 over 12 KB of L2-resident points, which costs
// less than the launch and the dependency they replace. Bit-identical to the three-launch path.
constexpr int kFpGridMaxKnown = 4096;  // LDS: m float4 + (max(2m / ppc, 64) + 1) offsets
constexpr float kFpgPointsPerCell = 2.0f;  // the LDS grid's points per cell (profiles/r4/ppc)
// threads per workgroup (a quad per unknown: FB / 4 unknowns). The known grid is built (or
// staged) once per workgroup, but fewer, bigger workgroups were slower at FP4: 512 / 1024
// threads 49.0 / 55.8 us against 46.9 (profiles/r5/ab_misc fb/), and so were 2 / 4 row blocks per
// 256-thread workgroup (54.9 / 80.9 us, profiles/r5/ab_misc rpw/): the search and the writes need
// the workgroups' parallelism more than the build needs amortising
constexpr int kFpgBlock = 256;
// DIAGNOSTIC build flag (tools/stamp_fp4.py): s_memtime at the phase boundaries of the first
// 4096 workgroups, read back with pn2_fpg_stamps()
#ifndef PN2_FPG_STAMP
#define PN2_FPG_STAMP 0
#endif
#if PN2_FPG_STAMP
__device__ unsigned long long g_fpg_stamp[4096 * 8];
#define PN2_FPG_T(K) if (t == 0 && Lg < 4096) g_fpg_stamp[Lg * 8 + (K)] = __builtin_amdgcn_s_memtime();
#else
#define PN2_FPG_T(K)
#endif

// LDS per workgroup of the current device (cached per device id)
size_t device_lds_per_block() {
  static size_t cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 64 * 1024;
  if (!cache[dev]) {
    int v = 0, o = 0;  // the per-block limit, or the opt-in one where the device reports it
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
      v = 0;
    if (hipDeviceGetAttribute(&o, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess)
      o = 0;
    v = std::max(v, o);
    if (v <= 0) return 64 * 1024;
    cache[dev] = (size_t)v;
  }
  return cache[dev];
}

// dynamic LDS: the m sorted points, then the ncell + 1 cell offsets as uint16 (m <= 4096)
inline size_t fp_grid_lds(int m) {
  const size_t cells = (size_t)ceil((double)m * kAutoPointsPerCell / kFpgPointsPerCell);
  return (size_t)m * 16 + ((std::max(cells, (size_t)kAutoMinCells) + 1) * 2 + 3) / 4 * 4;
}

// KPT: known points per thread (m <= KPT * kNNBlock), kept in registers between the count
// and the scatter. LDS at FP4 (m = 1024, B = 16): 16 KB points + 2 KB offsets + 1.75 KB, so
// 8 workgroups fit a CU (the LDS bound; their 32 waves are the wave bound).
// kgrid (pn2_fp_grid_fused_known): a grid of the known points built before (the SA1 sampler
// builds it, fps.hip): a workgroup copies its cloud's header, offsets and points into LDS
// instead of steps 1-2 -- a third of the kernel's time at FP4 (profiles/r5/ab). A grid with
// more cells than the LDS holds (an explicit edge) falls back to the build.
template <int V2, int V1, int UN, int KPT, int FB>
__global__ __launch_bounds__(FB) void fp_grid_fused_kernel(FpLayer p, float* __restrict__ dist,
                                                        int32_t* __restrict__ idx,
                                                        const char* __restrict__ kgrid) {
  constexpr int NW = FB / kWave;
  constexpr int FR = FB / kNNGroup;  // unknowns per workgroup
  extern __shared__ float4 s_pts[];  // m known points sorted by cell, then ncell + 1 offsets
  __shared__ int4 s_idx[FR];     // the row's three neighbours and its output row
  __shared__ float s_wv[3][FR];  // the row's IDW weights; before the search: the build's
                                      // scratch (bbox partials, scan partials, header)
  float(*red)[NW] = reinterpret_cast<float(*)[NW]>(&s_wv[0][0]);  // [6][NW] <= 64 floats
  int* wsum = reinterpret_cast<int*>(&s_wv[1][0]);
  GridHdr* shp = reinterpret_cast<GridHdr*>(&s_wv[2][0]);
  static_assert(6 * NW <= FR && sizeof(GridHdr) <= FR * 4, "build scratch fits");
  const int n = p.n, m = p.m;
  const int R = (n + FR - 1) / FR;
  const int total = R * p.B;
  const int Lg = xcd_block(blockIdx.x, total);
  if (Lg >= total) return;
  const int b = Lg / R;
  const int j0 = (Lg - b * R) * FR;
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  uint16_t* s_off = reinterpret_cast<uint16_t*>(s_pts + m);
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_pts + m);  // the offsets as counter pairs
  PN2_FPG_T(0)
  GridHdr h;
  bool built = false;
  if (kgrid) {  // the prebuilt grid, when its offsets fit the LDS's max(m, 64) + 1
    const char* G = kgrid + (size_t)b * grid_stride(m);
    h = *reinterpret_cast<const GridHdr*>(G);
    if (h.ncell >= 1 && h.ncell <= max(m, kAutoMinCells)) {
      const int* goff = reinterpret_cast<const int*>(G + sizeof(GridHdr));
      const float4* gpts = reinterpret_cast<const float4*>(G + kGridOffBytes);
      for (int i = t; i < m; i += FB) s_pts[i] = gpts[i];
      for (int i = t; i <= h.ncell; i += FB) s_off[i] = (uint16_t)goff[i];
      __syncthreads();
      built = true;
    }
  }
  if (!built) {
    const float* __restrict__ K = p.xyz2 + (size_t)b * m * 3;
    // 1. bounding box -> header
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int k = t + i * FB;
      if (k < m) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const float v = K[3 * k + a];
          mn[a] = fminf(mn[a], v);
          mx[a] = fmaxf(mx[a], v);
        }
      }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      mn[a] = wave_min_f(mn[a]);
      mx[a] = wave_max_f(mx[a]);
    }
    if (lane == 0) {
#pragma unroll
      for (int a = 0; a < 3; ++a) { red[a][w] = mn[a]; red[3 + a][w] = mx[a]; }
    }
    __syncthreads();
    if (t == 0) {
      float lo[3], hi[3];
      for (int a = 0; a < 3; ++a) {
        lo[a] = red[a][0];
        hi[a] = red[3 + a][0];
        for (int i = 1; i < NW; ++i) { lo[a] = fminf(lo[a], red[a][i]); hi[a] = fmaxf(hi[a], red[3 + a][i]); }
        if (!(hi[a] >= lo[a])) { lo[a] = 0.0f; hi[a] = 0.0f; }  // NaN-only axis
      }
      *shp = grid_dims(lo, hi, m, 0.0f, kFpgPointsPerCell);
    }
    __syncthreads();
    h = *shp;
    PN2_FPG_T(1)
    auto cell_at = [&](float x, float y, float z) {
      const int ix = cell_coord(x, h.ox, h.inv, h.nx);
      const int iy = cell_coord(y, h.oy, h.inv, h.ny);
      const int iz = cell_coord(z, h.oz, h.inv, h.nz);
      return (iz * h.ny + iy) * h.nx + ix;
    };

    // 2. counting sort in one atomic pass: each point's count atomic (16-bit halves of 32-bit
    // words; counts <= m < 2^16) returns its rank in its cell, kept with its cell in registers;
    // an exclusive scan turns the counts into the cells' offsets; the scatter needs no cursor
    for (int i = t; i < (h.ncell + 2) / 2; i += FB) s_cnt[i] = 0u;
    __syncthreads();
    int kc[KPT], kr[KPT];
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int k = t + i * FB;
      kc[i] = 0;
      kr[i] = 0;
      if (k < m) {
        const int c = cell_at(K[3 * k + 0], K[3 * k + 1], K[3 * k + 2]);
        const int sh = 16 * (c & 1);
        const uint32_t old = atomicAdd(&s_cnt[c >> 1], 1u << sh);
        kc[i] = c;
        kr[i] = (int)((old >> sh) & 0xFFFFu);
      }
    }
    __syncthreads();
    {
      const int per = (h.ncell + FB - 1) / FB;
      const int s0 = t * per, s1 = min(s0 + per, h.ncell);
      int sum = 0;
      for (int i = s0; i < s1; ++i) sum += s_off[i];
      const int incl = wave_incl_scan(sum, lane);
      if (lane == kWave - 1) wsum[w] = incl;
      __syncthreads();
      int base = incl - sum;
      for (int i = 0; i < w; ++i) base += wsum[i];
      for (int i = s0; i < s1; ++i) {
        const int c = s_off[i];
        s_off[i] = (uint16_t)base;
        base += c;
      }
      if (t == 0) s_off[h.ncell] = (uint16_t)m;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < KPT; ++i) {
      const int k = t + i * FB;
      if (k < m)
        s_pts[s_off[kc[i]] + kr[i]] = make_float4(K[3 * k + 0], K[3 * k + 1], K[3 * k + 2],
                                                  __int_as_float(k));
    }
    __syncthreads();
  }

  PN2_FPG_T(2)
  // 3. the search, a quad per unknown (the quad's lanes share j)
  const int jl = t / kNNGroup, q = t & (kNNGroup - 1);
  const int j = j0 + jl;
  {
    const bool valid = j < n;
    const int jc = valid ? j : n - 1;
    float px, py, pz;
    int u;
    if (p.ugrid) {
      const float4 U = grid_view(p.ugrid, b, n).pts[jc];
      px = U.x; py = U.y; pz = U.z;
      u = __float_as_int(U.w);
    } else {
      const float* U = p.xyz1 + ((size_t)b * n + jc) * 3;
      px = U[0]; py = U[1]; pz = U[2];
      u = jc;
    }
    const Best3 res = grid_nn3_wave<kNNGroup, uint16_t>(h, s_pts, s_off, px, py, pz, q, valid);
    if (valid && q == 0) {
      float w1, w2, w3;
      idw(res.d1, res.d2, res.d3, w1, w2, w3);
      s_idx[jl] = make_int4(res.i1, res.i2, res.i3, u);
      s_wv[0][jl] = w1;
      s_wv[1][jl] = w2;
      s_wv[2][jl] = w3;
      if (dist) {
        float* D = dist + ((size_t)b * n + u) * 3;
        int32_t* I = idx + ((size_t)b * n + u) * 3;
        D[0] = res.d1; D[1] = res.d2; D[2] = res.d3;
        I[0] = res.i1; I[1] = res.i2; I[2] = res.i3;
      }
    }
  }
  __syncthreads();
  PN2_FPG_T(3)
  // 4. the rows
  fp_write_rows<V2, V1, UN, FB>(p, b, 0, j0, [&](int rl) {
    const int4 I = s_idx[rl];
    return FpRow{I, make_float4(s_wv[0][rl], s_wv[1][rl], s_wv[2][rl], 0.0f), I.w};
  });
  PN2_FPG_T(4)
}

// Several FP layers in one launch (the FP layers that wait for the same sampler): logical
// blocks [first[i], first[i+1]) are layer i's, in fp_fused_kernel's order.
constexpr int kFpMaxLayers = PN2_FP_MAX_LAYERS;
struct FpLayers {
  FpLayer l[kFpMaxLayers];
  int first[kFpMaxLayers + 1];
  int nlayers, B;
};
template <int V2, int V1, bool PRE, int UN>
__global__ __launch_bounds__(kNNBlock) void fp_fused_layers_kernel(FpLayers a, int tile) {
  extern __shared__ float4 sk[];
  // cloud-major: cloud b's blocks of every layer are contiguous (each XCD gets whole clouds
  // and the same mix of layers); first[] = each layer's first block within a cloud
  const int per_cloud_all = a.first[a.nlayers];
  const int total = per_cloud_all * a.B;
  const int L = xcd_block(blockIdx.x, total);
  if (L >= total) return;
  const int b = L / per_cloud_all;
  const int lc = L - b * per_cloud_all;
  int li = 0;
  while (li + 1 < a.nlayers && lc >= a.first[li + 1]) ++li;
  const int per_cloud = a.first[li + 1] - a.first[li];
  fp_fused_body<V2, V1, PRE, UN>(a.l[li], b * per_cloud + (lc - a.first[li]), sk, tile);
}

// Largest batch chunk whose 32-bit row arithmetic stays exact (rows*n < 2^32, see FastDiv).
int batch_chunk(int B, int n, int C, int rows) {
  if ((long long)rows * C * C >= (1LL << 32)) return 0;
  long long per_b = (long long)n * n;  // rows of one cloud times the divisor n
  if (per_b >= (1LL << 32)) return 0;
  long long ch = ((1LL << 32) - 1) / (per_b > 0 ? per_b : 1);
  if ((long long)n * ch >= (1LL << 31)) ch = ((1LL << 31) - 1) / (n > 0 ? n : 1);
  return (int)(ch < B ? ch : B);
}

// Channel split of an FP layer over grid.z (tools/bench_layers.py): split until kFpMinBlocks
// workgroups, keeping >= kFpMinCols vector columns per workgroup and (search variant, which
// scans the m known points again per slice) m * slices <= the budget
constexpr int kFpMinBlocks = 512;  // (round 6, tools/bench_side.py: 128 / 256 / 1024 / 2048 slower)
constexpr int kFpMinCols = 16;
constexpr int kFpScanBudget = 4096;

// One layer's launch configuration: the FpLayer and its kernel variant (vector widths, PRE).
struct FpPlan {
  FpLayer p;
  int v2, v1, pre, blocks;
};

// The search (xyz1, xyz2) or precomputed neighbours (pdist, pidx).
int fp_plan(const float* xyz1, const float* xyz2, const float* pdist, const int32_t* pidx,
            const void* ugrid, const float* points1, int C1, const float* points2, int C2,
            int B, int n, int m, float* out, FpPlan& f, bool split = true) {
  const bool pre = pdist != nullptr;
  // interpolated columns of 4 floats when C2 % 4 == 0 (16 B aligned loads and, on rows that
  // start 16 B aligned, stores); concat columns of 4 when C1 % 4 == 0 as well
  const bool v2 = C2 % 4 == 0 && ((((uintptr_t)points2 | (uintptr_t)out) & 15) == 0);
  // concat columns of 4 floats when C1 % 4 == 0 (16 B aligned), of 2 when C1 is even
  // (cfg3's C1 = 6: rows of C2 + 6 floats start 8 B aligned; float2 loads and stores instead
  // of dwords), else 1
  const int v1 = !v2 ? 1
                 : C1 % 4 == 0 && (((uintptr_t)points1 & 15) == 0) ? 4
                 : C1 % 2 == 0 && (((uintptr_t)points1 & 7) == 0) ? 2 : 1;
  const int coutv = C2 / (v2 ? 4 : 1) + C1 / v1;
  const int row_blocks = (n + kNNRows - 1) / kNNRows;
  // split the channels over grid.z until ~2 workgroups per CU, keeping >= 16 vector columns
  // per workgroup and (search variant) not re-running a long known-point scan too often
  int zsplit = 1;
  while (split && (long long)row_blocks * B * zsplit < kFpMinBlocks &&
         coutv / (zsplit * 2) >= kFpMinCols &&
         (pre || (long long)m * zsplit * 2 <= kFpScanBudget))
    zsplit *= 2;
  const int cw = (coutv + zsplit - 1) / zsplit;
  if ((long long)kNNRows * cw * cw >= (1LL << 32)) return PN2_EINVAL;
  if ((long long)row_blocks * B * zsplit >= (1LL << 31) - 8) return PN2_EINVAL;
  f.p = FpLayer{xyz1, xyz2, pdist, pidx, ugrid, points1, points2, out,
                C1, C2, n, m, cw, B, zsplit, make_fastdiv((uint32_t)cw)};
  f.v2 = v2;
  f.v1 = v1;
  f.pre = pre;
  f.blocks = row_blocks * B * zsplit;
  return PN2_OK;
}

// the kernel variant of `f` over `blocks` logical blocks: K = fp_fused_kernel (arg FpLayer) or
// fp_fused_layers_kernel (arg FpLayers); two elements' loads in flight per thread
// (tools/bench_fp.py: 1 and 4 measured slower)
constexpr int kFpUnroll = 2;
// MAXM: the largest m of the launch; the search variant stages the known points in an LDS
// tile of min(MAXM, kNNTile) float4
#define PN2_FP_DISPATCH(KERNEL, f, arg, blocks, MAXM, stream)                                  \
  do {                                                                                         \
    const dim3 grid__(xcd_grid(blocks));                                                       \
    const int tile__ = std::max(1, std::min((int)(MAXM), kNNTile));                            \
    if ((f).v1 == 4) { PN2_FP_PRE(KERNEL, 4, 4, f, arg, grid__, tile__, stream); }             \
    else if ((f).v1 == 2) { PN2_FP_PRE(KERNEL, 4, 2, f, arg, grid__, tile__, stream); }        \
    else if ((f).v2) { PN2_FP_PRE(KERNEL, 4, 1, f, arg, grid__, tile__, stream); }             \
    else { PN2_FP_PRE(KERNEL, 1, 1, f, arg, grid__, tile__, stream); }                         \
  } while (0)
#define PN2_FP_PRE(KERNEL, V2, V1, f, arg, grid, tile, stream)                                 \
  if ((f).pre) hipLaunchKernelGGL((KERNEL<V2, V1, true, kFpUnroll>), grid, dim3(kNNBlock), 0, stream, arg, tile); \
  else hipLaunchKernelGGL((KERNEL<V2, V1, false, kFpUnroll>), grid, dim3(kNNBlock), (size_t)(tile) * sizeof(float4), stream, arg, tile)

int fp_launch(const float* xyz1, const float* xyz2, const float* pdist, const int32_t* pidx,
              const void* ugrid, const float* points1, int C1, const float* points2, int C2,
              int B, int n, int m, float* out, hipStream_t stream) {
  FpPlan f;
  const int rc = fp_plan(xyz1, xyz2, pdist, pidx, ugrid, points1, C1, points2, C2, B, n, m, out, f);
  if (rc != PN2_OK) return rc;
  PN2_FP_DISPATCH(fp_fused_kernel, f, f.p, f.blocks, m, stream);
  PN2_RETURN_LAUNCH();
}

// pn2_fp_grid_fused: one workgroup per 64 unknowns and all columns (no channel split: each
// workgroup searches its rows once)
int fp_grid_launch(const float* xyz1, const float* xyz2, const void* ugrid, const float* points1,
                   int C1, const float* points2, int C2, int B, int n, int m, float* out,
                   float* dist, int32_t* idx, const void* kgrid, hipStream_t stream) {
  FpPlan f;
  const int rc = fp_plan(xyz1, xyz2, nullptr, nullptr, ugrid, points1, C1, points2, C2, B, n, m,
                         out, f, /*split=*/false);
  if (rc != PN2_OK) return rc;
  const dim3 grid(xcd_grid((long long)((n + kFpgBlock / kNNGroup - 1) / (kFpgBlock / kNNGroup)) *
                           B)),
      blk(kFpgBlock);
  const size_t lds = fp_grid_lds(m);
  // the known grid must fit this device's LDS per workgroup (160 KB on gfx950; m = 4096 needs
  // ~74 KB): a smaller part reports PN2_ENOTSUP, and fp_interpolate then takes the
  // three-launch path (grid build + three_nn_grid + fp_apply)
  constexpr int FR = kFpgBlock / kNNGroup;
  if (lds + 28 * FR + 64 > device_lds_per_block()) return PN2_ENOTSUP;  // (+ s_idx, s_wv, hdr)
  if ((long long)FR * f.p.cw * f.p.cw >= (1LL << 32)) return PN2_EINVAL;
  const char* kg = (const char*)kgrid;
#define PN2_FPG_K(V2, V1, U)                                                                   \
  if (m <= 4 * kFpgBlock) hipLaunchKernelGGL((fp_grid_fused_kernel<V2, V1, U, 4, kFpgBlock>), grid, blk, lds, stream, f.p, dist, idx, kg); \
  else hipLaunchKernelGGL((fp_grid_fused_kernel<V2, V1, U, (kFpGridMaxKnown + kFpgBlock - 1) / kFpgBlock, kFpgBlock>), grid, blk, lds, stream, f.p, dist, idx, kg)
#define PN2_FPG(V2, V1) PN2_FPG_K(V2, V1, kFpUnroll);
  if (f.v1 == 4) { PN2_FPG(4, 4) }
  else if (f.v1 == 2) { PN2_FPG(4, 2) }
  else if (f.v2) { PN2_FPG(4, 1) }
  else { PN2_FPG(1, 1) }
#undef PN2_FPG
#undef PN2_FPG_K
  PN2_RETURN_LAUNCH();
}

int fp_layers_launch(const pn2_fp_layer* layers, int nlayers, int B, hipStream_t stream) {
  if (!layers || nlayers < 1 || nlayers > PN2_FP_MAX_LAYERS || B < 0 || B > 65535)
    return PN2_EINVAL;
  FpLayers a{};
  FpPlan f0{};
  long long blocks = 0;
  int nl = 0, maxm = 0;
  for (int i = 0; i < nlayers; ++i) {
    const pn2_fp_layer& s = layers[i];
    if (s.n < 0 || s.m < 0 || s.C1 < 0 || s.C2 < 0) return PN2_EINVAL;
    if (!s.points1 && s.C1 != 0) return PN2_EINVAL;
    if ((long long)B * s.n == 0 || s.C1 + s.C2 == 0) continue;  // nothing to write
    if (!s.xyz1 || !s.out || (s.m > 0 && !s.xyz2) || (s.C2 > 0 && !s.points2)) return PN2_EINVAL;
    if (s.m == 0 && s.C2 > 0) return PN2_EINVAL;
    FpPlan f;
    const int rc = fp_plan(s.xyz1, s.xyz2, nullptr, nullptr, nullptr, s.points1, s.C1,
                                s.points2, s.C2, B, s.n, s.m, s.out, f);
    if (rc != PN2_OK) return rc;
    if (nl == 0) f0 = f;
    if (f.v2 != f0.v2 || f.v1 != f0.v1) {
      // another kernel variant: this layer runs as its own launch
      PN2_FP_DISPATCH(fp_fused_kernel, f, f.p, f.blocks, s.m, stream);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return (int)e;
      continue;
    }
    a.l[nl] = f.p;
    maxm = std::max(maxm, s.m);
    a.first[nl] = (int)blocks;
    blocks += f.blocks / B;  // per cloud
    ++nl;
  }
  if (nl == 0) return PN2_OK;
  a.first[nl] = (int)blocks;
  a.nlayers = nl;
  a.B = B;
  PN2_FP_DISPATCH(fp_fused_layers_kernel, f0, a, blocks * B, maxm, stream);
  PN2_RETURN_LAUNCH();
}

}  // namespace
}  // namespace pn2

extern "C" {

int pn2_three_nn(const float* xyz1, const float* xyz2, int B, int n, int m, float* dist,
                 int32_t* idx, pn2_stream_t stream) {
  if (B < 0 || n < 0 || m < 0 || B > 65535) return PN2_EINVAL;
  if ((long long)B * n == 0) return PN2_OK;
  if (!xyz1 || !dist || !idx || (m > 0 && !xyz2)) return PN2_EINVAL;
  hipLaunchKernelGGL(pn2::three_nn_kernel, dim3((n + pn2::kNNRows - 1) / pn2::kNNRows, B),
                     dim3(pn2::kNNBlock), 0, (hipStream_t)stream, xyz1, xyz2, n, m, dist, idx);
  PN2_RETURN_LAUNCH();
}

int pn2_idw_weights(const float* dist, int B, int n, float* weight, pn2_stream_t stream) {
  if (B < 0 || n < 0) return PN2_EINVAL;
  const long long total = (long long)B * n;
  if (total == 0) return PN2_OK;
  if (total > INT32_MAX || !dist || !weight) return PN2_EINVAL;
  hipLaunchKernelGGL(pn2::idw_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, dist, (int)total, weight);
  PN2_RETURN_LAUNCH();
}

int pn2_three_interpolate(const float* points, const int32_t* idx, const float* weight, int B,
                          int m, int C, int n, float* out, pn2_stream_t stream) {
  if (B < 0 || m < 0 || C < 0 || n < 0) return PN2_EINVAL;
  if ((long long)B * n == 0 || C == 0) return PN2_OK;
  if (!points || !idx || !weight || !out) return PN2_EINVAL;
  const int rows = C >= pn2::kTileElems ? 1 : pn2::kTileElems / C;
  const int chunk = pn2::batch_chunk(B, n, C, rows);
  if (chunk <= 0) return PN2_EINVAL;
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nb = B - b0 < chunk ? B - b0 : chunk;
    const long long total_rows = (long long)nb * n;
    const long long tiles = (total_rows + rows - 1) / rows;
    hipLaunchKernelGGL(pn2::three_interp_kernel, dim3((unsigned)tiles), dim3(pn2::kBlock), 0,
                       (hipStream_t)stream, points + (size_t)b0 * m * C, idx + (size_t)b0 * n * 3,
                       weight + (size_t)b0 * n * 3, m, C, n, rows, pn2::make_fastdiv((uint32_t)C),
                       pn2::make_fastdiv((uint32_t)n), (uint32_t)total_rows,
                       out + (size_t)b0 * n * C);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return PN2_OK;
}

int pn2_three_interpolate_grad(const float* grad_out, const int32_t* idx, const float* weight,
                               int B, int n, int C, int m, float* grad_points,
                               pn2_stream_t stream) {
  if (B < 0 || m < 0 || C < 0 || n < 0) return PN2_EINVAL;
  const size_t bytes = (size_t)B * m * C * sizeof(float);
  if (bytes) {
    if (!grad_points) return PN2_EINVAL;
    hipError_t e = hipMemsetAsync(grad_points, 0, bytes, (hipStream_t)stream);
    if (e != hipSuccess) return (int)e;
  }
  if ((long long)B * n == 0 || C == 0) return PN2_OK;
  if (!grad_out || !idx || !weight) return PN2_EINVAL;
  const int rows = C >= pn2::kTileElems ? 1 : pn2::kTileElems / C;
  const int chunk = pn2::batch_chunk(B, n, C, rows);
  if (chunk <= 0) return PN2_EINVAL;
  for (int b0 = 0; b0 < B; b0 += chunk) {
    const int nb = B - b0 < chunk ? B - b0 : chunk;
    const long long total_rows = (long long)nb * n;
    const long long tiles = (total_rows + rows - 1) / rows;
    hipLaunchKernelGGL(pn2::three_interp_grad_kernel, dim3((unsigned)tiles), dim3(pn2::kBlock), 0,
                       (hipStream_t)stream, grad_out + (size_t)b0 * n * C,
                       idx + (size_t)b0 * n * 3, weight + (size_t)b0 * n * 3, m, C, rows,
                       pn2::make_fastdiv((uint32_t)C), pn2::make_fastdiv((uint32_t)n),
                       (uint32_t)total_rows, grad_points + (size_t)b0 * m * C);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return PN2_OK;
}

int pn2_fp_fused(const float* xyz1, const float* xyz2, const float* points1, int C1,
                 const float* points2, int C2, int B, int n, int m, float* out,
                 pn2_stream_t stream) {
  if (B < 0 || n < 0 || m < 0 || C1 < 0 || C2 < 0 || B > 65535) return PN2_EINVAL;
  if (!points1 && C1 != 0) return PN2_EINVAL;
  if ((long long)B * n == 0 || C1 + C2 == 0) return PN2_OK;
  if (!xyz1 || !out || (m > 0 && !xyz2) || (C2 > 0 && !points2)) return PN2_EINVAL;
  if (m == 0 && C2 > 0) return PN2_EINVAL;  // nothing to interpolate from
  return pn2::fp_launch(xyz1, xyz2, nullptr, nullptr, nullptr, points1, C1, points2, C2, B, n,
                        m, out, (hipStream_t)stream);
}

int pn2_fp_fused_layers(const pn2_fp_layer* layers, int nlayers, int B, pn2_stream_t stream) {
  return pn2::fp_layers_launch(layers, nlayers, B, (hipStream_t)stream);
}

int pn2_fp_apply(const float* dist, const int32_t* idx, const void* unknown_grid,
                 const float* points1, int C1, const float* points2, int C2, int B, int n, int m,
                 float* out, pn2_stream_t stream) {
  if (B < 0 || n < 0 || m < 0 || C1 < 0 || C2 < 0 || B > 65535) return PN2_EINVAL;
  if (!points1 && C1 != 0) return PN2_EINVAL;
  if ((long long)B * n == 0 || C1 + C2 == 0) return PN2_OK;
  if (!dist || !idx || !out || (C2 > 0 && !points2)) return PN2_EINVAL;
  if (m == 0 && C2 > 0) return PN2_EINVAL;
  return pn2::fp_launch(nullptr, nullptr, dist, idx, unknown_grid, points1, C1, points2, C2, B,
                        n, m, out, (hipStream_t)stream);
}

int pn2_fp_grid_fused(const float* xyz1, const float* xyz2, const void* unknown_grid,
                      const float* points1, int C1, const float* points2, int C2, int B, int n,
                      int m, float* out, float* dist, int32_t* idx, pn2_stream_t stream) {
  if (B < 0 || n < 0 || m < 1 || m > pn2::kFpGridMaxKnown || C1 < 0 || C2 < 0 || B > 65535)
    return PN2_EINVAL;
  if (!points1 && C1 != 0) return PN2_EINVAL;
  if ((dist == nullptr) != (idx == nullptr)) return PN2_EINVAL;
  if ((long long)B * n == 0) return PN2_OK;
  if (C1 + C2 == 0) return dist ? PN2_EINVAL : PN2_OK;  // (the search alone: pn2_three_nn_grid)
  if (!xyz2 || (!xyz1 && !unknown_grid) || !out || (C2 > 0 && !points2))
    return PN2_EINVAL;
  return pn2::fp_grid_launch(xyz1, xyz2, unknown_grid, points1, C1, points2, C2, B, n, m, out,
                             dist, idx, nullptr, (hipStream_t)stream);
}

#if PN2_FPG_STAMP
int pn2_fpg_stamps(unsigned long long* host_out) {  // 4096 x 8 u64 (DIAGNOSTIC builds only)
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(pn2::g_fpg_stamp),
                                  sizeof(unsigned long long) * 4096 * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

int pn2_fp_grid_fused_known(const void* known_grid, const float* xyz1, const float* xyz2,
                            const void* unknown_grid, const float* points1, int C1,
                            const float* points2, int C2, int B, int n, int m, float* out,
                            float* dist, int32_t* idx, pn2_stream_t stream) {
  if (!known_grid || ((uintptr_t)known_grid & 15)) return PN2_EINVAL;
  if (B < 0 || n < 0 || m < 1 || m > pn2::kFpGridMaxKnown || C1 < 0 || C2 < 0 || B > 65535)
    return PN2_EINVAL;
  if (!points1 && C1 != 0) return PN2_EINVAL;
  if ((dist == nullptr) != (idx == nullptr)) return PN2_EINVAL;
  if ((long long)B * n == 0) return PN2_OK;
  if (C1 + C2 == 0) return dist ? PN2_EINVAL : PN2_OK;
  if (!xyz2 || (!xyz1 && !unknown_grid) || !out || (C2 > 0 && !points2))
    return PN2_EINVAL;
  return pn2::fp_grid_launch(xyz1, xyz2, unknown_grid, points1, C1, points2, C2, B, n, m, out,
                             dist, idx, known_grid, (hipStream_t)stream);
}

int pn2_three_nn_grid(const void* known_grid, const void* unknown_grid, const float* xyz1,
                      int B, int n, int m, float* dist, int32_t* idx, pn2_stream_t stream) {
  if (B < 0 || n < 0 || m < 0 || B > 65535) return PN2_EINVAL;
  if ((long long)B * n == 0) return PN2_OK;
  if (!known_grid || !dist || !idx || (!unknown_grid && !xyz1)) return PN2_EINVAL;
  constexpr int BLOCK = 256;
  if ((long long)((n + BLOCK / 4 - 1) / (BLOCK / 4)) * B >= (1LL << 31) - 8) return PN2_EINVAL;
  // an automatic-edge known grid has at most max(m, kAutoMinCells) cells (grid.h); an
  // explicit-edge one may have up to kGridCap and is read from global memory
  const size_t lds = (size_t)m * 16 + (size_t)(std::max(m, pn2::kAutoMinCells) + 1) * 4;
  constexpr int G = 4, K = 1;  // a quad per unknown, one row block per workgroup
  const dim3 grid(pn2::xcd_grid((long long)((n + BLOCK / G * K - 1) / (BLOCK / G * K)) * B));
  if (lds <= 64 * 1024)
    hipLaunchKernelGGL((pn2::three_nn_grid_kernel<BLOCK, true, G, K>), grid, dim3(BLOCK), lds,
                       (hipStream_t)stream, known_grid, m, unknown_grid, xyz1, n, B, dist, idx);
  else
    hipLaunchKernelGGL((pn2::three_nn_grid_kernel<BLOCK, false, G, K>), grid, dim3(BLOCK), 0,
                       (hipStream_t)stream, known_grid, m, unknown_grid, xyz1, n, B, dist, idx);
  PN2_RETURN_LAUNCH();
}

}  // extern "C"
