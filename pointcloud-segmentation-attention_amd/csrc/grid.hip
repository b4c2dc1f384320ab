// Ball query over a uniform spatial grid, for gfx950.
//
// Same results as the brute-force scan of ball_query.hip and of the reference
// (query_ball_point_gpu, tf_grouping_g.cu:3-36): the FIRST nsample points in index order with
// max(sqrtf(d2), 1e-20f) < radius (tested as d2 < T, see pn2_ball_threshold), slots after the
// last hit repeat the first hit, pts_cnt = hits capped at nsample, 0-filled rows without hits.
//
// Why: at SA1 (8192 points, r = 0.1) almost every query has fewer than nsample hits, so the
// in-order scan with early exit degenerates into 8192 distance tests per query. Here a query
// tests only the points of the cells its ball overlaps, marks hits in a per-wave bitmask over
// point INDICES in LDS, and reads the first nsample set bits back in index order — the
// reference's order, whatever order the cells were visited in.
//
// Exactness: every point with d2 < T lies in the scanned cell range. A hit has |p - q| per
// axis <= r (1 + 3 eps); the range is computed from q -/+ (r + margin) with a margin of 1e-5
// relative to max(r, |q|, 1), far above fp32 rounding, and the cell of a coordinate,
// clamp(floor((v - o) * inv)), is a monotone function of v — the same function for points and
// for the range ends. The hit test itself is the brute-force expression.
//
// Grid layout: grid.h. pn2_grid_build sorts each cloud into cells in one workgroup (LDS
// counting sort); the cell edge is the caller's (the radius, for a ball query) or, when <= 0,
// chosen for ~2 points per cell of the bounding box; it grows until the cells fit kGridCap.
#include <math.h>

#include <algorithm>

#include "grid.h"

namespace pn2 {
namespace {

constexpr int kBuildBlock = 1024;
// rows of at least this many points on average are walked one by one (tools/bench_msg_grid.py:
// the flattened walk won on short rows, lost at r = 0.4 on r-sized cells)
constexpr int kGqLongRows = 24;
constexpr int kMaxBitWords = 4096;  // bitmask words per wave (N <= 131072)

// The cloud's points are read ONCE into registers (PPT per thread, every load issued before
// the first is used): the bounding box, the count and the scatter all work from them. The
// first version looped over the cloud three times from memory with one dependent load trip per
// iteration (~35 us for a 16,384-point cloud); PPT = 0 keeps that loop for clouds beyond
// kBuildBlock * kBuildMaxPpt points.
constexpr int kBuildMaxPpt = 16;
constexpr int kBuildSmallN = 2048;     // clouds up to this many points: 256-thread workgroups
// LDS count words of an explicit-edge build: the full cap (an 8192-word array, 32 KB, sent the
// SA1 crops' 0.1-edge grids to the global-count path: their build 24 -> 65 us, profiles/r6/gb)
constexpr int kBuildCapEdge = kGridCap;

// One workgroup of BLOCK threads per cloud. The count array lives in dynamic LDS of `cap`
// words, which the host sizes to the cells the grid can have: max(N, 64) for the automatic
// edge (grid_dims' bound), kBuildCapEdge for an explicit edge, the full kGridCap for the
// point-loop build (PPT = 0). A workgroup with ~128 KB of LDS -- the array sized kGridCap for
// every grid, as rounds 1-5 had it -- waits in a busy pipeline for a CU to drain completely
// (cfg3's 1,024-point known grid: 78.7 us per build in the pipeline against ~14 alone). A
// grid with more cells than `cap` (an explicit edge over a big extent; PPT > 0 then) counts
// in its own offset array in global memory instead.
template <int PPT, int BLOCK>
__global__ __launch_bounds__(BLOCK) void grid_build_kernel(const float* __restrict__ xyz, int N,
                                                           float edge, char* __restrict__ grid,
                                                           int cap) {
  constexpr int NW = BLOCK / kWave;
  constexpr int R = PPT > 0 ? PPT : 1;  // register slots
  extern __shared__ uint32_t s_cnt[];   // cap words
  __shared__ float red[6][NW];
  __shared__ int wsum[NW];
  __shared__ GridHdr sh;
  const int b = blockIdx.x, t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  char* G = grid + (size_t)b * grid_stride(N);
  int* __restrict__ off = (int*)(G + sizeof(GridHdr));
  float4* __restrict__ pts = (float4*)(G + kGridOffBytes);

  // 0. the thread's points (k = t + i * BLOCK), all loads in flight at once
  float rx[R], ry[R], rz[R];
  if constexpr (PPT > 0) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int k = min(t + i * BLOCK, N - 1);  // clamped: loads stay in bounds (N > 0)
      rx[i] = P[3 * k + 0];
      ry[i] = P[3 * k + 1];
      rz[i] = P[3 * k + 2];
    }
  }

  // 1. bounding box
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  if constexpr (PPT > 0) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      if (t + i * BLOCK < N) {
        mn[0] = fminf(mn[0], rx[i]); mx[0] = fmaxf(mx[0], rx[i]);
        mn[1] = fminf(mn[1], ry[i]); mx[1] = fmaxf(mx[1], ry[i]);
        mn[2] = fminf(mn[2], rz[i]); mx[2] = fmaxf(mx[2], rz[i]);
      }
    }
  } else {
    for (int k = t; k < N; k += BLOCK) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const float v = P[3 * k + a];
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
      if (!(hi[a] >= lo[a])) { lo[a] = 0.0f; hi[a] = 0.0f; }  // N == 0 or NaN-only axis
    }
    sh = grid_dims(lo, hi, N, edge);
    *(GridHdr*)G = sh;
  }
  __syncthreads();
  const GridHdr h = sh;
  auto cell_at = [&](float x, float y, float z) {
    const int ix = cell_coord(x, h.ox, h.inv, h.nx);
    const int iy = cell_coord(y, h.oy, h.inv, h.ny);
    const int iz = cell_coord(z, h.oz, h.inv, h.nz);
    return (iz * h.ny + iy) * h.nx + ix;
  };

  if (PPT > 0 && h.ncell > cap) {
    // ---- more cells than the LDS array: counts, offsets and ranks in the grid's offset array
    // (global atomics; the loads that read other threads' results bypass L1, and an agent-scope
    // fence orders each phase's writes before the barrier)
    auto fence_barrier = [] {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    };
    auto ld = [&](int i) { return __hip_atomic_load(&off[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    for (int i = t; i < h.ncell; i += BLOCK) off[i] = 0;
    fence_barrier();
    int rc[R], rk[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      rc[i] = cell_at(rx[i], ry[i], rz[i]);
      rk[i] = t + i * BLOCK < N ? atomicAdd(&off[rc[i]], 1) : 0;
    }
    fence_barrier();
    const int per = (h.ncell + BLOCK - 1) / BLOCK;
    const int s0 = min(t * per, h.ncell), s1 = min(s0 + per, h.ncell);
    int sum = 0;
    for (int i = s0; i < s1; ++i) sum += ld(i);
    const int incl = wave_incl_scan(sum, lane);
    if (lane == kWave - 1) wsum[w] = incl;
    __syncthreads();
    int base = incl - sum;
    for (int i = 0; i < w; ++i) base += wsum[i];
    for (int i = s0; i < s1; ++i) {
      const int c = ld(i);
      off[i] = base;
      base += c;
    }
    if (t == 0) off[h.ncell] = N;
    fence_barrier();
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int k = t + i * BLOCK;
      if (k < N) pts[ld(rc[i]) + rk[i]] = make_float4(rx[i], ry[i], rz[i], __int_as_float(k));
    }
    return;
  }

  uint32_t* cnt = s_cnt;
  for (int i = t; i < h.ncell; i += BLOCK) cnt[i] = 0;
  __syncthreads();

  // 2. count points per cell
  // (with the points in registers the count's atomic returns each point's rank in its cell,
  // kept beside its cell: the scatter then needs no second atomic pass)
  int rc[R], rk[R];
  if constexpr (PPT > 0) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      rc[i] = cell_at(rx[i], ry[i], rz[i]);
      rk[i] = t + i * BLOCK < N ? (int)atomicAdd(&cnt[rc[i]], 1u) : 0;
    }
  } else {
    for (int k = t; k < N; k += BLOCK)
      atomicAdd(&cnt[cell_at(P[3 * k + 0], P[3 * k + 1], P[3 * k + 2])], 1u);
  }
  __syncthreads();

  // 3. exclusive scan of the counts (contiguous chunk per thread) -> offsets and cursors
  const int per = (h.ncell + BLOCK - 1) / BLOCK;
  const int s0 = min(t * per, h.ncell), s1 = min(s0 + per, h.ncell);
  int sum = 0;
  for (int i = s0; i < s1; ++i) sum += (int)cnt[i];
  const int incl = wave_incl_scan(sum, lane);
  if (lane == kWave - 1) wsum[w] = incl;
  __syncthreads();
  int base = incl - sum;
  for (int i = 0; i < w; ++i) base += wsum[i];
  for (int i = s0; i < s1; ++i) {
    const int c = (int)cnt[i];
    cnt[i] = (uint32_t)base;
    off[i] = base;
    base += c;
  }
  if (t == 0) off[h.ncell] = N;
  __syncthreads();

  // 4. scatter the points, sorted by cell (order inside a cell does not matter)
  if constexpr (PPT > 0) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int k = t + i * BLOCK;
      if (k < N) pts[(int)cnt[rc[i]] + rk[i]] = make_float4(rx[i], ry[i], rz[i], __int_as_float(k));
    }
  } else {
    for (int k = t; k < N; k += BLOCK) {
      const float x = P[3 * k + 0], y = P[3 * k + 1], z = P[3 * k + 2];
      const int pos = (int)atomicAdd(&cnt[cell_at(x, y, z)], 1u);
      pts[pos] = make_float4(x, y, z, __int_as_float(k));
    }
  }
}

// The radii of one launch (NR of them; MSG's SA1 serves its three from one walk): per radius
// the hit threshold (pn2_ball_threshold), nsample and outputs.
struct BqRadii {
  float thresh[PN2_BQ_MAX_RADII];
  int ns[PN2_BQ_MAX_RADII];
  int32_t* idx[PN2_BQ_MAX_RADII];
  int32_t* cnt[PN2_BQ_MAX_RADII];
  float* gout[PN2_BQ_MAX_RADII];  // GROUP: the grouped rows of radius r (B,M,ns,Cout)
  const float* points;            // GROUP: the features (B,N,C), or null (C = 0)
  int C, xoff, foff, cout;        // features, xyz / feature column offsets, row width
  FastDiv div_cout;
  int nsmax;                      // max ns[r]: each wave's hit list holds NR x nsmax
};

// GROUP: also the grouped rows (B,M,ns,Cout) of sample_and_group (pointnet_util.py:38-52, the
// MSG order :186-191): the centred xyz1[idx] - xyz2 at columns xoff.. and, with features, the
// points[idx] at foff.. (SSG [xyz, points], MSG [points, xyz]; C = 0: grouped_xyz alone), so an
// SA layer's query + grouping is one launch. A wave first ranks its hits into an LDS list
// (index order, padded with the first hit as the reference pads, tf_grouping_g.cu:26-29),
// then writes the query's idx row and its ns x Cout floats as one coalesced range.
// NR radii: the cells of the largest (`radius`) are walked once, every candidate's distance is
// tested against each radius' threshold into that radius' bitmask, and each radius' rows are
// written from its own bitmask -- the same outputs as NR single-radius launches.
template <int BLOCK, bool GROUP, int NR, bool FEAT = false>
__global__ __launch_bounds__(BLOCK) void ball_query_grid_kernel(
    const char* __restrict__ grid, const float* __restrict__ xyz2, int N, int M, float radius,
    int qpb, int words, int gx, int nblk, const BqRadii rd, const float* __restrict__ xyz1) {
  constexpr int NW = BLOCK / kWave;
  extern __shared__ uint32_t bits[];  // NW x NR x words, then NW x NR x nsmax hit lists
  // XCD-aware order (common.h): each XCD takes a contiguous range of (cloud, query chunk)
  // blocks, so a cloud's grid is fetched into one L2, not into all eight
  const int lb = xcd_block((int)blockIdx.x, nblk);
  if (lb >= nblk) return;
  const int b = lb / gx, bx = lb - b * gx;
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const GridView g = grid_view(grid, b, N);
  const GridHdr& h = g.h;
  const int* __restrict__ off = g.off;
  const float4* __restrict__ pts = g.pts;
  uint32_t* mine = bits + (size_t)w * NR * words;  // radius r: mine + r * words
  // FEAT: each wave's hit lists (NR x nsmax) after the bitmasks
  int* hl = reinterpret_cast<int*>(bits + (size_t)NW * NR * words) + (size_t)w * NR * rd.nsmax;
  const int wpl = (words + kWave - 1) / kWave;  // bitmask words per lane, in lane order

  const int q_end = min(M, (bx + 1) * qpb);
  for (int q = bx * qpb + w; q < q_end; q += NW) {
    for (int i = lane; i < NR * words; i += kWave) mine[i] = 0u;
    const float* Q = xyz2 + ((size_t)b * M + q) * 3;
    const float qx = Q[0], qy = Q[1], qz = Q[2];
    auto hit = [&](const float4& p) {  // tf_grouping_g.cu:24-25, per radius
      const float d = sqdist(qx, qy, qz, p.x, p.y, p.z);
      const int k = __float_as_int(p.w);
#pragma unroll
      for (int r = 0; r < NR; ++r)
        if (d < rd.thresh[r]) atomicOr(&mine[r * words + (k >> 5)], 1u << (k & 31));
    };
    const float big = fmaxf(fmaxf(fmaxf(fabsf(qx), fabsf(qy)), fmaxf(fabsf(qz), radius)), 1.0f);
    const float rr = radius + big * 1e-5f;
    const int x0 = cell_coord(qx - rr, h.ox, h.inv, h.nx), x1 = cell_coord(qx + rr, h.ox, h.inv, h.nx);
    const int y0 = cell_coord(qy - rr, h.oy, h.inv, h.ny), y1 = cell_coord(qy + rr, h.oy, h.inv, h.ny);
    const int z0 = cell_coord(qz - rr, h.oz, h.inv, h.nz), z1 = cell_coord(qz + rr, h.oz, h.inv, h.nz);
    // the cell range as rows (z, y) of contiguous cells x0..x1: the sorted-point ranges of up
    // to 64 rows are fetched at once (lane j: row r0 + j), then the wave walks the
    // concatenation of those ranges 64 points at a time -- one dependent memory trip per 64
    // points, where a loop over the rows made two per row (its offsets) plus one per row's
    // points, most rows holding a few points
    const int nyr = y1 - y0 + 1;
    const int nrows = (z1 - z0 + 1) * nyr;
    for (int r0 = 0; r0 < nrows; r0 += kWave) {
      int beg = 0, len = 0;
      const int r = r0 + lane;
      if (r < nrows) {
        const int zr = r / nyr;
        const int row = ((z0 + zr) * h.ny + y0 + (r - zr * nyr)) * h.nx;
        beg = off[row + x0];
        len = off[row + x1 + 1] - beg;  // cells x0..x1 of a row are contiguous
      }
      const int incl = wave_incl_scan(len, lane);
      const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
      const int excl = incl - len;
      const int nr = min(kWave, nrows - r0);
      if (total >= kGqLongRows * nr) {
        // long rows (a large radius over small cells): row by row, offsets already in hand
        for (int j = 0; j < nr; ++j) {
          const int bj = __builtin_amdgcn_readlane(beg, j);
          const int lj = __builtin_amdgcn_readlane(len, j);
          for (int i = lane; i < lj; i += kWave) hit(pts[bj + i]);
        }
        continue;
      }
      for (int i0 = 0; i0 < total; i0 += kWave) {
        // the rows overlapping [i0, i0 + 64): each lane takes the last one starting at or
        // before its position (empty rows never qualify)
        const int i = i0 + lane;
        uint64_t span = __ballot(len > 0 && incl > i0 && excl < i0 + kWave);
        int base = 0;
        while (span) {
          const int j = (int)__builtin_ctzll(span);
          span &= span - 1;
          const int ej = __builtin_amdgcn_readlane(excl, j);
          const int bj = __builtin_amdgcn_readlane(beg, j);
          base = ej <= i ? bj - ej : base;
        }
        if (i < total) hit(pts[base + i]);
      }
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const uint32_t* mr = mine + r * words;
      // hits in index order: lane l owns bitmask words [l*wpl, (l+1)*wpl)
      int pop = 0, myfirst = -1;
      for (int j = 0; j < wpl; ++j) {
        const int wi = lane * wpl + j;
        if (wi < words) {
          const uint32_t v = mr[wi];
          if (myfirst < 0 && v) myfirst = 32 * wi + __builtin_ctz(v);
          pop += __popc(v);
        }
      }
      const int incl = wave_incl_scan(pop, lane);
      const int total = __shfl(incl, kWave - 1, kWave);
      const int ns = rd.ns[r];
      const int cnt = min(total, ns);
      int32_t* __restrict__ row = rd.idx[r] + ((size_t)b * M + q) * ns;
      if constexpr (!FEAT) {
        // no features: each lane writes the rows of the hits it ranks (measured faster than
        // the hit list for 3-float rows: 22.1 vs 23.8 us at cfg2's SA1, profiles/r5/grp)
        float* __restrict__ grow = GROUP ? rd.gout[r] + ((size_t)b * M + q) * ns * 3 : nullptr;
        const float* __restrict__ X1 = GROUP ? xyz1 + (size_t)b * N * 3 : nullptr;
        int rank = incl - pop;
        for (int j = 0; j < wpl && rank < ns; ++j) {
          const int wi = lane * wpl + j;
          uint32_t v = wi < words ? mr[wi] : 0u;
          while (v && rank < ns) {
            const int k = 32 * wi + __builtin_ctz(v);
            if constexpr (GROUP) {
              grow[3 * rank + 0] = X1[3 * k + 0] - qx;  // pointnet_util.py:40
              grow[3 * rank + 1] = X1[3 * k + 1] - qy;
              grow[3 * rank + 2] = X1[3 * k + 2] - qz;
            }
            row[rank++] = k;
            v &= v - 1u;
          }
        }
        const uint64_t has = __ballot(pop > 0);
        const int first = has ? __shfl(myfirst, __ffsll((unsigned long long)has) - 1, kWave) : 0;
        for (int p = cnt + lane; p < ns; p += kWave) {
          row[p] = first;  // :26-29 (0 when no hit)
          if constexpr (GROUP) {
            grow[3 * p + 0] = X1[3 * first + 0] - qx;
            grow[3 * p + 1] = X1[3 * first + 1] - qy;
            grow[3 * p + 2] = X1[3 * first + 2] - qz;
          }
        }
      } else {
        int* lst = hl + r * rd.nsmax;
        int rank = incl - pop;
        for (int j = 0; j < wpl && rank < ns; ++j) {
          const int wi = lane * wpl + j;
          uint32_t v = wi < words ? mr[wi] : 0u;
          while (v && rank < ns) {
            lst[rank++] = 32 * wi + __builtin_ctz(v);
            v &= v - 1u;
          }
        }
        const uint64_t has = __ballot(pop > 0);
        const int first = has ? __shfl(myfirst, __ffsll((unsigned long long)has) - 1, kWave) : 0;
        for (int p = cnt + lane; p < ns; p += kWave) lst[p] = first;  // :26-29 (0 when no hit)
        // (one wave's DS operations execute in order: the reads below see every lane's writes)
        for (int p = lane; p < ns; p += kWave) row[p] = lst[p];
        {
          const int Cout = rd.cout, C = rd.C;
          const float* __restrict__ X1 = xyz1 + (size_t)b * N * 3;
          const float* __restrict__ F = C ? rd.points + (size_t)b * N * C : nullptr;
          float* __restrict__ out = rd.gout[r] + ((size_t)b * M + q) * ns * Cout;
          const int E = ns * Cout;
          // four elements' gathers in flight per lane before any is stored
          for (int e0 = lane; e0 < E; e0 += 4 * kWave) {
            float v[4], sub[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int e = min(e0 + u * kWave, E - 1);
              const int rr = (int)fdiv((uint32_t)e, rd.div_cout);
              const int c = e - rr * Cout;
              const int k = lst[rr];
              const int cx = c - rd.xoff;
              const bool isx = cx >= 0 && cx < 3;
              const float* src = isx ? X1 + 3 * k + cx : F + (size_t)k * C + (c - rd.foff);
              v[u] = *src;
              // a feature column subtracts +0.0f: x - 0 == x, bit for bit (-0.0 included)
              sub[u] = !isx ? 0.0f : cx == 0 ? qx : cx == 1 ? qy : qz;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int e = e0 + u * kWave;
              if (e < E) out[e] = v[u] - sub[u];  // pointnet_util.py:40
            }
          }
        }
      }
      if (lane == 0) rd.cnt[r][(size_t)b * M + q] = cnt;
    }
  }
}


// NR = 1 without features (cfg2's SA1: the query and its grouped xyz) with TWO queries per
// wave at once. One query per wave left each wave a chain of dependent memory trips per query
// (its centre, its rows' offsets, their points, the hits' coordinates), and with every wave of
// the launch resident at once the launch time was two such chains. Here the two queries' rows
// sit side by side in one 64-lane row list (query a's first), the walk takes the
// concatenation of all their points 64 at a time, each lane testing its point against its
// row's query into that query's bitmask, and the ranking runs lanes 0-31 over query a's
// bitmask and 32-63 over b's: one chain per pair. Same tests, same bitmasks, same ranks and
// rows as ball_query_grid_kernel. (cfg2's SA1: 21.0 -> 20.1 us standalone, tools/bench_side.py,
// profiles/r6/side: the chains were a smaller part of the launch than their count suggests.)
template <int BLOCK, bool GROUP>
__global__ __launch_bounds__(BLOCK) void ball_query_grid_pair_kernel(
    const char* __restrict__ grid, const float* __restrict__ xyz2, int N, int M, float radius,
    int qpb, int words, int gx, int nblk, const BqRadii rd, const float* __restrict__ xyz1) {
  constexpr int NW = BLOCK / kWave;
  constexpr int HALF = kWave / 2;
  extern __shared__ uint32_t bits[];  // NW x 2 x words: query a's bitmask, then b's
  const int lb = xcd_block((int)blockIdx.x, nblk);
  if (lb >= nblk) return;
  const int b = lb / gx, bx = lb - b * gx;
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const GridView g = grid_view(grid, b, N);
  const GridHdr& h = g.h;
  const int* __restrict__ off = g.off;
  const float4* __restrict__ pts = g.pts;
  uint32_t* const mine = bits + (size_t)w * 2 * words;
  const int hb = lane >= HALF ? 1 : 0, hl = lane - hb * HALF;  // ranking: half and its lane
  const int wph = (words + HALF - 1) / HALF;                    // bitmask words per lane of a half
  const float thresh = rd.thresh[0];
  const int ns = rd.ns[0];
  const int q_end = min(M, (bx + 1) * qpb);
  for (int qa = bx * qpb + 2 * w; qa < q_end; qa += 2 * NW) {
    const bool two = qa + 1 < q_end;
    for (int i = lane; i < 2 * words; i += kWave) mine[i] = 0u;
    const float* Qa = xyz2 + ((size_t)b * M + qa) * 3;
    const float* Qb = two ? Qa + 3 : Qa;
    const float ax = Qa[0], ay = Qa[1], az = Qa[2], bxq = Qb[0], byq = Qb[1], bzq = Qb[2];
    // each query's cell block (ball_query_grid_kernel's ranges)
    int x0[2], x1[2], y0[2], z0[2], nyr[2], nrows[2];
    {
      const float qc[2][3] = {{ax, ay, az}, {bxq, byq, bzq}};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float qx = qc[s][0], qy = qc[s][1], qz = qc[s][2];
        const float big = fmaxf(fmaxf(fmaxf(fabsf(qx), fabsf(qy)), fmaxf(fabsf(qz), radius)), 1.0f);
        const float rr = radius + big * 1e-5f;
        x0[s] = cell_coord(qx - rr, h.ox, h.inv, h.nx);
        x1[s] = cell_coord(qx + rr, h.ox, h.inv, h.nx);
        y0[s] = cell_coord(qy - rr, h.oy, h.inv, h.ny);
        const int y1 = cell_coord(qy + rr, h.oy, h.inv, h.ny);
        z0[s] = cell_coord(qz - rr, h.oz, h.inv, h.nz);
        const int z1 = cell_coord(qz + rr, h.oz, h.inv, h.nz);
        nyr[s] = y1 - y0[s] + 1;
        nrows[s] = s == 1 && !two ? 0 : (z1 - z0[s] + 1) * nyr[s];
      }
    }
    const int R = nrows[0] + nrows[1];
    for (int r0 = 0; r0 < R; r0 += kWave) {
      // lane j: row r0 + j of the pair's list (query a's rows, then b's)
      int beg = 0, len = 0;
      const int r = r0 + lane;
      const bool rb = r >= nrows[0];
      if (r < R) {
        const int s = rb ? 1 : 0, rq = rb ? r - nrows[0] : r;
        const int zr = rq / nyr[s];
        const int row = ((z0[s] + zr) * h.ny + y0[s] + (rq - zr * nyr[s])) * h.nx;
        beg = off[row + x0[s]];
        len = off[row + x1[s] + 1] - beg;
      }
      const uint64_t rowb = __ballot(rb);  // rows of query b (by lane)
      const int incl = wave_incl_scan(len, lane);
      const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
      const int excl = incl - len;
      for (int i0 = 0; i0 < total; i0 += kWave) {
        // the rows overlapping [i0, i0 + 64): each lane takes the last one starting at or
        // before its position, and that row's query
        const int i = i0 + lane;
        uint64_t span = __ballot(len > 0 && incl > i0 && excl < i0 + kWave);
        int base = 0;
        bool qb = false;
        while (span) {
          const int j = (int)__builtin_ctzll(span);
          span &= span - 1;
          const int ej = __builtin_amdgcn_readlane(excl, j);
          const int bj = __builtin_amdgcn_readlane(beg, j);
          const bool sel = ej <= i;
          base = sel ? bj - ej : base;
          qb = sel ? ((rowb >> j) & 1ull) != 0 : qb;
        }
        if (i < total) {  // tf_grouping_g.cu:24-25
          const float4 p = pts[base + i];
          const float d = qb ? sqdist(bxq, byq, bzq, p.x, p.y, p.z) : sqdist(ax, ay, az, p.x, p.y, p.z);
          const int k = __float_as_int(p.w);
          if (d < thresh) atomicOr(&mine[(qb ? words : 0) + (k >> 5)], 1u << (k & 31));
        }
      }
    }
    // ranking: lanes 0-31 own query a's bitmask words [hl*wph, (hl+1)*wph), lanes 32-63 b's
    const uint32_t* mr = mine + hb * words;
    int pop = 0, myfirst = -1;
    for (int j = 0; j < wph; ++j) {
      const int wi = hl * wph + j;
      if (wi < words) {
        const uint32_t v = mr[wi];
        if (myfirst < 0 && v) myfirst = 32 * wi + __builtin_ctz(v);
        pop += __popc(v);
      }
    }
    const int incl = wave_incl_scan(pop, lane);
    const int tot_a = __builtin_amdgcn_readlane(incl, HALF - 1);
    const int tot_b = __builtin_amdgcn_readlane(incl, kWave - 1) - tot_a;
    const int total = hb ? tot_b : tot_a;
    const int cnt = min(total, ns);
    const int q = qa + hb;
    const bool mineq = hb == 0 || two;
    const float qx = hb ? bxq : ax, qy = hb ? byq : ay, qz = hb ? bzq : az;
    int32_t* __restrict__ row = rd.idx[0] + ((size_t)b * M + q) * ns;
    float* __restrict__ grow = GROUP ? rd.gout[0] + ((size_t)b * M + q) * ns * 3 : nullptr;
    const float* __restrict__ X1 = GROUP ? xyz1 + (size_t)b * N * 3 : nullptr;
    int rank = incl - pop - (hb ? tot_a : 0);
    if (mineq) {
      for (int j = 0; j < wph && rank < ns; ++j) {
        const int wi = hl * wph + j;
        uint32_t v = wi < words ? mr[wi] : 0u;
        while (v && rank < ns) {
          const int k = 32 * wi + __builtin_ctz(v);
          if constexpr (GROUP) {
            grow[3 * rank + 0] = X1[3 * k + 0] - qx;  // pointnet_util.py:40
            grow[3 * rank + 1] = X1[3 * k + 1] - qy;
            grow[3 * rank + 2] = X1[3 * k + 2] - qz;
          }
          row[rank++] = k;
          v &= v - 1u;
        }
      }
    }
    const uint64_t has = __ballot(pop > 0);
    const uint64_t hma = has & 0xFFFFFFFFull, hmb = has >> HALF;
    const int fa = hma ? __builtin_amdgcn_readlane(myfirst, (int)__builtin_ctzll(hma)) : 0;
    const int fbl = hmb ? (int)__builtin_ctzll(hmb) + HALF : 0;
    const int fb = hmb ? __builtin_amdgcn_readlane(myfirst, fbl) : 0;
    const int first = hb ? fb : fa;
    if (mineq) {
      for (int p = cnt + hl; p < ns; p += HALF) {
        row[p] = first;  // :26-29 (0 when no hit)
        if constexpr (GROUP) {
          grow[3 * p + 0] = X1[3 * first + 0] - qx;
          grow[3 * p + 1] = X1[3 * first + 1] - qy;
          grow[3 * p + 2] = X1[3 * first + 2] - qz;
        }
      }
      if (hl == 0) rd.cnt[0][(size_t)b * M + q] = cnt;
    }
  }
}

}  // namespace
}  // namespace pn2

extern "C" {

float pn2_ball_threshold(float radius);

size_t pn2_grid_size(int B, int N) {
  if (B <= 0 || N < 0) return 0;
  return (size_t)B * pn2::grid_stride(N);
}

int pn2_grid_build(const float* xyz, int B, int N, float cell_edge, void* grid,
                   size_t grid_bytes, pn2_stream_t stream) {
  if (B < 0 || N < 0 || cell_edge != cell_edge) return PN2_EINVAL;
  if (B == 0) return PN2_OK;
  if (!grid || grid_bytes < pn2_grid_size(B, N) || (N > 0 && !xyz)) return PN2_EINVAL;
  if ((uintptr_t)grid % 16 || B > 65535) return PN2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  char* g = (char*)grid;
  const dim3 grd(B);
  // (dynamic LDS up to the full kGridCap array, 128 KB: opted into once per instantiation)
  static const hipError_t attr = [] {
    hipError_t e = hipSuccess;
    auto opt = [&](const void* f) {
      const hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)(pn2::kGridCap * 4));
      if (r != hipSuccess) e = r;
    };
    opt(reinterpret_cast<const void*>(&pn2::grid_build_kernel<0, 256>));
    opt(reinterpret_cast<const void*>(&pn2::grid_build_kernel<2, 256>));
    opt(reinterpret_cast<const void*>(&pn2::grid_build_kernel<4, 256>));
    opt(reinterpret_cast<const void*>(&pn2::grid_build_kernel<8, 256>));
    opt(reinterpret_cast<const void*>(&pn2::grid_build_kernel<2, pn2::kBuildBlock>));
    opt(reinterpret_cast<const void*>(&pn2::grid_build_kernel<4, pn2::kBuildBlock>));
    opt(reinterpret_cast<const void*>(&pn2::grid_build_kernel<8, pn2::kBuildBlock>));
    opt(reinterpret_cast<const void*>(&pn2::grid_build_kernel<pn2::kBuildMaxPpt, pn2::kBuildBlock>));
    opt(reinterpret_cast<const void*>(&pn2::grid_build_kernel<0, pn2::kBuildBlock>));
    return e;
  }();
  if (attr != hipSuccess) return (int)attr;
  // the count array's words (grid_build_kernel): what the grid's cells can number
  const bool loop = N > pn2::kBuildBlock * pn2::kBuildMaxPpt;
  const int cap = loop ? pn2::kGridCap
                       : (cell_edge > 0.0f ? pn2::kBuildCapEdge : std::max(N, pn2::kAutoMinCells));
  const size_t lds = (size_t)cap * 4;
#define PN2_GB(PPT, BLK) \
  hipLaunchKernelGGL((pn2::grid_build_kernel<PPT, BLK>), grd, dim3(BLK), lds, s, xyz, N, cell_edge, g, cap)
  if (N <= pn2::kBuildSmallN) {  // 256 threads: PPT <= 8
    const int ppt = (N + 255) / 256;
    if (N == 0) PN2_GB(0, 256);
    else if (ppt <= 2) PN2_GB(2, 256);
    else if (ppt <= 4) PN2_GB(4, 256);
    else PN2_GB(8, 256);
  } else {
    const int ppt = (N + pn2::kBuildBlock - 1) / pn2::kBuildBlock;
    if (ppt <= 2) PN2_GB(2, pn2::kBuildBlock);
    else if (ppt <= 4) PN2_GB(4, pn2::kBuildBlock);
    else if (ppt <= 8) PN2_GB(8, pn2::kBuildBlock);
    else if (ppt <= pn2::kBuildMaxPpt) PN2_GB(pn2::kBuildMaxPpt, pn2::kBuildBlock);
    else PN2_GB(0, pn2::kBuildBlock);
  }
#undef PN2_GB
  PN2_RETURN_LAUNCH();
}

namespace {
// nr radii (1..PN2_BQ_MAX_RADII) in one launch; gout[r] all set (GROUP) or all NULL; GROUP
// rows: [xyz1[idx] - xyz2, points[idx]] (xyz_last: [points, xyz]) of C + 3 columns
int ball_query_grid(const void* grid, const float* xyz2, int B, int N, int M, int nr,
                    const float* radii, const int* nsample, int32_t* const* idx,
                    int32_t* const* pts_cnt, const float* xyz1, float* const* gout,
                    hipStream_t stream, const float* points = nullptr, int C = 0,
                    bool xyz_last = false) {
  if (nr < 1 || nr > PN2_BQ_MAX_RADII || B < 0 || N < 0 || M < 0) return PN2_EINVAL;
  for (int r = 0; r < nr; ++r)
    if (!(radii[r] > 0.0f) || nsample[r] <= 0) return PN2_EINVAL;
  if ((long long)B * M == 0) return PN2_OK;
  if (!grid || !xyz2 || B > 65535) return PN2_EINVAL;
  const bool group = gout != nullptr;
  if (group && !xyz1) return PN2_EINVAL;
  if (C < 0 || (C > 0 && (!group || !points)) || C > 4096) return PN2_EINVAL;
  pn2::BqRadii rd{};
  float rmax = 0.0f;
  int nsmax = 1;
  for (int r = 0; r < nr; ++r) {
    if (!idx[r] || !pts_cnt[r] || (group && !gout[r])) return PN2_EINVAL;
    rd.thresh[r] = pn2_ball_threshold(radii[r]);
    rd.ns[r] = nsample[r];
    rd.idx[r] = idx[r];
    rd.cnt[r] = pts_cnt[r];
    rd.gout[r] = group ? gout[r] : nullptr;
    rmax = std::max(rmax, radii[r]);
    nsmax = std::max(nsmax, nsample[r]);
  }
  rd.points = C ? points : nullptr;
  rd.C = C;
  rd.cout = C + 3;
  rd.xoff = xyz_last ? C : 0;
  rd.foff = xyz_last ? 0 : 3;
  rd.div_cout = pn2::make_fastdiv((uint32_t)rd.cout);
  rd.nsmax = nsmax;
  // the 32-bit element arithmetic of a query's rows (fdiv: e * Cout < 2^32)
  if ((long long)nsmax * rd.cout * rd.cout >= (1LL << 32)) return PN2_EINVAL;
  const int words = (N + 31) / 32;
  if (words > pn2::kMaxBitWords) return PN2_EINVAL;
  constexpr int BLOCK = 256, NW = BLOCK / pn2::kWave;
  // ~2048 workgroups over the batch, a whole number of queries per wave
  const long long queries = (long long)B * M;
  long long qpb = (queries + 2047) / 2048;
  qpb = ((qpb + NW - 1) / NW) * NW;
  const unsigned gx = (unsigned)((M + qpb - 1) / qpb);
  const size_t lds = (size_t)NW * nr * ((words > 0 ? words : 1) + (C > 0 ? nsmax : 0)) * 4;
  if (lds > 64 * 1024) return PN2_EINVAL;  // (dynamic LDS; nr = 1 fits up to N ~ 130000)
  const long long nblk = (long long)gx * B;
  if (nblk > INT32_MAX - pn2::kXcds) return PN2_EINVAL;
  const dim3 grd(pn2::xcd_grid(nblk)), blk(BLOCK);
  const char* g = (const char*)grid;
#define PN2_BQG(GROUP, NR)                                                                     \
  hipLaunchKernelGGL((pn2::ball_query_grid_kernel<BLOCK, GROUP, NR>), grd, blk, lds, stream, g, \
                     xyz2, N, M, rmax, (int)qpb, words, (int)gx, (int)nblk, rd,               \
                     GROUP ? xyz1 : nullptr)
  if (C > 0) {  // features: the hit-list output phase (one radius per launch)
    if (nr != 1) return PN2_EINVAL;
    hipLaunchKernelGGL((pn2::ball_query_grid_kernel<BLOCK, true, 1, true>), grd, blk, lds, stream,
                       g, xyz2, N, M, rmax, (int)qpb, words, (int)gx, (int)nblk, rd, xyz1);
  } else if (nr == 1 && 2 * lds <= 64 * 1024) {
    // two queries per wave (ball_query_grid_pair_kernel): a workgroup's queries a whole number
    // of pairs per wave
    const long long qpb2 = ((qpb + 2 * NW - 1) / (2 * NW)) * (2 * NW);
    const unsigned gx2 = (unsigned)((M + qpb2 - 1) / qpb2);
    const long long nblk2 = (long long)gx2 * B;
    const dim3 grd2(pn2::xcd_grid(nblk2));
    if (group)
      hipLaunchKernelGGL((pn2::ball_query_grid_pair_kernel<BLOCK, true>), grd2, blk, 2 * lds,
                         stream, g, xyz2, N, M, rmax, (int)qpb2, words, (int)gx2, (int)nblk2, rd,
                         xyz1);
    else
      hipLaunchKernelGGL((pn2::ball_query_grid_pair_kernel<BLOCK, false>), grd2, blk, 2 * lds,
                         stream, g, xyz2, N, M, rmax, (int)qpb2, words, (int)gx2, (int)nblk2, rd,
                         nullptr);
  } else if (group) {
    if (nr == 1) PN2_BQG(true, 1);
    else if (nr == 2) PN2_BQG(true, 2);
    else PN2_BQG(true, 3);
  } else {
    if (nr == 1) PN2_BQG(false, 1);
    else if (nr == 2) PN2_BQG(false, 2);
    else PN2_BQG(false, 3);
  }
#undef PN2_BQG
  PN2_RETURN_LAUNCH();
}
}  // namespace

int pn2_ball_query_grid(const void* grid, const float* xyz2, int B, int N, int M, float radius,
                        int nsample, int32_t* idx, int32_t* pts_cnt, pn2_stream_t stream) {
  if (!idx || !pts_cnt) return PN2_EINVAL;
  return ball_query_grid(grid, xyz2, B, N, M, 1, &radius, &nsample, &idx, &pts_cnt, nullptr,
                         nullptr, (hipStream_t)stream);
}

int pn2_ball_group_xyz_grid(const void* grid, const float* xyz1, const float* xyz2, int B, int N,
                            int M, float radius, int nsample, int32_t* idx, int32_t* pts_cnt,
                            float* grouped_xyz, pn2_stream_t stream) {
  if (!grouped_xyz || !idx || !pts_cnt) return PN2_EINVAL;
  return ball_query_grid(grid, xyz2, B, N, M, 1, &radius, &nsample, &idx, &pts_cnt, xyz1,
                         &grouped_xyz, (hipStream_t)stream);
}

int pn2_ball_group_grid(const void* grid, const float* xyz1, const float* points, int C,
                        int flags, const float* xyz2, int B, int N, int M, float radius,
                        int nsample, int32_t* idx, int32_t* pts_cnt, float* new_points,
                        pn2_stream_t stream) {
  if (!new_points || !idx || !pts_cnt || C < 0 || (C > 0 && !points)) return PN2_EINVAL;
  if (C > 0 && !(flags & PN2_USE_XYZ)) return PN2_EINVAL;  // (points only: pn2_group_point)
  return ball_query_grid(grid, xyz2, B, N, M, 1, &radius, &nsample, &idx, &pts_cnt, xyz1,
                         &new_points, (hipStream_t)stream, points, C, (flags & PN2_XYZ_LAST) != 0);
}

int pn2_ball_group_xyz_grid_radii(const void* grid, const float* xyz1, const float* xyz2, int B,
                                  int N, int M, int nr, const float* radii, const int* nsample,
                                  int32_t* const* idx, int32_t* const* pts_cnt,
                                  float* const* grouped_xyz, pn2_stream_t stream) {
  if (!radii || !nsample || !idx || !pts_cnt || !grouped_xyz) return PN2_EINVAL;
  if (nr < 1 || nr > PN2_BQ_MAX_RADII) return PN2_EINVAL;
  return ball_query_grid(grid, xyz2, B, N, M, nr, radii, nsample, idx, pts_cnt, xyz1,
                         grouped_xyz, (hipStream_t)stream);
}

}  // extern "C"
