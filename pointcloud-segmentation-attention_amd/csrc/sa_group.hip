// Ball query + fused group/centre/concat of SEVERAL set-abstraction layers in ONE launch.
//
// Per layer the result is exactly pn2_ball_query followed by pn2_group_concat
// (tf_grouping_g.cu:3-36 then :40-57 and pointnet_util.py:39-56 / :186-193): the same
// membership test (d2 < T with T = pn2_ball_threshold(radius), tf_grouping_g.cu:24-25), the
// first nsample hits in index order, empty slots repeating the first hit (:26-29),
// pts_cnt = hits capped at nsample (:34), and the grouped rows xyz[idx] - new_xyz (one fp32
// subtraction, pointnet_util.py:40) concatenated with points[idx].
//
// Why one kernel: SA2..SA4 of the SSG stack (and the MSG radii of a level) all wait for the
// same sampler and each is a small launch (5-20 us). As two launches per layer they were six
// back-to-back kernels on one side lane, each paying a launch gap; here they are one grid.
// Fusing the query with the grouping also drops the idx round trip: the wave that found a
// query's neighbours writes that query's grouped rows from the hits it holds in LDS, reading
// neighbour coordinates from the LDS copy of the cloud it just scanned.
//
// Layout: workgroup = (cloud, layer, tile of queries), 4 waves. The cloud's xyz (N <= kSgCap
// points) is staged in LDS as SoA; one wave per query scans it into an LDS hit row. The tile's
// grouped rows are one contiguous output range, streamed by the whole workgroup with four
// elements' gathers in flight per thread (they hit L2: a cloud's feature rows are shared by
// its tiles, which the cloud-major XCD-aware order keeps on one XCD).
#include "common.h"

namespace pn2 {
namespace {

constexpr int kSgBlock = 256;
constexpr int kSgWaves = kSgBlock / kWave;
constexpr int kSgCap = 1024;    // points per cloud staged in LDS
constexpr int kSgMaxNs = 128;   // nsample
constexpr int kSgUnroll = 4;    // 64-point steps per scan iteration
constexpr int kSgHits = 2048;   // hit slots per workgroup: qpb * nsample
constexpr int kSgMaxQpb = 64;   // queries per workgroup
// measured on MI355X (tools/bench_layers.py, profiles/r3/sgs, r4/pf): output bytes per
// workgroup, the split of a query of many channels, gathers in flight per thread
constexpr int kSgTileKB = 32;      // output per workgroup over whole queries
constexpr int kSgSplitKB = 24;     // a query above this is split over workgroups ...
constexpr int kSgSplitStage = 4096;  // ... when its cloud stages in this many LDS bytes
constexpr int kSgU = 4;            // elements whose gathers are in flight per thread
constexpr int kSgVecFloats = 4096;  // the vector write phase's LDS staging chunk (16 KB)

enum SgLayout : int {
  PN2_SG_POINTS_ONLY = 0,  // out = points[idx]                       (Cout = C)
  PN2_SG_XYZ_ONLY = 1,     // out = xyz[idx] - new_xyz                (Cout = 3)
  PN2_SG_XYZ_FIRST = 2,    // out = [xyz[idx] - new_xyz, points[idx]] (Cout = 3 + C)
  PN2_SG_XYZ_LAST = 3,     // out = [points[idx], xyz[idx] - new_xyz] (Cout = C + 3)
};

struct SgLayer {
  const float* xyz;
  const float* points;
  const float* new_xyz;
  int32_t* idx;
  int32_t* cnt;
  float* grouped_xyz;
  float* out;
  int N, C, M, ns, Cout, layout, qpb, tiles;  // workgroups per cloud = tiles * parts
  int parts, chunk;  // a query split over `parts` workgroups of `chunk` elements each
  int vec;           // the vector write phase applies (host-checked)
  float thresh;
  FastDiv div_cout, div_ns, div_c4;
};

struct SgArgs {
  SgLayer l[PN2_SA_MAX_LAYERS];
  int first[PN2_SA_MAX_LAYERS + 1];  // first block of each layer within a cloud's range
  int nlayers, B;
};

// out element c of a grouped row: xyz channel (>= 0) or -1 for a feature channel, and the
// feature channel (SSG [xyz, points], MSG [points, xyz], xyz only, points only)
PN2_DEV int xyz_channel(int layout, int c, int C, int& cp) {
  cp = c;
  if (layout == PN2_SG_XYZ_ONLY) return c;
  if (layout == PN2_SG_XYZ_FIRST) {
    if (c < 3) return c;
    cp = c - 3;
    return -1;
  }
  if (layout == PN2_SG_XYZ_LAST) return c >= C ? c - C : -1;
  return -1;
}

__global__ __launch_bounds__(kSgBlock) void ball_group_layers_kernel(SgArgs a) {
  __shared__ float sx[kSgCap], sy[kSgCap], sz[kSgCap];
  __shared__ int s_hit[kSgHits];          // the tile's rows: query qi's hits at qi*ns ..
  __shared__ float s_q[3 * kSgMaxQpb];    // the tile's query centres
  // vector phase: the chunk image, dynamic LDS sized by the host -- 16 KB when some layer of
  // the launch has the vector phase, none otherwise (the scalar-only launches keep their
  // occupancy)
  extern __shared__ float4 s_out4[];
  // logical blocks cloud-major: cloud b's blocks of every layer are one contiguous range, so
  // the XCD-aware order gives each XCD whole clouds (their rows in one L2) and every XCD the
  // same mix of layers
  const int per_cloud_all = a.first[a.nlayers];
  const int total = per_cloud_all * a.B;
  const int L = xcd_block((int)blockIdx.x, total);
  if (L >= total) return;  // padding blocks (before any barrier)
  const int b = L / per_cloud_all;
  const int lc = L - b * per_cloud_all;
  int li = 0;
  while (li + 1 < a.nlayers && lc >= a.first[li + 1]) ++li;
  const SgLayer& g = a.l[li];
  const int local = lc - a.first[li];
  const int tile = local / g.parts;
  const int part = local - tile * g.parts;
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const int N = g.N, C = g.C, M = g.M, ns = g.ns, Cout = g.Cout, layout = g.layout;
  const int q0 = tile * g.qpb, nq = min(g.qpb, M - q0);
  const float* __restrict__ P = g.xyz + (size_t)b * N * 3;
  for (int e = t; e < N; e += kSgBlock) {
    sx[e] = P[3 * e + 0];
    sy[e] = P[3 * e + 1];
    sz[e] = P[3 * e + 2];
  }
  const float* __restrict__ Q = g.new_xyz + ((size_t)b * M + q0) * 3;
  for (int e = t; e < 3 * nq; e += kSgBlock) s_q[e] = Q[e];
  __syncthreads();
  // ---- phase 1: one wave per query, the ball query (tf_grouping_g.cu:15-33) into s_hit
  const uint64_t lower = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int qi = w; qi < nq; qi += kSgWaves) {
    const float qx = s_q[3 * qi + 0], qy = s_q[3 * qi + 1], qz = s_q[3 * qi + 2];
    int* hit = s_hit + qi * ns;
    int cnt = 0, first = 0;
    for (int base = 0; base < N && cnt < ns; base += kWave * kSgUnroll) {
      bool h[kSgUnroll];
#pragma unroll
      for (int u = 0; u < kSgUnroll; ++u) {
        const int k = base + u * kWave + lane;
        h[u] = k < N && sqdist(qx, qy, qz, sx[k], sy[k], sz[k]) < g.thresh;
      }
#pragma unroll
      for (int u = 0; u < kSgUnroll; ++u) {
        const uint64_t mask = __ballot(h[u]);
        if (mask != 0ull && cnt < ns) {
          if (cnt == 0) first = base + u * kWave + (__ffsll((unsigned long long)mask) - 1);
          const int pos = cnt + __popcll(mask & lower);
          if (h[u] && pos < ns) hit[pos] = base + u * kWave + lane;
          cnt += __popcll(mask);
        }
      }
    }
    if (cnt > ns) cnt = ns;
    // the hits other lanes of this wave wrote are visible before the fill reads them
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const size_t gq = (size_t)b * M + q0 + qi;
    int32_t* __restrict__ row = g.idx + gq * ns;
    for (int p = lane; p < ns; p += kWave) {
      const int v = p < cnt ? hit[p] : first;  // :26-29 (0 when no hit)
      hit[p] = v;
      if (part == 0) row[p] = v;
    }
    if (lane == 0 && part == 0) g.cnt[gq] = cnt;
  }
  __syncthreads();
  // ---- phase 2: the tile's grouped rows (nq * ns rows of Cout floats) are ONE contiguous
  // range of the output: the whole workgroup streams it, one float per lane per element and
  // four elements' loads in flight before any store (16-byte stores and loads of four
  // channels measured 3 % slower: profiles/r3/sgs)
  const size_t r_base = ((size_t)b * M + q0) * ns;  // first output row of the tile
  float* __restrict__ O = g.out + r_base * Cout;
  float* __restrict__ GX = g.grouped_xyz ? g.grouped_xyz + r_base * 3 : nullptr;
  const float* __restrict__ F = g.points ? g.points + (size_t)b * N * C : nullptr;
  if (g.vec) {
    {
      // ---- phase 2, vector form: the tile's rows go out in chunks of CH rows through LDS.
      // Feature columns are gathered as float4 (a points row is 16-B aligned: C % 4 == 0) and
      // the xyz columns computed from the LDS cloud copy, both into the chunk's row-major
      // image; then the chunk leaves as aligned float4 stores (CH, the tile's first row and
      // ns are multiples of 4, so every chunk starts on a 16-B boundary of the output). One
      // gather round trip per chunk instead of one per four elements of each thread.
      float* s_out = reinterpret_cast<float*>(s_out4);
      const int C4 = C >> 2;
      const int foff = layout == PN2_SG_XYZ_FIRST ? 3 : 0;  // first feature column
      const int xoff = layout == PN2_SG_XYZ_LAST ? C : 0;   // first xyz column
      const bool has_xyz = layout != PN2_SG_POINTS_ONLY;
      const int CH = (kSgVecFloats / Cout) & ~3;  // >= 4 (host: Cout <= kSgVecFloats / 4)
      // this workgroup's rows of the tile: all, or part `part` of a query split over
      // g.parts workgroups (row ranges of a multiple of 4 rows)
      const int R = nq * ns;
      const int RP = (((R + g.parts - 1) / g.parts) + 3) & ~3;
      const int rbeg = part * RP, rend = min(R, rbeg + RP);
      const float4* __restrict__ F4 = reinterpret_cast<const float4*>(F);
      constexpr int UV = 4;
      float4 v[UV];
      int dst[UV];
      // the gathers of chunk c0 (its rows' feature float4s) into v / dst, issued, not waited for
      auto gather = [&](int c0, int f0) {
        const int nf = min(CH, rend - c0) * C4;
#pragma unroll
        for (int u = 0; u < UV; ++u) {
          const int f = min(f0 + u * kSgBlock, nf - 1);  // (a surplus lane reloads the last)
          const int rr = (int)fdiv((uint32_t)f, g.div_c4);
          const int cc = f - rr * C4;
          v[u] = F4[(size_t)s_hit[c0 + rr] * C4 + cc];
          dst[u] = rr * Cout + foff + 4 * cc;
        }
      };
      // prefetch: a chunk that one pass of UV float4s per thread covers has its
      // successor's gathers issued before its own stores, so the gather round trip overlaps
      // the store phase instead of following it
      const bool one_pass = CH * C4 <= kSgBlock * UV;
      if (one_pass && rbeg < rend) gather(rbeg, t);
      for (int c0 = rbeg; c0 < rend; c0 += CH) {
        const int nr = min(CH, rend - c0);
        const int nf = nr * C4;
        for (int f0 = t; f0 < nf; f0 += kSgBlock * UV) {
          if (!one_pass) gather(c0, f0);
#pragma unroll
          for (int u = 0; u < UV; ++u) {
            if (f0 + u * kSgBlock < nf) {
              s_out[dst[u]] = v[u].x;
              s_out[dst[u] + 1] = v[u].y;
              s_out[dst[u] + 2] = v[u].z;
              s_out[dst[u] + 3] = v[u].w;
            }
          }
        }
        if (has_xyz) {
          for (int e = t; e < nr * 3; e += kSgBlock) {
            const int rr = e / 3, cx = e - 3 * rr;
            const int r = c0 + rr;
            const int qi = (int)fdiv((uint32_t)r, g.div_ns);
            const int i = s_hit[r];
            const float sv = cx == 0 ? sx[i] : (cx == 1 ? sy[i] : sz[i]);
            s_out[rr * Cout + xoff + cx] = sv - s_q[3 * qi + cx];  // pointnet_util.py:40
          }
        }
        __syncthreads();
        if (one_pass && c0 + CH < rend) gather(c0 + CH, t);
        float4* __restrict__ O4 = reinterpret_cast<float4*>(O + (size_t)c0 * Cout);
        const int n4 = (nr * Cout) >> 2;  // nr % 4 == 0 (R, RP and CH are multiples of 4)
        for (int k = t; k < n4; k += kSgBlock) O4[k] = s_out4[k];
        __syncthreads();  // the image is free for the next chunk
      }
      return;
    }
  }
  // this workgroup's elements of the tile: all, or part `part` of a split query
  const int e_beg = part * g.chunk;
  const int E = min(nq * ns * Cout, e_beg + g.chunk);
  auto value = [&](int e) -> float {
    const int r = (int)fdiv((uint32_t)e, g.div_cout);  // row of the tile
    const int c = e - r * Cout;
    const int qi = (int)fdiv((uint32_t)r, g.div_ns);
    const int i = s_hit[r];
    int cp;
    const int cx = xyz_channel(layout, c, C, cp);
    if (cx >= 0) {
      const float s = cx == 0 ? sx[i] : (cx == 1 ? sy[i] : sz[i]);
      const float v = s - s_q[3 * qi + cx];  // pointnet_util.py:40
      if (GX) GX[(size_t)r * 3 + cx] = v;
      return v;
    }
    return F[(size_t)i * C + cp];
  };
  constexpr int U = kSgU;
  for (int e0 = e_beg + t; e0 < E; e0 += kSgBlock * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * kSgBlock;
      v[u] = e < E ? value(e) : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * kSgBlock;
      if (e < E) O[e] = v[u];
    }
  }
  // points-only rows carry no xyz channel: grouped_xyz (still an output of sample_and_group,
  // pointnet_util.py:58) gets its own pass over the tile, by the query's first part
  if (GX && layout == PN2_SG_POINTS_ONLY && part == 0) {
    for (int e = t; e < nq * ns * 3; e += kSgBlock) {
      const int r = e / 3, cx = e - 3 * (e / 3);
      const int qi = (int)fdiv((uint32_t)r, g.div_ns);
      const int i = s_hit[r];
      const float s = cx == 0 ? sx[i] : (cx == 1 ? sy[i] : sz[i]);
      GX[e] = s - s_q[3 * qi + cx];  // pointnet_util.py:40
    }
  }
}

}  // namespace
}  // namespace pn2

extern "C" {

int pn2_ball_group_layers(const pn2_sa_layer* layers, int nlayers, int B, pn2_stream_t stream) {
  if (!layers || nlayers < 1 || nlayers > PN2_SA_MAX_LAYERS || B < 0 || B > 65535)
    return PN2_EINVAL;
  pn2::SgArgs a{};
  a.nlayers = nlayers;
  long long blocks = 0;
  for (int i = 0; i < nlayers; ++i) {
    const pn2_sa_layer& s = layers[i];
    pn2::SgLayer& g = a.l[i];
    if (!(s.radius > 0.0f) || s.nsample <= 0 || s.nsample > pn2::kSgMaxNs || s.N < 0 ||
        s.N > pn2::kSgCap || s.M < 0 || s.C < 0)
      return PN2_EINVAL;
    using namespace pn2;
    int layout, Cout;
    if (!s.points || s.C == 0) { layout = PN2_SG_XYZ_ONLY; Cout = 3; }
    else if (!(s.flags & PN2_USE_XYZ)) { layout = PN2_SG_POINTS_ONLY; Cout = s.C; }
    else { layout = (s.flags & PN2_XYZ_LAST) ? PN2_SG_XYZ_LAST : PN2_SG_XYZ_FIRST; Cout = s.C + 3; }
    if ((long long)B * s.M > 0) {
      if (!s.xyz || !s.new_xyz || !s.idx || !s.pts_cnt || !s.new_points) return PN2_EINVAL;
      if (s.N == 0) return PN2_EINVAL;  // nothing to group from
    }
    g.xyz = s.xyz;
    g.points = layout == PN2_SG_XYZ_ONLY ? nullptr : s.points;
    g.new_xyz = s.new_xyz;
    g.idx = s.idx;
    g.cnt = s.pts_cnt;
    g.grouped_xyz = s.grouped_xyz;  // written in every layout (= out when xyz-only)
    g.out = s.new_points;
    g.N = s.N; g.C = layout == PN2_SG_XYZ_ONLY ? 0 : s.C; g.M = s.M; g.ns = s.nsample;
    g.Cout = Cout; g.layout = layout;
    g.thresh = pn2_ball_threshold(s.radius);
    g.div_cout = pn2::make_fastdiv((uint32_t)Cout);
    // work per workgroup: ~kSgTileKB of output over whole queries; a query of many
    // channels on a small cloud (cheap to stage and scan again) is split over several
    // workgroups of ~kSgSplitKB each, so the grid has enough waves to hide the gathers
    const long long per_q = (long long)s.nsample * Cout * 4;
    long long qpb = (kSgTileKB * 1024 + per_q / 2) / per_q;
    if (qpb < 1) qpb = 1;
    if (qpb > pn2::kSgMaxQpb) qpb = pn2::kSgMaxQpb;
    if (qpb * s.nsample > pn2::kSgHits) qpb = pn2::kSgHits / s.nsample;
    long long parts = 1;
    if (s.N * 12 <= kSgSplitStage && per_q > kSgSplitKB * 1024) {
      qpb = 1;
      parts = (per_q + kSgSplitKB * 1024 - 1) / (kSgSplitKB * 1024);
    }
    const long long E = qpb * s.nsample * Cout;
    g.chunk = (int)(((E + parts - 1) / parts + 3) / 4 * 4);
    g.parts = (int)((E + g.chunk - 1) / g.chunk);
    // 32-bit FastDiv of tile elements by Cout and of tile rows by nsample stays exact
    if (E * (long long)Cout >= (1LL << 32)) return PN2_EINVAL;
    g.qpb = (int)qpb;
    g.div_ns = pn2::make_fastdiv((uint32_t)s.nsample);
    g.tiles = s.M > 0 ? (int)((s.M + qpb - 1) / qpb) : 0;
    // the vector write phase: float4 feature rows, whole queries per
    // workgroup, 16-B aligned buffers, ns % 4 == 0 (chunks start on 16-B boundaries), no
    // grouped_xyz output, at least 4 rows per LDS chunk
    g.div_c4 = pn2::make_fastdiv((uint32_t)(s.C / 4 > 0 ? s.C / 4 : 1));
    g.vec = layout != PN2_SG_XYZ_ONLY && s.C % 4 == 0 && s.nsample % 4 == 0 &&
            !s.grouped_xyz && 4 * Cout <= pn2::kSgVecFloats &&
            (((uintptr_t)s.points | (uintptr_t)s.new_points) & 15) == 0;
    a.first[i] = (int)blocks;
    blocks += (long long)g.tiles * g.parts;  // per cloud
    if (blocks * B >= (1LL << 31) - 8) return PN2_EINVAL;
  }
  a.first[nlayers] = (int)blocks;
  a.B = B;
  if (blocks * B == 0) return PN2_OK;
  bool vec = false;
  for (int i = 0; i < nlayers; ++i) vec = vec || a.l[i].vec;
  const size_t lds = vec ? (size_t)pn2::kSgVecFloats * 4 : 0;
  hipLaunchKernelGGL(pn2::ball_group_layers_kernel, dim3(pn2::xcd_grid(blocks * B)),
                     dim3(pn2::kSgBlock), lds, (hipStream_t)stream, a);
  PN2_RETURN_LAUNCH();
}

}  // extern "C"
