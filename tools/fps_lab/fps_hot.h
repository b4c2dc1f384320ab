// Hot-set farthest-point sampler for large clouds (SA1: 8,192 -> 1,024) on gfx950.
// Reference: farthestpointsamplingKernel, pointnet2_tensorflow/tf_ops/sampling/
// tf_sampling_g.cu:105-170 -- running min distance (:139-145), argmax with the tie rule of the
// 512-thread tree (:146-163), the new centre is the argmax (:164-167).
//
// Same output as fps_v9_kernel, bit for bit, with a different schedule of the same arithmetic.
// v9 spends every iteration on a full block scan (8,192 distances) AND a block-wide argmax
// (wave max, LDS slot, barrier, cross-wave max, centre load): ~1,700 cycles, ~40 % of them in
// the dependent tail. Here:
//  * HOT SET. One wave (wave 0) holds K = 64 * PH candidate points with their exact running
//    min distance. While the best hot point provably beats every other point, it IS the next
//    centre: the hot wave picks it, updates only the K hot distances and goes on -- one wave,
//    no barrier, no block scan per pick.
//  * PROOF. Running min distances only decrease. At a refresh every other point's value is
//    bounded by U, the best (value, tie key) left outside the hot set; the hot winner h is
//    certified iff (T[h], key[h]) beats U in the reference's order (value desc, then key
//    (k mod 512, k div 512) asc). A stale U stays a valid bound, so no cold work is needed
//    between refreshes.
//  * REFRESH (all waves, when certification fails or the centre ring is full). The cold
//    points (v9's register layout, ascending (thread, slot) = tie order) apply every centre
//    picked since the last refresh in one pass (two centres per pass: v_min3), so each
//    (point, centre) distance is still computed exactly once. Every lane keeps its top 3
//    (value, slot) in slot order; each DPP row of 16 lanes then extracts its top E points in
//    tie order into the hot set and reports its (E+1)-th as its share of U. A lane asked for a
//    4th point reports its 3rd value as a strict bound (wins ties) and ends its row's
//    extraction: still a valid U.
//  * PROGRESS. The first certification after a refresh always succeeds unless a strict bound
//    ties the best value; then one exact block argmax (the v9 tail) picks the centre.
// A numpy model of this schedule on the SA1 crops (ScanNet-like, duplicates) refreshes ~48
// times for 1,023 picks with PH = 2, E = 8.
#pragma once
#include "../../pointcloud-segmentation-attention_amd/csrc/fps_kernels.h"

namespace pn2 {
namespace {

// phase boundary: s_memtime stamp in STAMP builds, a scheduling barrier when SB is set
#define PN2_HOT_PHASE(ph)                                   \
  if constexpr (SB && !STAMP) __builtin_amdgcn_sched_barrier(0); \
  PN2_STAMP(ph)

// Tie key: smaller = earlier in the reference's order (k mod 512, k div 512). N < 2^25.
PN2_DEV uint32_t hot_key(int k) { return ((uint32_t)(k & 511) << 16) | ((uint32_t)k >> 9); }
// Comparable value code: running mins are int bits >= 0 (or -1 = padding / none); the low bit
// marks a strict bound (it beats a real value of the same distance).
PN2_DEV uint32_t hot_enc(int v) { return (uint32_t)(v + 1) << 1; }

PN2_DEV uint32_t row16_min_lane(bool holder, int lane) {
  // lowest lane of each 16-lane row with holder set (16 = none): max of 16 - (lane & 15)
  const uint32_t r = row16_max_u32(holder ? 16u - (uint32_t)(lane & 15) : 0u);
  return 16u - r;
}

template <int BLOCK, int PPT, int PH, int E, int CLR = 256, bool STAMP = false, bool SB = false>
__global__ __launch_bounds__(BLOCK) void fps_hot_kernel(const float* __restrict__ xyz, int N,
                                                        int M, int32_t* __restrict__ idx,
                                                        float* __restrict__ new_xyz) {
  using Lay = Lay9<BLOCK, PPT>;
  constexpr int NW = BLOCK / kWave;
  constexpr int NROW = BLOCK / 16;
  constexpr int K = kWave * PH;
  static_assert(NROW * E == K, "each row fills E hot entries");
  static_assert(PPT % 2 == 0 && PH == 2, "packed pairs");
  static_assert((CLR & (CLR - 1)) == 0, "ring size");
  static_assert(3 * BLOCK * PPT * 4 + CLR * 16 + K * 8 + NROW * 8 + 64 <= 160 * 1024, "LDS");
  using f2 = float __attribute__((ext_vector_type(2)));
  constexpr int NP = PPT / 2;

  __shared__ float sxyz[3 * BLOCK * PPT];
  __shared__ float4 scl[CLR];   // centres picked since the last refresh (ring)
  __shared__ uint2 sh[K + NROW];  // hot entries, then the per-row bounds (value code, index)
  __shared__ uint2 sred[NW];    // stalled-refresh argmax: (value code, point index) per wave
  __shared__ int sj;

  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave, row = t >> 4;
  unsigned long long clk0 = 0, rt0 = 0;  // STAMP builds: kernel-entry clocks
  if constexpr (STAMP) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
  __syncthreads();

  f2 vx[NP], vy[NP], vz[NP];
  int tb[PPT];
  {
    float lx[PPT], ly[PPT], lz[PPT];
#pragma unroll
    for (int s = 0; s < PPT; ++s) {
      const int k = Lay::point(t, s);
      const int kk = k < N ? k : 0;
      lx[s] = sxyz[3 * kk + 0];
      ly[s] = sxyz[3 * kk + 1];
      lz[s] = sxyz[3 * kk + 2];
    }
#pragma unroll
    for (int s = 0; s < PPT; ++s) {
      const bool in = Lay::point(t, s) < N;
      vx[s / 2][s % 2] = in ? lx[s] : 0.0f;
      vy[s / 2][s % 2] = in ? ly[s] : 0.0f;
      vz[s / 2][s % 2] = in ? lz[s] : 0.0f;
      tb[s] = in ? __float_as_int(kInitTemp) : -1;
    }
  }
  if (t == 0) scl[0] = make_float4(sxyz[0], sxyz[1], sxyz[2], __int_as_float(0));

  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0;
  unsigned long long n_refresh = 0, n_hot = 0, n_tie = 0;  // STAMP builds: refresh rounds, hot picks
  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
  }
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int j = 1, la = 0;  // picks so far; centres [0, la) are applied to the cold registers
  bool stalled = false;
  // every two rounds pick at least one centre (a stalled round is followed by an exact pick),
  // so 2M + 2 rounds always suffice; the bound only guarantees that the grid drains
  for (int round = 0; round < 2 * M + 2; ++round) {
    __syncthreads();  // the centres in scl are visible to every wave
    PN2_HOT_PHASE(5)
    // outputs of the centres picked since the last round, coalesced (scl.w = point index)
    for (int e = la + t; e < j; e += BLOCK) {
      const float4 c = scl[e & (CLR - 1)];
      I[e] = __float_as_int(c.w);
      if (NX) { NX[3 * e] = c.x; NX[3 * e + 1] = c.y; NX[3 * e + 2] = c.z; }
    }
    if (j >= M) break;
    if constexpr (STAMP) ++n_refresh;
    // ---- cold pass: centres [la, j), two per pass (same rounding as sqdist, then v_min3)
    for (int c = la; c < j; c += 2) {
      const float4 c1 = scl[c & (CLR - 1)];
      const float4 c2 = scl[(c + 1 < j ? c + 1 : c) & (CLR - 1)];
      const f2 a1x = {c1.x, c1.x}, a1y = {c1.y, c1.y}, a1z = {c1.z, c1.z};
      const f2 a2x = {c2.x, c2.x}, a2y = {c2.y, c2.y}, a2z = {c2.z, c2.z};
#pragma unroll
      for (int h = 0; h < NP; ++h) {
        const f2 dx1 = vx[h] - a1x, dy1 = vy[h] - a1y, dz1 = vz[h] - a1z;
        const f2 d1 = (dx1 * dx1 + dy1 * dy1) + dz1 * dz1;
        const f2 dx2 = vx[h] - a2x, dy2 = vy[h] - a2y, dz2 = vz[h] - a2z;
        const f2 d2 = (dx2 * dx2 + dy2 * dy2) + dz2 * dz2;
        tb[2 * h] = min(min(tb[2 * h], __float_as_int(d1.x)), __float_as_int(d2.x));
        tb[2 * h + 1] = min(min(tb[2 * h + 1], __float_as_int(d1.y)), __float_as_int(d2.y));
      }
    }
    la = j;
    PN2_HOT_PHASE(0)

    // ---- per-lane top 3 (value, slot), strict '>' in slot order = tie order in the lane
    int m1 = -1, m2 = -1, m3 = -1, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int s = 0; s < PPT; ++s) {
      const int v = tb[s];
      const bool c1 = v > m1, c2 = v > m2, c3 = v > m3;
      s3 = c2 ? s2 : (c3 ? s : s3);
      s2 = c1 ? s1 : (c2 ? s : s2);
      s1 = c1 ? s : s1;
      m3 = c2 ? m2 : (c3 ? v : m3);
      m2 = c1 ? m1 : (c2 ? v : m2);
      m1 = c1 ? v : m1;
    }
    PN2_HOT_PHASE(1)

    if (stalled) {
      // exact block argmax (the v9 tail) when a strict bound tied the best value
      const uint32_t e1 = hot_enc(m1);
      const uint32_t wm = wave_max_u32(e1);
      const uint64_t hold = __builtin_amdgcn_ballot_w64(e1 == wm);
      const int L = (int)__builtin_amdgcn_readfirstlane((int)__builtin_ctzll(hold));
      const int sl = __builtin_amdgcn_readlane(s1, L);
      if (lane == 0) sred[w] = make_uint2(wm, (uint32_t)Lay::point(w * kWave + L, sl));
      __syncthreads();
      const uint2 r = (lane & 7) < NW ? sred[lane & 7] : make_uint2(0u, 0u);
      uint32_t bm = max_dpp_u32<kDppXor1>(r.x);
      bm = max_dpp_u32<kDppXor2>(bm);
      bm = max_dpp_u32<kDppHalfMirror>(bm);
      const uint64_t wins = __builtin_amdgcn_ballot_w64(r.x == bm) & 0xFFull;
      const int wi = (int)__builtin_amdgcn_readfirstlane((int)__builtin_ctzll(wins));
      const int k = __builtin_amdgcn_readlane((int)r.y, wi);
      if (t == 0)
        scl[j & (CLR - 1)] =
            make_float4(sxyz[3 * k], sxyz[3 * k + 1], sxyz[3 * k + 2], __int_as_float(k));
      ++j;
      stalled = false;
      __syncthreads();  // sred reads done before the next stalled round could write it
      continue;
    }

    // ---- row extraction: E hot entries per row in tie order, then the row's bound.
    // sh[0, K): hot entries, sh[K + row]: the row's bound; both (value code, point index).
    if ((lane & 15) <= E) sh[(lane & 15) < E ? row * E + (lane & 15) : K + row] = make_uint2(0u, 0u);
    {
      int p = 0;          // entries this lane has given
      bool done = false;  // row finished (uniform within the row)
#pragma unroll
      for (int r = 0; r <= E; ++r) {
        const int cv = p == 0 ? m1 : (p == 1 ? m2 : m3);
        const int cs = p == 0 ? s1 : (p == 1 ? s2 : s3);
        const uint32_t enc = p < 3 ? hot_enc(cv) : (hot_enc(m3) | 1u);
        const uint32_t rmax = row16_max_u32(done ? 0u : enc);
        const bool holder = !done && rmax != 0u && enc == rmax;
        const uint32_t wl = row16_min_lane(holder, lane);
        const bool win = holder && (uint32_t)(lane & 15) == wl;
        const bool bound = (enc & 1u) != 0u || r == E;
        if (win) sh[bound ? K + row : row * E + r] = make_uint2(enc, (uint32_t)Lay::point(t, cs));
        p += win ? 1 : 0;
        done = done || rmax == 0u || (rmax & 1u) != 0u;
      }
    }
    PN2_HOT_PHASE(2)
    __syncthreads();  // hot entries and bounds complete
    PN2_HOT_PHASE(3)

    if (wu == 0) {
      // ---- hot phase (wave 0 only; the other waves wait at the next barrier). Control is
      // wave-uniform: every decision is on readfirstlane / ballot / readlane values.
      int hv[PH], hk[PH];
      f2 hx, hy, hz;
#pragma unroll
      for (int q = 0; q < PH; ++q) {
        const uint2 e = sh[lane * PH + q];
        hv[q] = (int)(e.x >> 1) - 1;  // code 0 (no entry) -> -1
        hk[q] = (int)e.y;
        hx[q] = sxyz[3 * hk[q] + 0];
        hy[q] = sxyz[3 * hk[q] + 1];
        hz[q] = sxyz[3 * hk[q] + 2];
      }
      const uint32_t hkey0 = hot_key(hk[0]), hkey1 = hot_key(hk[1]);
      // U = best (value code desc, key asc) over the row bounds: 64-bit max of (code, ~key)
      uint64_t u = 0;
      if (lane < NROW) {
        const uint2 e = sh[K + lane];
        u = pack64(~hot_key((int)e.y), e.x);
      }
      u = wave_max_u64(u);
      const uint32_t Uenc = uniform_u32((uint32_t)(u >> 32));
      const uint32_t Ukey = ~uniform_u32((uint32_t)u);
      PN2_HOT_PHASE(6)
      int jj = j;
      for (;;) {
        const bool b1 = hv[1] > hv[0] || (hv[1] == hv[0] && hkey1 < hkey0);
        const int cv = b1 ? hv[1] : hv[0];
        const uint32_t ck = b1 ? hkey1 : hkey0;
        const uint32_t enc = hot_enc(cv);
        const uint32_t wm = uniform_u32(wave_max_u32(enc));
        const uint64_t hold = __builtin_amdgcn_ballot_w64(enc == wm);
        int L;
        if (__builtin_popcountll(hold) == 1) {
          L = (int)__builtin_ctzll(hold);
        } else {  // equal values: the smallest tie key among the holders
          if constexpr (STAMP) ++n_tie;
          const uint32_t km = ~uniform_u32(wave_max_u32(enc == wm ? ~ck : 0u));
          L = (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(enc == wm && ck == km));
        }
        const uint32_t wkey = (uint32_t)__builtin_amdgcn_readlane((int)ck, L);
        if (!(wm != 0u && (wm > Uenc || (wm == Uenc && wkey < Ukey)))) break;
        const float lx = b1 ? hx[1] : hx[0], ly = b1 ? hy[1] : hy[0], lz = b1 ? hz[1] : hz[0];
        const int lk = b1 ? hk[1] : hk[0];
        if (lane == L) scl[jj & (CLR - 1)] = make_float4(lx, ly, lz, __int_as_float(lk));
        const float cx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                             __builtin_bit_cast(int, lx), L));
        const float cy = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                             __builtin_bit_cast(int, ly), L));
        const float cz = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                             __builtin_bit_cast(int, lz), L));
        ++jj;
        if constexpr (STAMP) ++n_hot;
        if (jj >= M || jj - la >= CLR) break;
        const f2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
        const f2 dx = hx - c2x, dy = hy - c2y, dz = hz - c2z;
        const f2 d = (dx * dx + dy * dy) + dz * dz;
        hv[0] = min(hv[0], __float_as_int(d.x));
        hv[1] = min(hv[1], __float_as_int(d.y));
      }
      PN2_HOT_PHASE(7)
      if (lane == 0) sj = jj;
    }
    __syncthreads();
    PN2_HOT_PHASE(4)
    const int jn = sj;
    stalled = jn == j;
    j = jn;
  }
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x < 16) {
      for (int ph = 0; ph < 6; ++ph) g_stamp[(blockIdx.x * 16 + w) * 8 + ph] = st_acc[ph];
      g_stamp[(blockIdx.x * 16 + w) * 8 + 6] = n_refresh;
      g_stamp[(blockIdx.x * 16 + w) * 8 + 7] = n_hot;
      if (w == 0) {  // whole-kernel shader cycles and 100 MHz real time of this workgroup
        const unsigned long long clk1 = __builtin_amdgcn_s_memtime();
        const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
        g_stamp[(blockIdx.x * 16 + 8) * 8 + 0] = clk1 - clk0;
        g_stamp[(blockIdx.x * 16 + 8) * 8 + 1] = rt1 - rt0;
        g_stamp[(blockIdx.x * 16 + 8) * 8 + 2] = st_acc[6];  // hot setup (H and U loads)
        g_stamp[(blockIdx.x * 16 + 8) * 8 + 3] = st_acc[7];  // hot pick loop
        g_stamp[(blockIdx.x * 16 + 8) * 8 + 4] = n_tie;
      }
    }
  }
}


// ---- asynchronous variant: one hot wave + NCW cold waves in one workgroup ------------------
// Wave 0 runs ONLY the hot loop; waves 1..NCW hold the cold points (v9 layout over their
// 64*NCW threads) and apply each centre as soon as the hot wave publishes it (LDS ring +
// published count), so the cold distance work runs beside the hot loop instead of after it.
// A refresh (both barriers) is left only for the last few centres, the lane top-3 lists and
// the row extraction. The first pick after a refresh needs no certification: the hot set then
// holds every row's best point, so its best is the exact global argmax.
// Cross-wave protocol (LDS, one workgroup): the hot wave writes scl[jj] and then the count
// sj = jj + 1 from the same lane, in program order (DS instructions of one wave execute in
// order, so a wave that reads the new count reads the centre); at the end of its phase it
// writes sstop = 1 after its last count. A cold wave reads sstop, then sj (acquire), and
// leaves its loop only when it saw the stop flag AND has applied every centre below sj.
template <int NCW, int PPT, int E, int NMAX = 8192, int CLR = 256, bool STAMP = false,
          int PRIO = 0>
__global__ __launch_bounds__(64 * (NCW + 1)) void fps_hota_kernel(const float* __restrict__ xyz,
                                                                 int N, int M,
                                                                 int32_t* __restrict__ idx,
                                                                 float* __restrict__ new_xyz) {
  constexpr int CB = kWave * NCW;  // cold threads
  constexpr int BLOCK = CB + kWave;
  constexpr int NROW = CB / 16;
  constexpr int PH = 2;
  constexpr int K = kWave * PH;
  static_assert(NROW * E <= K, "each row fills E hot entries");
  static_assert(PPT % 2 == 0, "packed pairs");
  static_assert((CLR & (CLR - 1)) == 0, "ring size");
  static_assert(CB * PPT >= NMAX, "cold capacity");
  static_assert(3 * NMAX * 4 + CLR * 16 + (K + NROW) * 8 + 64 <= 160 * 1024, "LDS");
  using f2 = float __attribute__((ext_vector_type(2)));
  constexpr int NP = PPT / 2;

  __shared__ float sxyz[3 * NMAX];
  __shared__ float4 scl[CLR];     // picked centres (x, y, z, index bits), ring
  __shared__ uint2 sh[K + NROW];  // hot entries, then the per-row bounds (value code, index)
  __shared__ int sj, sstop;       // published picks; end of the hot phase

  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & (kWave - 1);
  const int wu = __builtin_amdgcn_readfirstlane(t / kWave);
  const bool hot = wu == 0;
  const int ct = t - kWave;  // cold thread (waves 1..NCW)
  const int row = ct >> 4;
  // Cold layout: the points in the reference's tie order (k mod 512, k div 512) -- position
  // q = (k mod 512) * H + k div 512 with H = ceil(N / 512) rows -- dealt in contiguous runs of
  // PPT: cold thread ct, slot s holds q = ct * PPT + s. Ascending (thread, slot) is then tie
  // order for any number of cold threads (v9's layout is the case CB | 512).
  const uint32_t H = (uint32_t)((N + 511) >> 9);
  const uint32_t hmagic = H <= 1 ? 0u : (uint32_t)((((uint64_t)1 << 32) + H - 1) / H);
  auto point = [&](int s) -> int {  // point index of slot s of this cold thread, N if padding
    const uint32_t q = (uint32_t)(ct * PPT + s);
    const uint32_t r = H <= 1 ? q : __umulhi(q, hmagic);
    const int k = (int)((q - r * H) * 512u + r);
    return (r < 512u && k < N) ? k : N;
  };
  unsigned long long clk0 = 0, rt0 = 0;
  if constexpr (STAMP) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
  if (t == 0) {
    sj = 1;
    sstop = 0;
  }
  for (int e = NROW * E + t; e < K; e += BLOCK) sh[e] = make_uint2(0u, 0u);  // never filled
  __syncthreads();

  f2 vx[NP], vy[NP], vz[NP];
  int tb[PPT];
  {
    float lx[PPT], ly[PPT], lz[PPT];
#pragma unroll
    for (int s = 0; s < PPT; ++s) {
      const int k = hot ? N : point(s);
      const int kk = k < N ? k : 0;
      lx[s] = sxyz[3 * kk + 0];
      ly[s] = sxyz[3 * kk + 1];
      lz[s] = sxyz[3 * kk + 2];
    }
#pragma unroll
    for (int s = 0; s < PPT; ++s) {
      const bool in = !hot && point(s) < N;
      vx[s / 2][s % 2] = in ? lx[s] : 0.0f;
      vy[s / 2][s % 2] = in ? ly[s] : 0.0f;
      vz[s / 2][s % 2] = in ? lz[s] : 0.0f;
      tb[s] = in ? __float_as_int(kInitTemp) : -1;
    }
  }
  if (t == 0) scl[0] = make_float4(sxyz[0], sxyz[1], sxyz[2], __int_as_float(0));

  // apply centres [c0, c1) (c1 - c0 in {1, 2}) to this lane's cold points
  // apply centres [c0, c1), 1 <= c1 - c0 <= 4, to this lane's cold points (a short batch
  // repeats its last centre: the min is unchanged)
  auto apply = [&](int c0, int c1) {
    float4 q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = scl[(c0 + i < c1 ? c0 + i : c1 - 1) & (CLR - 1)];
#pragma unroll
    for (int h = 0; h < NP; ++h) {
      int d[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f2 ax = {q[i].x, q[i].x}, ay = {q[i].y, q[i].y}, az = {q[i].z, q[i].z};
        const f2 dx = vx[h] - ax, dy = vy[h] - ay, dz = vz[h] - az;
        const f2 dd = (dx * dx + dy * dy) + dz * dz;
        d[i][0] = __float_as_int(dd.x);
        d[i][1] = __float_as_int(dd.y);
      }
#pragma unroll
      for (int e = 0; e < 2; ++e)
        tb[2 * h + e] = min(min(min(min(tb[2 * h + e], d[0][e]), d[1][e]), d[2][e]), d[3][e]);
    }
  };

  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0;
  unsigned long long n_refresh = 0, n_hot = 0, n_tie = 0, n_async = 0, n_spin = 0;
  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
  }
  int la = 0;       // centres written out / known to every wave
  int applied = 0;  // cold waves: centres applied to this wave's points
  for (int round = 0; round < M + 1; ++round) {  // every round picks at least one centre
    __syncthreads();  // B1: the hot phase is over and every cold wave has caught up
    PN2_STAMP(0)
    const int j = sj;
    for (int e = la + t; e < j; e += BLOCK) {  // outputs, coalesced (scl.w = point index)
      const float4 c = scl[e & (CLR - 1)];
      I[e] = __float_as_int(c.w);
      if (NX) { NX[3 * e] = c.x; NX[3 * e + 1] = c.y; NX[3 * e + 2] = c.z; }
    }
    PN2_STAMP(1)
    if (j >= M) break;
    if constexpr (STAMP) ++n_refresh;
    if (!hot) {
      for (int c = applied; c < j; c += 4) apply(c, c + 4 <= j ? c + 4 : j);
      applied = j;
      PN2_STAMP(2)
      // per-lane top 3 (value, slot), strict '>' in slot order = tie order in the lane
      int m1 = -1, m2 = -1, m3 = -1, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
      for (int s = 0; s < PPT; ++s) {
        const int v = tb[s];
        const bool c1 = v > m1, c2 = v > m2, c3 = v > m3;
        s3 = c2 ? s2 : (c3 ? s : s3);
        s2 = c1 ? s1 : (c2 ? s : s2);
        s1 = c1 ? s : s1;
        m3 = c2 ? m2 : (c3 ? v : m3);
        m2 = c1 ? m1 : (c2 ? v : m2);
        m1 = c1 ? v : m1;
      }
      // row extraction: E hot entries per row in tie order, then the row's bound
      if ((lane & 15) <= E) sh[(lane & 15) < E ? row * E + (lane & 15) : K + row] = make_uint2(0u, 0u);
      int p = 0;
      bool done = false;
#pragma unroll
      for (int r = 0; r <= E; ++r) {
        const int cv = p == 0 ? m1 : (p == 1 ? m2 : m3);
        const int cs = p == 0 ? s1 : (p == 1 ? s2 : s3);
        const uint32_t enc = p < 3 ? hot_enc(cv) : (hot_enc(m3) | 1u);
        const uint32_t rmax = row16_max_u32(done ? 0u : enc);
        const bool holder = !done && rmax != 0u && enc == rmax;
        const uint32_t wl = row16_min_lane(holder, lane);
        const bool win = holder && (uint32_t)(lane & 15) == wl;
        const bool bound = (enc & 1u) != 0u || r == E;
        if (win) sh[bound ? K + row : row * E + r] = make_uint2(enc, (uint32_t)point(cs));
        p += win ? 1 : 0;
        done = done || rmax == 0u || (rmax & 1u) != 0u;
      }
      PN2_STAMP(3)
    } else if (t == 0) {
      sstop = 0;
    }
    la = j;
    __syncthreads();  // B2: hot entries and bounds complete
    PN2_STAMP(4)
    if (hot) {
      int hv[PH], hk[PH];
      f2 hx, hy, hz;
#pragma unroll
      for (int q = 0; q < PH; ++q) {
        const uint2 e = sh[lane * PH + q];
        hv[q] = (int)(e.x >> 1) - 1;  // code 0 (no entry) -> -1
        hk[q] = (int)e.y;
        hx[q] = sxyz[3 * hk[q] + 0];
        hy[q] = sxyz[3 * hk[q] + 1];
        hz[q] = sxyz[3 * hk[q] + 2];
      }
      const uint32_t hkey0 = hot_key(hk[0]), hkey1 = hot_key(hk[1]);
      uint64_t u = 0;
      if (lane < NROW) {
        const uint2 e = sh[K + lane];
        u = pack64(~hot_key((int)e.y), e.x);
      }
      u = wave_max_u64(u);
      const uint32_t Uenc = uniform_u32((uint32_t)(u >> 32));
      const uint32_t Ukey = ~uniform_u32((uint32_t)u);
      PN2_STAMP(5)
      int jj = j;
      bool first = true;
      if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
      for (;;) {
        const bool b1 = hv[1] > hv[0] || (hv[1] == hv[0] && hkey1 < hkey0);
        const int cv = b1 ? hv[1] : hv[0];
        const uint32_t ck = b1 ? hkey1 : hkey0;
        const uint32_t enc = hot_enc(cv);
        const uint32_t wm = uniform_u32(wave_max_u32(enc));
        const uint64_t hold = __builtin_amdgcn_ballot_w64(enc == wm);
        int L;
        if (__builtin_popcountll(hold) == 1) {
          L = (int)__builtin_ctzll(hold);
        } else {  // equal values: the smallest tie key among the holders
          if constexpr (STAMP) ++n_tie;
          const uint32_t km = ~uniform_u32(wave_max_u32(enc == wm ? ~ck : 0u));
          L = (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(enc == wm && ck == km));
        }
        const float lx = b1 ? hx[1] : hx[0], ly = b1 ? hy[1] : hy[0], lz = b1 ? hz[1] : hz[0];
        const int lk = b1 ? hk[1] : hk[0];
        const float cx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                             __builtin_bit_cast(int, lx), L));
        const float cy = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                             __builtin_bit_cast(int, ly), L));
        const float cz = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                             __builtin_bit_cast(int, lz), L));
        // the hot update for the next pick goes first; certification and publishing of this
        // pick (scalar work) follow off the dependency chain. A pick that fails certification
        // ends the phase, and the hot values it touched are rebuilt at the refresh.
        {
          const f2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
          const f2 dx = hx - c2x, dy = hy - c2y, dz = hz - c2z;
          const f2 d = (dx * dx + dy * dy) + dz * dz;
          hv[0] = min(hv[0], __float_as_int(d.x));
          hv[1] = min(hv[1], __float_as_int(d.y));
        }
        const uint32_t wkey = (uint32_t)__builtin_amdgcn_readlane((int)ck, L);
        if (!first && !(wm > Uenc || (wm == Uenc && wkey < Ukey))) break;
        first = false;
        const int k = __builtin_amdgcn_readlane(lk, L);
        if (lane == 0) {
          scl[jj & (CLR - 1)] = make_float4(cx, cy, cz, __int_as_float(k));
          asm volatile("" ::: "memory");
          *(volatile int*)&sj = jj + 1;
        }
        ++jj;
        if constexpr (STAMP) ++n_hot;
        if (jj >= M || jj - la >= CLR) break;
      }
      if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(0);
      if (lane == 0) {
        asm volatile("" ::: "memory");
        *(volatile int*)&sstop = 1;
      }
      PN2_STAMP(6)
    } else {
      // apply centres as they are published, until the hot phase has stopped and all applied
      for (int spin = 0; spin < (1 << 22); ++spin) {
        int av = __hip_atomic_load(&sj, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (av == applied) {
          // the count is read again after the stop flag: the hot wave writes its last count
          // before the flag, so a set flag means the count read after it is final
          if (!__hip_atomic_load(&sstop, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            if constexpr (STAMP) ++n_spin;
            __builtin_amdgcn_s_sleep(1);
            continue;
          }
          av = __hip_atomic_load(&sj, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (av == applied) break;
        }
        const int c1 = av - applied >= 4 ? applied + 4 : av;
        apply(applied, c1);
        if constexpr (STAMP) n_async += c1 - applied;
        applied = c1;
      }
      PN2_STAMP(6)
    }
  }
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x < 16) {
      const int wv = t / kWave;
      for (int ph = 0; ph < 8; ++ph) g_stamp[(blockIdx.x * 16 + wv) * 8 + ph] = st_acc[ph];
      if (wv == 0) {
        g_stamp[(blockIdx.x * 16 + 12) * 8 + 0] = __builtin_amdgcn_s_memtime() - clk0;
        g_stamp[(blockIdx.x * 16 + 12) * 8 + 1] = __builtin_amdgcn_s_memrealtime() - rt0;
        g_stamp[(blockIdx.x * 16 + 12) * 8 + 2] = n_refresh;
        g_stamp[(blockIdx.x * 16 + 12) * 8 + 3] = n_hot;
        g_stamp[(blockIdx.x * 16 + 12) * 8 + 4] = n_tie;
      }
      if (wv == 1) {
        g_stamp[(blockIdx.x * 16 + 12) * 8 + 5] = n_async;
        g_stamp[(blockIdx.x * 16 + 12) * 8 + 6] = n_spin;
      }
    }
  }
}

template <int BLOCK, int PPT>
void launch_hot(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s,
                bool sb = false, bool async = false) {
  if (async && sb)
    hipLaunchKernelGGL((fps_hota_kernel<7, 20, 4, 8192, 256, false, 3>), dim3(B), dim3(512), 0, s,
                       xyz, N, M, idx, nx);
  else if (async)
    hipLaunchKernelGGL((fps_hota_kernel<7, 20, 4>), dim3(B), dim3(512), 0, s, xyz, N, M, idx, nx);
  else if (sb)
    hipLaunchKernelGGL((fps_hot_kernel<BLOCK, PPT, 2, 8, 256, false, true>), dim3(B), dim3(BLOCK),
                       0, s, xyz, N, M, idx, nx);
  else
    hipLaunchKernelGGL((fps_hot_kernel<BLOCK, PPT, 2, 8>), dim3(B), dim3(BLOCK), 0, s, xyz, N, M,
                       idx, nx);
}

}  // namespace
}  // namespace pn2
