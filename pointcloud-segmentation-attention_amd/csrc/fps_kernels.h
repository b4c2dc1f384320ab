// Device-side building blocks of the gfx950 farthest-point sampler, shared by the
// production dispatch (fps.hip) (and, in rounds 1-2, a variant lab since removed).
// Reference: farthestpointsamplingKernel, pointnet2_tensorflow/tf_ops/sampling/
// tf_sampling_g.cu:105-170 (tie rule :146-163).
#pragma once
#include "common.h"

namespace pn2 {
namespace {

constexpr float kInitTemp = 1e38f;  // tf_sampling_g.cu:118

// Low word of the argmax key: larger = earlier in the reference's tie order.
PN2_DEV uint32_t tie_low(int k) {
  const uint32_t tk = (((uint32_t)k & 511u) << 20) | ((uint32_t)k >> 9);
  return 0xFFFFFFFFu - tk;
}
PN2_DEV int tie_decode(uint32_t low) {
  const uint32_t tk = 0xFFFFFFFFu - low;
  return (int)((tk >> 20) + ((tk & 0xFFFFFu) << 9));
}

// Thread t owns points t + slot_off(i), i = 0..PPT-1. Slots are ordered so that, within one
// thread, ascending slot = ascending (k mod 512, k div 512); then a strict '>' scan over the
// slots keeps the reference's tie winner inside the thread.
template <int BLOCK, int PPT>
PN2_DEV constexpr int slot_off(int i) {
  if constexpr (BLOCK >= 512) {
    return BLOCK * i;  // k mod 512 is the same for every slot of the thread
  } else {
    constexpr int R = 512 / BLOCK;  // slots per residue class
    if constexpr (PPT <= R) {
      return BLOCK * i;  // all slots < 512: k mod 512 == k
    } else {
      constexpr int Q = PPT / R;  // slots that share one residue
      return BLOCK * ((i % Q) * R + i / Q);
    }
  }
}


// Diagnostic stamps (STAMP builds only; never in a timed production kernel): s_memtime
// deltas per phase accumulated in SGPRs, lane 0 of each wave writes them to g_stamp.
__device__ unsigned long long g_stamp[16 * 16 * 8];
__device__ unsigned long long g_iter[4096];  // STAMP builds: s_memtime at each iteration start
#define PN2_STAMP(ph)                                                              \
  if constexpr (STAMP) {                                                           \
    __builtin_amdgcn_sched_barrier(0);                                             \
    unsigned long long tt__;                                                       \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt__)::"memory");  \
    __builtin_amdgcn_sched_barrier(0);                                             \
    st_acc[ph] += tt__ - st_prev;                                                  \
    st_prev = tt__;                                                                \
  }

// Variant 9 (BLOCK <= 512): v2's register sampler with a cheaper scan and a shorter tail.
//  * point layout: thread t owns residues R*t .. R*t+R-1 of each 512-wide row (R = 512/BLOCK,
//    or all PPT points of a row < 512 wide), i.e. k = W*h + R*t + c with slot s = c*H + h.
//    Then ascending (lane, slot) IS the reference's tie order (k mod 512, k div 512)
//    (tf_sampling_g.cu:146-163), across lanes and waves as well as inside a thread;
//  * scan: slots in groups of G; per group one v_max3 chain folds the G new temps into the
//    running max and ONE compare+select remembers the first group that raised it (strict
//    '>', so the earliest group wins ties) -- (G+1)/G instead of 3 VALU ops per point;
//  * wave: ONE 32-bit max (DPP folded into v_max_u32_dpp + permlane swaps); the winner is
//    the lowest lane of ballot(hi == max) (s_ff1) because lane order is tie order; its group
//    is read with v_readlane and the first slot of that group holding the max is found with
//    scalar compares -- no second (tie-word) reduction;
//  * block: each wave publishes (max, point index) to a double-buffered LDS slot, ONE barrier,
//    then an 8-lane DPP max + ballot/s_ff1 picks the lowest wave holding the block max
//    (lower wave = lower t = earlier in tie order).
template <int BLOCK, int PPT>
struct Lay9 {
  static_assert(BLOCK <= 512 && 512 % BLOCK == 0, "v9 layout needs BLOCK | 512");
  static constexpr int R = PPT < 512 / BLOCK ? PPT : 512 / BLOCK;  // residues per thread
  static constexpr int H = PPT / R;                                 // rows
  static constexpr int W = R * BLOCK;                               // row width (<= 512)
  static_assert(R * H == PPT, "PPT must be a multiple of 512 / BLOCK or below it");
  PN2_DEV static constexpr int point(int t, int s) { return W * (s % H) + R * t + s / H; }
};

// The v9 sampler for one cloud, run by threads 0..BLOCK-1 of the calling workgroup (BLOCK ==
// blockDim.x, or BLOCK == 64 for wave 0 alone: a one-wave body has no barrier).
//   P     the cloud's N points (xyz AoS, global or LDS), loaded into registers once;
//   CXYZ  where the winners' coordinates are read each iteration (an LDS copy of P, or P);
//   I, NX the cloud's idx (M) and new_xyz (M x 3) outputs in global memory (NX may be null);
//   SNEXT optional LDS array that receives new_xyz too (the next sampler's input).
// LRES: every lane resolves its own winning slot with VALU selects right after the scan
// (independent of, so interleaved with, the wave max), leaving one v_readlane after the ballot
// instead of the scalar compare chain over the groups.
// PAD >= 0: that many s_nop right before the iteration loop, shifting the loop's code address
// by 4 * PAD bytes (code placement, tools/place_sa1_loop.py; profiles/r1/pad_fps.log).
// (Measured and removed: the block step as one 64-bit LDS atomic per wave, 794 vs 718 us at
// SA1; the winner's coordinates carried through the block step, chain 126 -> 156 us.)
template <int BLOCK, int PPT, int G, bool STAMP = false, bool LRES = false, int PAD = -1>
PN2_DEV void fps_v9_body(const float* P, int N, int M, const float* CXYZ, int32_t* I, float* NX,
                         float* SNEXT, uint2 (*red)[8]) {
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  using Lay = Lay9<BLOCK, PPT>;
  constexpr int NW = BLOCK / kWave;
  static_assert(BLOCK % kWave == 0 && NW <= 8, "the block step reduces 8 DPP lanes");
  static_assert(PPT % G == 0 && (G == 1 || G == 2 || G == 4), "slot groups");
  constexpr int NG = PPT / G;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int w = t / kWave;

  // Coordinates as float2 pairs of slots (2h, 2h+1): the distance is computed with packed
  // v_pk_* ops on register pairs the allocator cannot split (one op per 2 points).
  using f2 = float __attribute__((ext_vector_type(2)));
  constexpr bool PK = PPT % 2 == 0;
  constexpr int NP = PK ? PPT / 2 : 1;
  f2 vx[NP], vy[NP], vz[NP];
  float px[PK ? 1 : PPT], py[PK ? 1 : PPT], pz[PK ? 1 : PPT];
  int tb[PPT];  // running min distance as int bits; padding slots -1 never win
  // Branch-free loads (padding slots read point 0 and are masked after): all PPT loads are in
  // flight together instead of one load + wait per slot. From CXYZ, the LDS copy when there
  // is one (P == CXYZ otherwise).
  (void)P;
  float lx[PPT], ly[PPT], lz[PPT];
#pragma unroll
  for (int s = 0; s < PPT; ++s) {
    const int k = Lay::point(t, s);
    const int kk = k < N ? k : 0;
    lx[s] = CXYZ[3 * kk + 0];
    ly[s] = CXYZ[3 * kk + 1];
    lz[s] = CXYZ[3 * kk + 2];
  }
#pragma unroll
  for (int s = 0; s < PPT; ++s) {
    const bool in = Lay::point(t, s) < N;
    lx[s] = in ? lx[s] : 0.0f;
    ly[s] = in ? ly[s] : 0.0f;
    lz[s] = in ? lz[s] : 0.0f;
    tb[s] = in ? __float_as_int(kInitTemp) : -1;
    if constexpr (PK) {
      vx[s / 2][s % 2] = lx[s];
      vy[s / 2][s % 2] = ly[s];
      vz[s / 2][s % 2] = lz[s];
    } else {
      px[s] = lx[s]; py[s] = ly[s]; pz[s] = lz[s];
    }
  }
  float cx = CXYZ[0], cy = CXYZ[1], cz = CXYZ[2];
  if (t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
    if (SNEXT) { SNEXT[0] = cx; SNEXT[1] = cy; SNEXT[2] = cz; }
  }

  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
  }
  if constexpr (PAD > 0) asm volatile(".rept %0\n\ts_nop 0\n\t.endr" ::"n"(PAD));
  for (int j = 1; j < M; ++j) {
    int dv[PPT];  // this iteration's squared distances as int bits
    if constexpr (PK) {
      const f2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
#pragma unroll
      for (int h = 0; h < NP; ++h) {  // same rounding sequence as sqdist(), two points per op
        const f2 dx = vx[h] - c2x, dy = vy[h] - c2y, dz = vz[h] - c2z;
        const f2 d = (dx * dx + dy * dy) + dz * dz;
        dv[2 * h] = __float_as_int(d.x);
        dv[2 * h + 1] = __float_as_int(d.y);
      }
    } else {
#pragma unroll
      for (int s = 0; s < PPT; ++s)
        dv[s] = __float_as_int(sqdist(px[s], py[s], pz[s], cx, cy, cz));
    }
    int bd = -1, bg = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      int v[G];
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const int s = g * G + q;
        v[q] = min(dv[s], tb[s]);
        tb[s] = v[q];
      }
      int m;
      if constexpr (G == 4) m = max(max(max(max(v[0], v[1]), v[2]), v[3]), bd);
      else if constexpr (G == 2) m = max(max(v[0], v[1]), bd);
      else m = max(v[0], bd);
      bg = m > bd ? g : bg;
      bd = m;
    }
    // wave: lowest lane holding the wave max, then its first slot holding it
    const uint32_t hi = (uint32_t)(bd + 1);  // 0 for lanes with padding only
    int ls = 0;  // LRES: this lane's first slot holding bd
    if constexpr (LRES) {
      int a[G > 1 ? G - 1 : 1];
#pragma unroll
      for (int q = 0; q + 1 < G; ++q) a[q] = tb[q];
#pragma unroll
      for (int g = 1; g < NG; ++g) {
        const bool sel = bg == g;
#pragma unroll
        for (int q = 0; q + 1 < G; ++q) a[q] = sel ? tb[g * G + q] : a[q];
      }
      int r = G - 1;
#pragma unroll
      for (int q = G - 2; q >= 0; --q) r = a[q] == bd ? q : r;
      ls = bg * G + r;
    }
    PN2_STAMP(0)
    const uint32_t km = wave_max_u32(hi);
    PN2_STAMP(1)
    const uint64_t hold = __builtin_amdgcn_ballot_w64(hi == km);
    const int L = (int)__builtin_amdgcn_readfirstlane((int)__builtin_ctzll(hold));
    int sq = 0;
    if constexpr (LRES) {
      sq = __builtin_amdgcn_readlane(ls, L);
    } else {
      const int gq = __builtin_amdgcn_readlane(bg, L);
      const int kv = (int)km - 1;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if (g == gq) {
          int r = G - 1;
#pragma unroll
          for (int q = G - 2; q >= 0; --q)
            if (__builtin_amdgcn_readlane(tb[g * G + q], L) == kv) r = q;
          sq = g * G + r;
        }
      }
    }
    int old = Lay::point(w * kWave + L, sq);
    PN2_STAMP(2)
    if constexpr (NW > 1) {
      if (lane == 0) red[j & 1][w] = make_uint2(km, (uint32_t)old);
      __syncthreads();
      PN2_STAMP(3)
      const uint2 r = (lane & 7) < NW ? red[j & 1][lane & 7] : make_uint2(0u, 0u);
      uint32_t bm = max_dpp_u32<kDppXor1>(r.x);
      bm = max_dpp_u32<kDppXor2>(bm);
      bm = max_dpp_u32<kDppHalfMirror>(bm);
      const uint64_t wins = __builtin_amdgcn_ballot_w64(r.x == bm) & 0xFFull;
      const int wi = (int)__builtin_amdgcn_readfirstlane((int)__builtin_ctzll(wins));
      old = __builtin_amdgcn_readlane((int)r.y, wi);
    }
    PN2_STAMP(4)
    cx = CXYZ[3 * old + 0]; cy = CXYZ[3 * old + 1]; cz = CXYZ[3 * old + 2];
    if (t == 0) {
      I[j] = old;
      if (NX) { NX[3 * j + 0] = cx; NX[3 * j + 1] = cy; NX[3 * j + 2] = cz; }
      if (SNEXT) { SNEXT[3 * j + 0] = cx; SNEXT[3 * j + 1] = cy; SNEXT[3 * j + 2] = cz; }
    }
    PN2_STAMP(5)
  }
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x < 16)
      for (int ph = 0; ph < 6; ++ph) g_stamp[(blockIdx.x * 16 + w) * 8 + ph] = st_acc[ph];
  }
}

template <int BLOCK, int PPT, int G, bool XYZ_LDS, bool STAMP = false, bool LRES = false,
          int PAD = -1>
__global__ __launch_bounds__(BLOCK) void fps_v9_kernel(const float* __restrict__ xyz, int N,
                                                       int M, int32_t* __restrict__ idx,
                                                       float* __restrict__ new_xyz) {
  __shared__ uint2 red[2][8];
  __shared__ float sxyz[XYZ_LDS ? 3 * BLOCK * PPT : 1];
  const int b = blockIdx.x;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  if constexpr (XYZ_LDS) {
    for (int e = threadIdx.x; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
    __syncthreads();
  }
  fps_v9_body<BLOCK, PPT, G, STAMP, LRES, PAD>(
      P, N, M, XYZ_LDS ? sxyz : P, idx + (size_t)b * M,
      new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr, nullptr, red);
}

template <int BLOCK, int PPT, int G, bool LRES = false, int PAD = -1>
void launch_v9(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s) {
  if constexpr (3 * BLOCK * PPT * 4 + 256 <= 160 * 1024)
    hipLaunchKernelGGL((fps_v9_kernel<BLOCK, PPT, G, true, false, LRES, PAD>), dim3(B),
                       dim3(BLOCK), 0, s, xyz, N, M, idx, nx);
  else
    hipLaunchKernelGGL((fps_v9_kernel<BLOCK, PPT, G, false, false, LRES, PAD>), dim3(B),
                       dim3(BLOCK), 0, s, xyz, N, M, idx, nx);
}


}  // namespace
}  // namespace pn2
