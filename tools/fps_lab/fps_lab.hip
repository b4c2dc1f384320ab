// FPS variant lab: the sampler designs measured against the production kernel
// (fps_v2_kernel / fps_v9_kernel in fps_kernels.h) on the MI355X with tools/tune_fps.py
// and tools/stamp_fps.py. NOT part of libpn2hip.so: built into tools/fps_lab/libpn2fpslab.so
// by tools/fps_lab/Makefile. DESIGN.md records what each variant taught.
#include "../../pointcloud-segmentation-attention_amd/csrc/fps_kernels.h"
#include "fps_hot.h"
#include "../../pointcloud-segmentation-attention_amd/csrc/fps_cull.h"

namespace pn2 {
namespace {

// Variant 11 (measured SLOWER than v9: 808 vs 768 us at SA1; tools/stamp_fps.py shows the
// uniform-index moves and readlane chains cost more latency than the branch chain and the
// LDS centre load they replace). v9's layout and scan with a shorter tail. The winner's slot inside its group
// and its coordinates are read straight out of the winning lane's registers with
// uniform-index register moves (s_set_gpr_idx + v_readlane: no branch chain), and each
// wave publishes (max, index, x, y, z) so that after the barrier the new centre comes from
// v_readlane of the winning wave's entry instead of a dependent LDS load. No LDS copy of
// the cloud is needed.
template <int BLOCK, int PPT, int G, bool STAMP = false>
__global__ __launch_bounds__(BLOCK) void fps_v11_kernel(const float* __restrict__ xyz, int N,
                                                        int M, int32_t* __restrict__ idx,
                                                        float* __restrict__ new_xyz) {
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  using Lay = Lay9<BLOCK, PPT>;
  constexpr int NW = BLOCK / kWave;
  static_assert(BLOCK % kWave == 0 && NW <= 8, "the block step reduces 8 DPP lanes");
  static_assert(PPT % G == 0 && (G == 1 || G == 2 || G == 4), "slot groups");
  constexpr int NG = PPT / G;
  __shared__ uint2 red_k[2][8];
  __shared__ float4 red_c[2][8];

  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  float px[PPT], py[PPT], pz[PPT];
  int tb[PPT];  // running min distance as int bits; padding slots -1 never win
#pragma unroll
  for (int s = 0; s < PPT; ++s) {
    const int k = Lay::point(t, s);
    if (k < N) {
      px[s] = P[3 * k + 0];
      py[s] = P[3 * k + 1];
      pz[s] = P[3 * k + 2];
      tb[s] = __float_as_int(kInitTemp);
    } else {
      px[s] = py[s] = pz[s] = 0.0f;
      tb[s] = -1;
    }
  }

  float cx = P[0], cy = P[1], cz = P[2];
  if (t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }

  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
  }
  for (int j = 1; j < M; ++j) {
    int bd = -1, bg = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      int v[G];
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const int s = g * G + q;
        v[q] = min(__float_as_int(sqdist(px[s], py[s], pz[s], cx, cy, cz)), tb[s]);
        tb[s] = v[q];
      }
      int m;
      if constexpr (G == 4) m = max(max(max(max(v[0], v[1]), v[2]), v[3]), bd);
      else if constexpr (G == 2) m = max(max(v[0], v[1]), bd);
      else m = max(v[0], bd);
      bg = m > bd ? g : bg;
      bd = m;
    }
    const uint32_t hi = (uint32_t)(bd + 1);  // 0 for lanes with padding only
    PN2_STAMP(0)
    const uint32_t km = wave_max_u32(hi);
    PN2_STAMP(1)
    // lowest lane holding the wave max (lane order is tie order), its first slot holding it
    const uint64_t hold = __builtin_amdgcn_ballot_w64(hi == km);
    const int L = (int)__builtin_amdgcn_readfirstlane((int)__builtin_ctzll(hold));
    // everything below is wave-uniform (SGPRs): scalar compares, uniform-index moves
    const int base = __builtin_amdgcn_readlane(bg, L) * G;
    const int kv = __builtin_amdgcn_readfirstlane((int)km) - 1;
    int sq = base + G - 1;
#pragma unroll
    for (int q = G - 2; q >= 0; --q)
      if (__builtin_amdgcn_readlane(tb[base + q], L) == kv) sq = base + q;
    sq = __builtin_amdgcn_readfirstlane(sq);
    int old = Lay::point(w * kWave + L, sq);
    float wx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(px[sq]), L));
    float wy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(py[sq]), L));
    float wz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pz[sq]), L));
    PN2_STAMP(2)
    if constexpr (NW > 1) {
      if (lane == 0) {
        red_k[j & 1][w] = make_uint2(km, (uint32_t)old);
        red_c[j & 1][w] = make_float4(wx, wy, wz, 0.0f);
      }
      __syncthreads();
      PN2_STAMP(3)
      const int e = lane & 7;
      const uint2 r = e < NW ? red_k[j & 1][e] : make_uint2(0u, 0u);
      const float4 c = red_c[j & 1][e < NW ? e : 0];
      uint32_t bm = max_dpp_u32<kDppXor1>(r.x);
      if constexpr (NW > 2) bm = max_dpp_u32<kDppXor2>(bm);
      if constexpr (NW > 4) bm = max_dpp_u32<kDppHalfMirror>(bm);
      const uint64_t wins = __builtin_amdgcn_ballot_w64(r.x == bm) & 0xFFull;
      const int wi = (int)__builtin_amdgcn_readfirstlane((int)__builtin_ctzll(wins));
      old = __builtin_amdgcn_readlane((int)r.y, wi);
      wx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.x), wi));
      wy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.y), wi));
      wz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.z), wi));
    }
    PN2_STAMP(4)
    cx = wx; cy = wy; cz = wz;
    if (t == 0) {
      I[j] = old;
      if (NX) { NX[3 * j + 0] = cx; NX[3 * j + 1] = cy; NX[3 * j + 2] = cz; }
    }
    PN2_STAMP(5)
  }
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x < 16)
      for (int ph = 0; ph < 6; ++ph) g_stamp[(blockIdx.x * 16 + w) * 8 + ph] = st_acc[ph];
  }
}

template <int BLOCK, int PPT, int G>
void launch_v11(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s) {
  hipLaunchKernelGGL((fps_v11_kernel<BLOCK, PPT, G>), dim3(B), dim3(BLOCK), 0, s, xyz, N, M, idx,
                     nx);
}


// Variant 2 of the register sampler: the same selection, cheaper arithmetic.
//  * the running min-distance is kept as int32 bit patterns: for d >= 0 (or NaN) and
//    temp in {-1} U [0, 1e38] a signed-int min of the bits is exactly fminf (no IEEE-mode
//    canonicalisation before every v_min_f32); padding slots hold -1 and never win;
//  * the argmax is two 32-bit max-reductions (distance, then ~tiekey among the lanes that hold
//    the maximum distance) whose DPP moves fold into v_max_u32_dpp, instead of one 64-bit
//    reduction; the cross-wave step is the same pair over the per-wave results.
template <int BLOCK, int PPT, bool XYZ_LDS, bool STAMP = false>
__global__ __launch_bounds__(BLOCK) void fps_v2_kernel(const float* __restrict__ xyz, int N,
                                                       int M, int32_t* __restrict__ idx,
                                                       float* __restrict__ new_xyz) {
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  constexpr int NW = BLOCK / kWave;
  static_assert(NW <= 16, "the cross-wave step reduces one 16-lane DPP row");
  __shared__ uint2 red[2][16];
  __shared__ float sxyz[XYZ_LDS ? 3 * BLOCK * PPT : 1];

  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  float px[PPT], py[PPT], pz[PPT];
  int tb[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int k = t + slot_off<BLOCK, PPT>(i);
    if (k < N) {
      px[i] = P[3 * k + 0];
      py[i] = P[3 * k + 1];
      pz[i] = P[3 * k + 2];
      tb[i] = __float_as_int(kInitTemp);
    } else {
      px[i] = py[i] = pz[i] = 0.0f;
      tb[i] = -1;
    }
  }
  if constexpr (XYZ_LDS) {
    for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
    __syncthreads();
  }

  float cx = P[0], cy = P[1], cz = P[2];
  if (t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }

  if constexpr (STAMP) {
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
  }
  for (int j = 1; j < M; ++j) {
    int bd = -1, bi = 0;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int v = min(__float_as_int(sqdist(px[i], py[i], pz[i], cx, cy, cz)), tb[i]);
      tb[i] = v;
      if (v > bd) { bd = v; bi = i; }
    }
    int off;
    if constexpr (BLOCK >= 512 || PPT <= 512 / BLOCK) {
      off = BLOCK * bi;
    } else {
      constexpr int R = 512 / BLOCK, Q = PPT / R;
      off = BLOCK * ((bi % Q) * R + bi / Q);
    }
    const uint32_t hi = bd < 0 ? 0u : (uint32_t)bd + 1u;
    const uint32_t lo = bd < 0 ? 0u : tie_low(t + off);
    PN2_STAMP(0)
    uint32_t km = wave_max_u32(hi);
    uint32_t kl = wave_max_u32(hi == km ? lo : 0u);
    PN2_STAMP(1)
    if constexpr (NW > 1) {
      if (lane == 0) red[j & 1][w] = make_uint2(km, kl);
      __syncthreads();
      PN2_STAMP(2)
      const uint2 r = lane < NW ? red[j & 1][lane] : make_uint2(0u, 0u);
      km = row16_max_u32(r.x);
      kl = row16_max_u32(r.x == km ? r.y : 0u);
    }
    const int old = tie_decode(uniform_u32(kl));
    PN2_STAMP(3)
    if constexpr (XYZ_LDS) {
      cx = sxyz[3 * old + 0]; cy = sxyz[3 * old + 1]; cz = sxyz[3 * old + 2];
    } else {
      cx = P[3 * old + 0]; cy = P[3 * old + 1]; cz = P[3 * old + 2];
    }
    PN2_STAMP(4)
    if (t == 0) {
      I[j] = old;
      if (NX) { NX[3 * j + 0] = cx; NX[3 * j + 1] = cy; NX[3 * j + 2] = cz; }
    }
    PN2_STAMP(5)
  }
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x < 16)
      for (int ph = 0; ph < 6; ++ph) g_stamp[(blockIdx.x * 16 + w) * 8 + ph] = st_acc[ph];
  }
}


template <int BLOCK, int PPT>
void launch_v2(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s) {
  if constexpr (3 * BLOCK * PPT * 4 + 256 <= 160 * 1024)
    hipLaunchKernelGGL((fps_v2_kernel<BLOCK, PPT, true>), dim3(B), dim3(BLOCK), 0, s, xyz, N, M,
                       idx, nx);
  else
    hipLaunchKernelGGL((fps_v2_kernel<BLOCK, PPT, false>), dim3(B), dim3(BLOCK), 0, s, xyz, N,
                       M, idx, nx);
}


template <int BLOCK, int PPT, bool XYZ_LDS>
__global__ __launch_bounds__(BLOCK) void fps_reg_kernel(const float* __restrict__ xyz, int N,
                                                        int M, int32_t* __restrict__ idx,
                                                        float* __restrict__ new_xyz) {
  constexpr int NW = BLOCK / kWave;
  static_assert(NW <= 16, "the cross-wave step reduces one 16-lane DPP row");
  __shared__ uint64_t red[2][16];
  __shared__ float sxyz[XYZ_LDS ? 3 * BLOCK * PPT : 1];

  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  float px[PPT], py[PPT], pz[PPT], tm[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int k = t + slot_off<BLOCK, PPT>(i);
    if (k < N) {
      px[i] = P[3 * k + 0];
      py[i] = P[3 * k + 1];
      pz[i] = P[3 * k + 2];
      tm[i] = kInitTemp;
    } else {  // padding slot: min(d, -1) stays -1 and never wins
      px[i] = py[i] = pz[i] = 0.0f;
      tm[i] = -1.0f;
    }
  }
  if constexpr (XYZ_LDS) {
    for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
    __syncthreads();
  }

  float cx = P[0], cy = P[1], cz = P[2];  // old = 0 (tf_sampling_g.cu:114-116)
  if (t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }

  for (int j = 1; j < M; ++j) {
    float bd = -1.0f;
    int bi = 0;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const float d = sqdist(px[i], py[i], pz[i], cx, cy, cz);
      const float v = fminf(d, tm[i]);  // tf_sampling_g.cu:143
      tm[i] = v;
      if (v > bd) { bd = v; bi = i; }   // tf_sampling_g.cu:146-149
    }
    // runtime slot -> point index (same mapping as slot_off, shifts and masks only)
    int off;
    if constexpr (BLOCK >= 512 || PPT <= 512 / BLOCK) {
      off = BLOCK * bi;
    } else {
      constexpr int R = 512 / BLOCK, Q = PPT / R;
      off = BLOCK * ((bi % Q) * R + bi / Q);
    }
    uint64_t key = bd < 0.0f ? 0ull : pack64(tie_low(t + off), __float_as_uint(bd));
    key = wave_max_u64(key);
    if constexpr (NW > 1) {
      if (lane == 0) red[j & 1][w] = key;
      __syncthreads();
      key = row16_max_u64(lane < NW ? red[j & 1][lane] : 0ull);
    }
    const int old = tie_decode(uniform_u32((uint32_t)key));
    if constexpr (XYZ_LDS) {
      cx = sxyz[3 * old + 0]; cy = sxyz[3 * old + 1]; cz = sxyz[3 * old + 2];
    } else {
      cx = P[3 * old + 0]; cy = P[3 * old + 1]; cz = P[3 * old + 2];
    }
    if (t == 0) {
      I[j] = old;
      if (NX) { NX[3 * j + 0] = cx; NX[3 * j + 1] = cy; NX[3 * j + 2] = cz; }
    }
  }
}

// Variant 7: v2's scan with a short tail.
//  * wave: ONE 32-bit max of the distance word (folded DPP + permlane swaps);
//  * the lane(s) holding it issue ds_max_u64 of the packed (distance, tie word) key into one
//    LDS word — the LDS atomic resolves equal distances across lanes and waves exactly (max of
//    ~tiekey) and replaces the cross-wave reduction: after the barrier every wave reads one
//    word. The word is triple-buffered by iteration (j mod 3); wave 0 zeroes word (j+2) mod 3
//    right after barrier j, when every wave has finished reading it (iteration j-1) and before
//    anyone can add to it (iteration j+2, after barrier j+1);
//  * idx / new_xyz gathered in registers of wave 0 and stored 64 at a time.
template <int BLOCK, int PPT, bool STAMP = false>
__global__ __launch_bounds__(BLOCK) void fps_v7_kernel(const float* __restrict__ xyz, int N,
                                                       int M, int32_t* __restrict__ idx,
                                                       float* __restrict__ new_xyz) {
  constexpr int NW = BLOCK / kWave;
  constexpr bool XYZ_LDS = 12 * BLOCK * PPT + 64 <= 160 * 1024;
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  __shared__ unsigned long long s_key[3];
  __shared__ float sxyz[XYZ_LDS ? 3 * BLOCK * PPT : 1];

  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  float px[PPT], py[PPT], pz[PPT];
  int tb[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int k = t + slot_off<BLOCK, PPT>(i);
    if (k < N) {
      px[i] = P[3 * k + 0];
      py[i] = P[3 * k + 1];
      pz[i] = P[3 * k + 2];
      tb[i] = __float_as_int(kInitTemp);
    } else {
      px[i] = py[i] = pz[i] = 0.0f;
      tb[i] = -1;
    }
  }
  if constexpr (XYZ_LDS) {
    for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
  }
  if (t < 3) s_key[t] = 0ull;
  __syncthreads();

  float cx = P[0], cy = P[1], cz = P[2];
  int ring_i = 0;
  float ring_x = cx, ring_y = cy, ring_z = cz;
  if constexpr (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
  for (int j = 1; j < M; ++j) {
    int bd = -1, bi = 0;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int v = min(__float_as_int(sqdist(px[i], py[i], pz[i], cx, cy, cz)), tb[i]);
      tb[i] = v;
      if (v > bd) { bd = v; bi = i; }
    }
    int off;
    if constexpr (BLOCK >= 512 || PPT <= 512 / BLOCK) {
      off = BLOCK * bi;
    } else {
      constexpr int R = 512 / BLOCK, Q = PPT / R;
      off = BLOCK * ((bi % Q) * R + bi / Q);
    }
    const uint32_t hi = bd < 0 ? 0u : (uint32_t)bd + 1u;
    PN2_STAMP(0)
    const uint32_t wm = wave_max_u32(hi);
    PN2_STAMP(1)
    uint32_t kl;
    if constexpr (NW > 1) {
      if (hi == wm) atomicMax(&s_key[j % 3], pack64(tie_low(t + off), hi));
      __syncthreads();
      PN2_STAMP(2)
      if (w == 0 && lane == 0) s_key[(j + 2) % 3] = 0ull;
      kl = (uint32_t)s_key[j % 3];
    } else {
      const uint64_t ball = __ballot(hi == wm);
      const uint32_t lo = tie_low(t + off);
      if (__popcll(ball) == 1)
        kl = (uint32_t)__builtin_amdgcn_readlane((int)lo, __ffsll((unsigned long long)ball) - 1);
      else
        kl = uniform_u32(wave_max_u32(hi == wm ? lo : 0u));
    }
    const int old = tie_decode(uniform_u32(kl));
    PN2_STAMP(3)
    if constexpr (XYZ_LDS) {
      cx = sxyz[3 * old + 0]; cy = sxyz[3 * old + 1]; cz = sxyz[3 * old + 2];
    } else {
      cx = P[3 * old + 0]; cy = P[3 * old + 1]; cz = P[3 * old + 2];
    }
    PN2_STAMP(4)
    if (w == 0) {
      const int sl = j & (kWave - 1);
      const bool mine = lane == sl;
      ring_i = mine ? old : ring_i;
      ring_x = mine ? cx : ring_x;
      ring_y = mine ? cy : ring_y;
      ring_z = mine ? cz : ring_z;
      if (sl == kWave - 1 || j == M - 1) {
        const int jj = (j & ~(kWave - 1)) + lane;
        if (lane <= sl) {
          I[jj] = ring_i;
          if (NX) { NX[3 * jj] = ring_x; NX[3 * jj + 1] = ring_y; NX[3 * jj + 2] = ring_z; }
        }
      }
    }
    PN2_STAMP(5)
  }
  if (M == 1 && t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x < 16)
      for (int ph = 0; ph < 6; ++ph) g_stamp[(blockIdx.x * 16 + w) * 8 + ph] = st_acc[ph];
  }
}

// Variant 3: spatially culled sampler (exact).
// At setup the cloud is counting-sorted by a 12-bit Morton cell code (16^3 grid over its
// bounding box) in LDS, and thread slots are filled in that order, so every "cell" = SUB
// slots x 64 lanes of one wave holds 64*SUB spatially adjacent points. Each cell keeps, in
// SGPRs, its bounding box, its best key (max running distance km, tie word kl) and therefore
// U = max running distance inside it. When the new centre c is so far from the cell's box that
// even the smallest possible fp32 squared distance exceeds U (lb*(1-2^-16) > U, lb from the
// box; the margin covers fp32 rounding of both sides), no min(d, temp) of the
// cell can change: the cell's scan, its reductions and its key are skipped. The result is
// identical to the unculled sampler; only the work per iteration shrinks as sampling refines.
// Ties are broken by each point's ORIGINAL index (the per-point tie word tl), so the spatial
// reordering does not change the reference's choice.
constexpr int kCellBits = 4;                       // 16 cells per axis
constexpr int kNumCodes = 1 << (3 * kCellBits);    // 4096

PN2_DEV uint32_t spread3(uint32_t v) {  // 4 bits -> every third bit
  v &= 0xF;
  v = (v | (v << 4)) & 0x0C3;
  v = (v | (v << 2)) & 0x249;
  return v;
}

PN2_DEV float wave_min_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, kWave));
  return v;
}
PN2_DEV float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
PN2_DEV float uniform_f(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

template <int BLOCK, int PPT, int SUB, bool XYZ_LDS>
__global__ __launch_bounds__(BLOCK) void fps_cull_kernel(const float* __restrict__ xyz, int N,
                                                         int M, int32_t* __restrict__ idx,
                                                         float* __restrict__ new_xyz) {
  constexpr int NW = BLOCK / kWave;
  constexpr int CAP = BLOCK * PPT;
  constexpr int NCELL = PPT / SUB;
  static_assert(NW <= 16 && PPT % SUB == 0, "config");
  // LDS: [A] setup: cell code (u16) + sorted index (u16) per point; later: xyz copy (fp32)
  //      [H] histogram / offsets of the 4096 Morton cells
  constexpr int A_BYTES = XYZ_LDS ? 12 * CAP : 4 * CAP;
  __shared__ __attribute__((aligned(16))) unsigned char smem_a[A_BYTES];
  __shared__ uint32_t hist[kNumCodes];
  __shared__ uint2 red[2][16];
  __shared__ float bbox_red[16][6];
  uint16_t* s_code = reinterpret_cast<uint16_t*>(smem_a);
  uint16_t* s_sorted = s_code + CAP;
  float* sxyz = reinterpret_cast<float*>(smem_a);

  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  // ---- setup 1: bounding box of the cloud
  float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int k = t; k < N; k += BLOCK)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float v = P[3 * k + a];
      lo[a] = fminf(lo[a], v);
      hi[a] = fmaxf(hi[a], v);
    }
#pragma unroll
  for (int a = 0; a < 3; ++a) { lo[a] = wave_min_f(lo[a]); hi[a] = wave_max_f(hi[a]); }
  if (lane == 0)
#pragma unroll
    for (int a = 0; a < 3; ++a) { bbox_red[w][a] = lo[a]; bbox_red[w][3 + a] = hi[a]; }
  for (int e = t; e < kNumCodes; e += BLOCK) hist[e] = 0;
  __syncthreads();
  float scale[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float l = bbox_red[0][a], h = bbox_red[0][3 + a];
    for (int q = 1; q < NW; ++q) { l = fminf(l, bbox_red[q][a]); h = fmaxf(h, bbox_red[q][3 + a]); }
    lo[a] = l;
    scale[a] = h > l ? (float)(1 << kCellBits) / (h - l) : 0.0f;
  }
  // ---- setup 2: counting sort by Morton cell (any order inside a cell: ties use original k)
  for (int k = t; k < N; k += BLOCK) {
    uint32_t q[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const int c = (int)((P[3 * k + a] - lo[a]) * scale[a]);
      q[a] = (uint32_t)min(max(c, 0), (1 << kCellBits) - 1);
    }
    const uint32_t code = spread3(q[0]) | (spread3(q[1]) << 1) | (spread3(q[2]) << 2);
    s_code[k] = (uint16_t)code;
    atomicAdd(&hist[code], 1u);
  }
  __syncthreads();
  {  // exclusive scan of hist[4096]: each thread owns kNumCodes/BLOCK consecutive entries
    constexpr int PER = kNumCodes / BLOCK;
    uint32_t loc[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int e = 0; e < PER; ++e) { loc[e] = hist[t * PER + e]; sum += loc[e]; }
    uint32_t incl = sum;  // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += y;
    }
    if (lane == kWave - 1) red[0][w].x = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int q = 0; q < w; ++q) base += red[0][q].x;
    uint32_t run = base + incl - sum;
#pragma unroll
    for (int e = 0; e < PER; ++e) { hist[t * PER + e] = run; run += loc[e]; }
  }
  __syncthreads();
  for (int k = t; k < N; k += BLOCK) s_sorted[atomicAdd(&hist[s_code[k]], 1u)] = (uint16_t)k;
  __syncthreads();

  // ---- setup 3: per-slot points in sorted order; per-cell boxes
  float px[PPT], py[PPT], pz[PPT];
  int tb[PPT];
  uint32_t tl[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int pos = w * (kWave * PPT) + i * kWave + lane;
    if (pos < N) {
      const int k = s_sorted[pos];
      px[i] = P[3 * k + 0];
      py[i] = P[3 * k + 1];
      pz[i] = P[3 * k + 2];
      tb[i] = __float_as_int(kInitTemp);
      tl[i] = tie_low(k);
    } else {  // padding: key (0, 0) never wins, min(d, 0) stays 0
      px[i] = py[i] = pz[i] = 0.0f;
      tb[i] = 0;
      tl[i] = 0u;
    }
  }
  float clo[NCELL][3], chi[NCELL][3];
  uint32_t ckm[NCELL], ckl[NCELL];
#pragma unroll
  for (int c = 0; c < NCELL; ++c) {
    float l0 = __builtin_inff(), l1 = l0, l2 = l0, h0 = -l0, h1 = -l0, h2 = -l0;
#pragma unroll
    for (int i = c * SUB; i < (c + 1) * SUB; ++i)
      if (tl[i] != 0u) {
        l0 = fminf(l0, px[i]); h0 = fmaxf(h0, px[i]);
        l1 = fminf(l1, py[i]); h1 = fmaxf(h1, py[i]);
        l2 = fminf(l2, pz[i]); h2 = fmaxf(h2, pz[i]);
      }
    clo[c][0] = uniform_f(wave_min_f(l0)); chi[c][0] = uniform_f(wave_max_f(h0));
    clo[c][1] = uniform_f(wave_min_f(l1)); chi[c][1] = uniform_f(wave_max_f(h1));
    clo[c][2] = uniform_f(wave_min_f(l2)); chi[c][2] = uniform_f(wave_max_f(h2));
    ckm[c] = 0u;
    ckl[c] = 0u;
  }
  __syncthreads();  // s_sorted is dead; smem_a becomes the xyz copy
  if constexpr (XYZ_LDS) {
    for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
    __syncthreads();
  }

  float cx = P[0], cy = P[1], cz = P[2];
  if (t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }
  bool first = true;
  for (int j = 1; j < M; ++j) {
    uint32_t wkm = 0u, wkl = 0u;
#pragma unroll
    for (int c = 0; c < NCELL; ++c) {
      // lower bound of the squared distance from c to the cell's box
      const float dx = fmaxf(fmaxf(clo[c][0] - cx, cx - chi[c][0]), 0.0f);
      const float dy = fmaxf(fmaxf(clo[c][1] - cy, cy - chi[c][1]), 0.0f);
      const float dz = fmaxf(fmaxf(clo[c][2] - cz, cz - chi[c][2]), 0.0f);
      const float lb = (dx * dx + dy * dy) + dz * dz;
      const float U = __uint_as_float(ckm[c]);
      const bool skip = !first && lb > 1e-30f && lb * 0.99998f > U;
      if (!skip) {
        uint32_t bh = 0u, bl = 0u;
#pragma unroll
        for (int i = c * SUB; i < (c + 1) * SUB; ++i) {
          const int v = min(__float_as_int(sqdist(px[i], py[i], pz[i], cx, cy, cz)), tb[i]);
          tb[i] = v;
          const uint64_t kv = pack64(tl[i], (uint32_t)v), kb = pack64(bl, bh);
          if (kv > kb) { bh = (uint32_t)v; bl = tl[i]; }
        }
        const uint32_t km = uniform_u32(wave_max_u32(bh));
        ckm[c] = km;
        ckl[c] = uniform_u32(wave_max_u32(bh == km ? bl : 0u));
      }
      if (ckm[c] > wkm || (ckm[c] == wkm && ckl[c] > wkl)) { wkm = ckm[c]; wkl = ckl[c]; }
    }
    first = false;
    uint32_t kl = wkl;
    if constexpr (NW > 1) {
      if (lane == 0) red[j & 1][w] = make_uint2(wkm, wkl);
      __syncthreads();
      const uint2 r = lane < NW ? red[j & 1][lane] : make_uint2(0u, 0u);
      const uint32_t km = row16_max_u32(r.x);
      kl = row16_max_u32(r.x == km ? r.y : 0u);
    }
    const int old = tie_decode(uniform_u32(kl));
    if constexpr (XYZ_LDS) {
      cx = sxyz[3 * old + 0]; cy = sxyz[3 * old + 1]; cz = sxyz[3 * old + 2];
    } else {
      cx = P[3 * old + 0]; cy = P[3 * old + 1]; cz = P[3 * old + 2];
    }
    if (t == 0) {
      I[j] = old;
      if (NX) { NX[3 * j + 0] = cx; NX[3 * j + 1] = cy; NX[3 * j + 2] = cz; }
    }
  }
}

// Variant 5: the iteration tail rebuilt for latency (optionally spatially culled as v3).
//  * per-lane key (running distance bits, tie word of the ORIGINAL index) compared as one u64,
//    so any slot order is exact; the lane also keeps the coordinates of its best point;
//  * wave argmax = one 32-bit max of the distance plus a ballot: when a single lane holds the
//    maximum (the common case) its tie word and coordinates are read with v_readlane; only a
//    real tie runs the second (tie-word) reduction;
//  * each wave publishes ONE 20-byte record {dist, tie, x, y, z} per iteration; after the
//    barrier every wave reduces the records of the 16-lane row and v_readlane's the winner's
//    coordinates: no dependent LDS lookup of the new centre.
template <int BLOCK, int PPT, int SUB, bool CULL>
__global__ __launch_bounds__(BLOCK) void fps_v5_kernel(const float* __restrict__ xyz, int N,
                                                       int M, int32_t* __restrict__ idx,
                                                       float* __restrict__ new_xyz) {
  constexpr int NW = BLOCK / kWave;
  constexpr int CAP = BLOCK * PPT;
  constexpr int NCELL = PPT / SUB;
  static_assert(NW <= 16 && PPT % SUB == 0, "config");
  __shared__ __attribute__((aligned(16))) uint16_t s_sort[CULL ? 2 * CAP : 2];
  __shared__ uint32_t hist[CULL ? kNumCodes : 1];
  __shared__ uint4 recA[2][16];
  __shared__ float recZ[2][16];
  __shared__ float bbox_red[16][6];
  __shared__ uint32_t scan_red[16];

  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  if constexpr (CULL) {  // counting sort by Morton cell (see fps_cull_kernel)
    uint16_t* s_code = s_sort;
    uint16_t* s_sorted = s_sort + CAP;
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    for (int k = t; k < N; k += BLOCK)
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const float v = P[3 * k + a];
        lo[a] = fminf(lo[a], v);
        hi[a] = fmaxf(hi[a], v);
      }
#pragma unroll
    for (int a = 0; a < 3; ++a) { lo[a] = wave_min_f(lo[a]); hi[a] = wave_max_f(hi[a]); }
    if (lane == 0)
#pragma unroll
      for (int a = 0; a < 3; ++a) { bbox_red[w][a] = lo[a]; bbox_red[w][3 + a] = hi[a]; }
    for (int e = t; e < kNumCodes; e += BLOCK) hist[e] = 0;
    __syncthreads();
    float scale[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      float l = bbox_red[0][a], h = bbox_red[0][3 + a];
      for (int q = 1; q < NW; ++q) { l = fminf(l, bbox_red[q][a]); h = fmaxf(h, bbox_red[q][3 + a]); }
      lo[a] = l;
      scale[a] = h > l ? (float)(1 << kCellBits) / (h - l) : 0.0f;
    }
    for (int k = t; k < N; k += BLOCK) {
      uint32_t q[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int c = (int)((P[3 * k + a] - lo[a]) * scale[a]);
        q[a] = (uint32_t)min(max(c, 0), (1 << kCellBits) - 1);
      }
      const uint32_t code = spread3(q[0]) | (spread3(q[1]) << 1) | (spread3(q[2]) << 2);
      s_code[k] = (uint16_t)code;
      atomicAdd(&hist[code], 1u);
    }
    __syncthreads();
    {
      constexpr int PER = kNumCodes / BLOCK;
      uint32_t loc[PER];
      uint32_t sum = 0;
#pragma unroll
      for (int e = 0; e < PER; ++e) { loc[e] = hist[t * PER + e]; sum += loc[e]; }
      uint32_t incl = sum;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, kWave);
        if (lane >= o) incl += y;
      }
      if (lane == kWave - 1) scan_red[w] = incl;
      __syncthreads();
      uint32_t base = 0;
      for (int q = 0; q < w; ++q) base += scan_red[q];
      uint32_t run = base + incl - sum;
#pragma unroll
      for (int e = 0; e < PER; ++e) { hist[t * PER + e] = run; run += loc[e]; }
    }
    __syncthreads();
    for (int k = t; k < N; k += BLOCK) s_sorted[atomicAdd(&hist[s_code[k]], 1u)] = (uint16_t)k;
    __syncthreads();
  }

  float px[PPT], py[PPT], pz[PPT];
  int tb[PPT];
  uint32_t tl[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    int k;
    if constexpr (CULL) {
      const int pos = w * (kWave * PPT) + i * kWave + lane;
      k = pos < N ? (int)s_sort[CAP + pos] : N;
    } else {
      k = t + slot_off<BLOCK, PPT>(i);
    }
    if (k < N) {
      px[i] = P[3 * k + 0];
      py[i] = P[3 * k + 1];
      pz[i] = P[3 * k + 2];
      tb[i] = __float_as_int(kInitTemp);
      tl[i] = tie_low(k);
    } else {  // padding: key (0, 0) never wins, min(d, 0) stays 0
      px[i] = py[i] = pz[i] = 0.0f;
      tb[i] = 0;
      tl[i] = 0u;
    }
  }
  float clo[NCELL][3], chi[NCELL][3];
  uint32_t ckm[NCELL], ckl[NCELL];
  float crx[NCELL], cry[NCELL], crz[NCELL];
#pragma unroll
  for (int c = 0; c < NCELL; ++c) {
    if constexpr (CULL) {
      float l0 = __builtin_inff(), l1 = l0, l2 = l0, h0 = -l0, h1 = -l0, h2 = -l0;
#pragma unroll
      for (int i = c * SUB; i < (c + 1) * SUB; ++i)
        if (tl[i] != 0u) {
          l0 = fminf(l0, px[i]); h0 = fmaxf(h0, px[i]);
          l1 = fminf(l1, py[i]); h1 = fmaxf(h1, py[i]);
          l2 = fminf(l2, pz[i]); h2 = fmaxf(h2, pz[i]);
        }
      clo[c][0] = uniform_f(wave_min_f(l0)); chi[c][0] = uniform_f(wave_max_f(h0));
      clo[c][1] = uniform_f(wave_min_f(l1)); chi[c][1] = uniform_f(wave_max_f(h1));
      clo[c][2] = uniform_f(wave_min_f(l2)); chi[c][2] = uniform_f(wave_max_f(h2));
    }
    ckm[c] = ckl[c] = 0u;
    crx[c] = cry[c] = crz[c] = 0.0f;
  }

  float cx = P[0], cy = P[1], cz = P[2];
  if (t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }
  bool first = true;
  for (int j = 1; j < M; ++j) {
    uint32_t wkm = 0u, wkl = 0u;
    float wx = 0.0f, wy = 0.0f, wz = 0.0f;
#pragma unroll
    for (int c = 0; c < NCELL; ++c) {
      bool skip = false;
      if constexpr (CULL) {
        const float dx = fmaxf(fmaxf(clo[c][0] - cx, cx - chi[c][0]), 0.0f);
        const float dy = fmaxf(fmaxf(clo[c][1] - cy, cy - chi[c][1]), 0.0f);
        const float dz = fmaxf(fmaxf(clo[c][2] - cz, cz - chi[c][2]), 0.0f);
        const float lb = (dx * dx + dy * dy) + dz * dz;
        skip = !first && lb > 1e-30f && lb * 0.99998f > __uint_as_float(ckm[c]);
      }
      if (!skip) {
        uint32_t bh = 0u, bl = 0u;
        int bi = c * SUB;
#pragma unroll
        for (int i = c * SUB; i < (c + 1) * SUB; ++i) {
          const int v = min(__float_as_int(sqdist(px[i], py[i], pz[i], cx, cy, cz)), tb[i]);
          tb[i] = v;
          if (pack64(tl[i], (uint32_t)v) > pack64(bl, bh)) { bh = (uint32_t)v; bl = tl[i]; bi = i; }
        }
        float bx = px[c * SUB], by = py[c * SUB], bz = pz[c * SUB];
#pragma unroll
        for (int i = c * SUB + 1; i < (c + 1) * SUB; ++i)
          if (bi == i) { bx = px[i]; by = py[i]; bz = pz[i]; }
        const uint32_t km = uniform_u32(wave_max_u32(bh));
        const uint64_t ball = __ballot(bh == km);
        uint32_t kl;
        int L;
        if (__popcll(ball) == 1) {
          L = __ffsll((unsigned long long)ball) - 1;
          kl = (uint32_t)__builtin_amdgcn_readlane((int)bl, L);
        } else {  // a real tie on the distance: smallest original-order tie key wins
          kl = uniform_u32(wave_max_u32(bh == km ? bl : 0u));
          L = __ffsll((unsigned long long)__ballot(bh == km && bl == kl)) - 1;
        }
        ckm[c] = km;
        ckl[c] = kl;
        crx[c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bx), L));
        cry[c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(by), L));
        crz[c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(bz), L));
      }
      if (ckm[c] > wkm || (ckm[c] == wkm && ckl[c] > wkl)) {
        wkm = ckm[c]; wkl = ckl[c]; wx = crx[c]; wy = cry[c]; wz = crz[c];
      }
    }
    first = false;
    uint32_t kl = wkl;
    if constexpr (NW > 1) {
      if (lane == 0) {
        recA[j & 1][w] = make_uint4(wkm, wkl, __float_as_uint(wx), __float_as_uint(wy));
        recZ[j & 1][w] = wz;
      }
      __syncthreads();
      const bool in = lane < NW;
      const uint4 r = in ? recA[j & 1][lane] : make_uint4(0u, 0u, 0u, 0u);
      const float rz = in ? recZ[j & 1][lane] : 0.0f;
      const uint32_t km = (uint32_t)__builtin_amdgcn_readlane((int)row16_max_u32(r.x), 0);
      const uint64_t ball = __ballot(in && r.x == km);
      int L;
      if (__popcll(ball) == 1) {
        L = __ffsll((unsigned long long)ball) - 1;
      } else {
        const uint32_t kt = (uint32_t)__builtin_amdgcn_readlane(
            (int)row16_max_u32(in && r.x == km ? r.y : 0u), 0);
        L = __ffsll((unsigned long long)__ballot(in && r.x == km && r.y == kt)) - 1;
      }
      kl = (uint32_t)__builtin_amdgcn_readlane((int)r.y, L);
      cx = __int_as_float(__builtin_amdgcn_readlane((int)r.z, L));
      cy = __int_as_float(__builtin_amdgcn_readlane((int)r.w, L));
      cz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rz), L));
    } else {
      cx = wx; cy = wy; cz = wz;
    }
    const int old = tie_decode(kl);
    if (t == 0) {
      I[j] = old;
      if (NX) { NX[3 * j + 0] = cx; NX[3 * j + 1] = cy; NX[3 * j + 2] = cz; }
    }
  }
}

// Variant 6: culled sampler with a short iteration tail (production path for large clouds).
//  * points counting-sorted by Morton cell as in v3; wave w owns PPT*64 consecutive sorted
//    points (a compact region) split into NCELL cells of SUB slots;
//  * every lane keeps, per cell, the best (running distance, tie word) of its slots, so a cell
//    that did not change needs no rescan and the wave needs ONE reduction per iteration — and
//    none at all when the new centre is provably too far from the wave's whole box
//    (wave-level skip); cells are skipped the same way inside an active wave. The skip bound is
//    the wave's max running distance U_w (>= every cell's), test lb*(1-2^-16) > U_w;
//  * argmax tie-breaks by ballot: a second reduction only when several lanes/waves share the
//    maximum distance;
//  * the winner's coordinates from an LDS copy of the cloud (one broadcast read);
//  * idx / new_xyz are collected in registers of wave 0 (lane = j mod 64, one select each) and
//    stored 64 at a time, instead of a masked global store per iteration.
template <int BLOCK, int PPT, int SUB, bool STAMP = false>
__global__ __launch_bounds__(BLOCK) void fps_v6_kernel(const float* __restrict__ xyz, int N,
                                                       int M, int32_t* __restrict__ idx,
                                                       float* __restrict__ new_xyz) {
  constexpr int NW = BLOCK / kWave;
  constexpr int CAP = BLOCK * PPT;
  constexpr int NCELL = PPT / SUB;
  constexpr bool XYZ_LDS = 12 * CAP + 4 * kNumCodes + 2048 <= 160 * 1024;
  static_assert(NW <= 16 && PPT % SUB == 0, "config");
  constexpr int A_BYTES = XYZ_LDS ? 12 * CAP : 4 * CAP;
  __shared__ __attribute__((aligned(16))) unsigned char smem_a[A_BYTES];
  __shared__ uint32_t hist[kNumCodes];
  __shared__ uint2 red[2][16];
  __shared__ float bbox_red[16][6];
  __shared__ uint32_t scan_red[16];
  uint16_t* s_code = reinterpret_cast<uint16_t*>(smem_a);
  uint16_t* s_sorted = s_code + CAP;
  float* sxyz = reinterpret_cast<float*>(smem_a);
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  if constexpr (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");

  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  // ---- setup: bounding box, counting sort by Morton cell
  {
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    for (int k = t; k < N; k += BLOCK)
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const float v = P[3 * k + a];
        lo[a] = fminf(lo[a], v);
        hi[a] = fmaxf(hi[a], v);
      }
#pragma unroll
    for (int a = 0; a < 3; ++a) { lo[a] = wave_min_f(lo[a]); hi[a] = wave_max_f(hi[a]); }
    if (lane == 0)
#pragma unroll
      for (int a = 0; a < 3; ++a) { bbox_red[w][a] = lo[a]; bbox_red[w][3 + a] = hi[a]; }
    for (int e = t; e < kNumCodes; e += BLOCK) hist[e] = 0;
    __syncthreads();
    float scale[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      float l = bbox_red[0][a], h = bbox_red[0][3 + a];
      for (int q = 1; q < NW; ++q) { l = fminf(l, bbox_red[q][a]); h = fmaxf(h, bbox_red[q][3 + a]); }
      lo[a] = l;
      scale[a] = h > l ? (float)(1 << kCellBits) / (h - l) : 0.0f;
    }
    for (int k = t; k < N; k += BLOCK) {
      uint32_t q[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int c = (int)((P[3 * k + a] - lo[a]) * scale[a]);
        q[a] = (uint32_t)min(max(c, 0), (1 << kCellBits) - 1);
      }
      const uint32_t code = spread3(q[0]) | (spread3(q[1]) << 1) | (spread3(q[2]) << 2);
      s_code[k] = (uint16_t)code;
      atomicAdd(&hist[code], 1u);
    }
    __syncthreads();
    constexpr int PER = kNumCodes / BLOCK;
    uint32_t loc[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int e = 0; e < PER; ++e) { loc[e] = hist[t * PER + e]; sum += loc[e]; }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += y;
    }
    if (lane == kWave - 1) scan_red[w] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int q = 0; q < w; ++q) base += scan_red[q];
    uint32_t run = base + incl - sum;
#pragma unroll
    for (int e = 0; e < PER; ++e) { hist[t * PER + e] = run; run += loc[e]; }
    __syncthreads();
    for (int k = t; k < N; k += BLOCK) s_sorted[atomicAdd(&hist[s_code[k]], 1u)] = (uint16_t)k;
    __syncthreads();
  }

  float px[PPT], py[PPT], pz[PPT];
  int tb[PPT];
  uint32_t tl[PPT];
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int pos = w * (kWave * PPT) + i * kWave + lane;
    const int k = pos < N ? (int)s_sorted[pos] : N;
    if (k < N) {
      px[i] = P[3 * k + 0];
      py[i] = P[3 * k + 1];
      pz[i] = P[3 * k + 2];
      tb[i] = __float_as_int(kInitTemp);
      tl[i] = tie_low(k);
    } else {  // padding: key (0, 0) never wins, min(d, 0) stays 0
      px[i] = py[i] = pz[i] = 0.0f;
      tb[i] = 0;
      tl[i] = 0u;
    }
  }
  // per-cell boxes (wave-uniform) and the wave's box
  float clo[NCELL][3], chi[NCELL][3], wlo[3], whi[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) { wlo[a] = __builtin_inff(); whi[a] = -__builtin_inff(); }
#pragma unroll
  for (int c = 0; c < NCELL; ++c) {
    float l0 = __builtin_inff(), l1 = l0, l2 = l0, h0 = -l0, h1 = -l0, h2 = -l0;
#pragma unroll
    for (int i = c * SUB; i < (c + 1) * SUB; ++i)
      if (tl[i] != 0u) {
        l0 = fminf(l0, px[i]); h0 = fmaxf(h0, px[i]);
        l1 = fminf(l1, py[i]); h1 = fmaxf(h1, py[i]);
        l2 = fminf(l2, pz[i]); h2 = fmaxf(h2, pz[i]);
      }
    clo[c][0] = uniform_f(wave_min_f(l0)); chi[c][0] = uniform_f(wave_max_f(h0));
    clo[c][1] = uniform_f(wave_min_f(l1)); chi[c][1] = uniform_f(wave_max_f(h1));
    clo[c][2] = uniform_f(wave_min_f(l2)); chi[c][2] = uniform_f(wave_max_f(h2));
#pragma unroll
    for (int a = 0; a < 3; ++a) { wlo[a] = fminf(wlo[a], clo[c][a]); whi[a] = fmaxf(whi[a], chi[c][a]); }
  }
  __syncthreads();  // s_sorted is dead; smem_a becomes the xyz copy
  if constexpr (XYZ_LDS) {
    for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
    __syncthreads();
  }

  uint32_t cbh[NCELL], cbl[NCELL];  // per lane, per cell: best (distance bits, tie word)
#pragma unroll
  for (int c = 0; c < NCELL; ++c) cbh[c] = cbl[c] = 0u;
  uint32_t wkm = 0u, wkl = 0u;       // the wave's record (uniform)
  float cx = P[0], cy = P[1], cz = P[2];
  int ring_i = 0;                    // wave 0: idx / new_xyz of 64 iterations, lane = j & 63
  float ring_x = cx, ring_y = cy, ring_z = cz;
  PN2_STAMP(5)

  for (int j = 1; j < M; ++j) {
    if constexpr (STAMP) {
      if (t == 0 && j < 4096) g_iter[j] = st_prev;
    }
    const bool first = j == 1;
    const float Uw = __uint_as_float(wkm);
    auto far_box = [&](const float* lo, const float* hi) {
      const float dx = fmaxf(fmaxf(lo[0] - cx, cx - hi[0]), 0.0f);
      const float dy = fmaxf(fmaxf(lo[1] - cy, cy - hi[1]), 0.0f);
      const float dz = fmaxf(fmaxf(lo[2] - cz, cz - hi[2]), 0.0f);
      const float lb = (dx * dx + dy * dy) + dz * dz;
      return !first && lb > 1e-30f && lb * 0.99998f > Uw;
    };
    if (!far_box(wlo, whi)) {
#pragma unroll
      for (int c = 0; c < NCELL; ++c) {
        if (far_box(clo[c], chi[c])) continue;
        uint32_t bh = 0u, bl = 0u;
#pragma unroll
        for (int i = c * SUB; i < (c + 1) * SUB; ++i) {
          const int v = min(__float_as_int(sqdist(px[i], py[i], pz[i], cx, cy, cz)), tb[i]);
          tb[i] = v;
          if (pack64(tl[i], (uint32_t)v) > pack64(bl, bh)) { bh = (uint32_t)v; bl = tl[i]; }
        }
        cbh[c] = bh;
        cbl[c] = bl;
      }
      PN2_STAMP(0)
      uint32_t bh = cbh[0], bl = cbl[0];
#pragma unroll
      for (int c = 1; c < NCELL; ++c)
        if (pack64(cbl[c], cbh[c]) > pack64(bl, bh)) { bh = cbh[c]; bl = cbl[c]; }
      wkm = uniform_u32(wave_max_u32(bh));
      const uint64_t ball = __ballot(bh == wkm);
      if (__popcll(ball) == 1)
        wkl = (uint32_t)__builtin_amdgcn_readlane((int)bl, __ffsll((unsigned long long)ball) - 1);
      else
        wkl = uniform_u32(wave_max_u32(bh == wkm ? bl : 0u));
      PN2_STAMP(1)
    }
    uint32_t kl = wkl;
    if constexpr (NW > 1) {
      if (lane == 0) red[j & 1][w] = make_uint2(wkm, wkl);
      __syncthreads();
      PN2_STAMP(2)
      const bool in = lane < NW;
      const uint2 r = in ? red[j & 1][lane] : make_uint2(0u, 0u);
      const uint32_t km = (uint32_t)__builtin_amdgcn_readlane((int)row16_max_u32(r.x), 0);
      const uint64_t ball = __ballot(in && r.x == km);
      if (__popcll(ball) == 1)
        kl = (uint32_t)__builtin_amdgcn_readlane((int)r.y, __ffsll((unsigned long long)ball) - 1);
      else
        kl = (uint32_t)__builtin_amdgcn_readlane(
            (int)row16_max_u32(in && r.x == km ? r.y : 0u), 0);
    }
    const int old = tie_decode(kl);
    PN2_STAMP(3)
    if constexpr (XYZ_LDS) {
      cx = sxyz[3 * old + 0]; cy = sxyz[3 * old + 1]; cz = sxyz[3 * old + 2];
    } else {
      cx = P[3 * old + 0]; cy = P[3 * old + 1]; cz = P[3 * old + 2];
    }
    PN2_STAMP(4)
    if (w == 0) {  // wave-uniform: ring of the last 64 results, flushed when full
      const int sl = j & (kWave - 1);
      const bool mine = lane == sl;
      ring_i = mine ? old : ring_i;
      ring_x = mine ? cx : ring_x;
      ring_y = mine ? cy : ring_y;
      ring_z = mine ? cz : ring_z;
      if (sl == kWave - 1 || j == M - 1) {
        const int jj = (j & ~(kWave - 1)) + lane;
        if (lane <= sl) {
          I[jj] = ring_i;
          if (NX) { NX[3 * jj] = ring_x; NX[3 * jj + 1] = ring_y; NX[3 * jj + 2] = ring_z; }
        }
      }
    }
    PN2_STAMP(5)
  }
  if (M == 1 && t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x < 16)
      for (int ph = 0; ph < 6; ++ph) g_stamp[(blockIdx.x * 16 + w) * 8 + ph] = st_acc[ph];
  }
}

// Variant 8: culled sampler with the culled work spread over the SIMDs.
//  * points counting-sorted by Morton cell (v3 setup); a "cell" is 64 consecutive sorted points
//    = one slot of one wave, and cells are dealt round-robin (cell g -> wave g % NW, slot
//    g / NW), so the few cells near the new centre land in DIFFERENT waves / SIMDs;
//  * lane i of a wave holds the box of the wave's slot i, so all its slots are tested at once
//    (lb*(1-2^-16) > U_w, U_w = the wave's max running distance) and a ballot gives the
//    active slots; only those are rescanned (uniform scalar branches per slot);
//  * argmax: one 32-bit wave max, then the lanes holding it ds_max_u64 their (distance, tie)
//    key into a triple-buffered LDS word (v7) — inactive waves re-offer their unchanged best
//    the same way; after the barrier one LDS read gives the winner.
template <int BLOCK, int PPT, bool STAMP = false>
__global__ __launch_bounds__(BLOCK) void fps_v8_kernel(const float* __restrict__ xyz, int N,
                                                       int M, int32_t* __restrict__ idx,
                                                       float* __restrict__ new_xyz) {
  constexpr int NW = BLOCK / kWave;
  constexpr int CAP = BLOCK * PPT;
  static_assert(NW <= 16 && PPT <= kWave, "config");
  constexpr bool XYZ_LDS = 12 * CAP + 4 * kNumCodes + 1024 <= 160 * 1024;
  constexpr int A_BYTES = XYZ_LDS ? 12 * CAP : 4 * CAP;
  __shared__ __attribute__((aligned(16))) unsigned char smem_a[A_BYTES];
  __shared__ uint32_t hist[kNumCodes];
  __shared__ uint2 red[2][16];
  __shared__ float bbox_red[16][6];
  __shared__ uint32_t scan_red[16];
  uint16_t* s_code = reinterpret_cast<uint16_t*>(smem_a);
  uint16_t* s_sorted = s_code + CAP;
  float* sxyz = reinterpret_cast<float*>(smem_a);
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;

  const int b = blockIdx.x;
  const int t = threadIdx.x;
  const int lane = t & (kWave - 1);
  const int w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;

  {  // setup: cloud box, counting sort by 12-bit Morton cell
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    for (int k = t; k < N; k += BLOCK)
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const float v = P[3 * k + a];
        lo[a] = fminf(lo[a], v);
        hi[a] = fmaxf(hi[a], v);
      }
#pragma unroll
    for (int a = 0; a < 3; ++a) { lo[a] = wave_min_f(lo[a]); hi[a] = wave_max_f(hi[a]); }
    if (lane == 0)
#pragma unroll
      for (int a = 0; a < 3; ++a) { bbox_red[w][a] = lo[a]; bbox_red[w][3 + a] = hi[a]; }
    for (int e = t; e < kNumCodes; e += BLOCK) hist[e] = 0;
    __syncthreads();
    float scale[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      float l = bbox_red[0][a], h = bbox_red[0][3 + a];
      for (int q = 1; q < NW; ++q) { l = fminf(l, bbox_red[q][a]); h = fmaxf(h, bbox_red[q][3 + a]); }
      lo[a] = l;
      scale[a] = h > l ? (float)(1 << kCellBits) / (h - l) : 0.0f;
    }
    for (int k = t; k < N; k += BLOCK) {
      uint32_t q[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int c = (int)((P[3 * k + a] - lo[a]) * scale[a]);
        q[a] = (uint32_t)min(max(c, 0), (1 << kCellBits) - 1);
      }
      const uint32_t code = spread3(q[0]) | (spread3(q[1]) << 1) | (spread3(q[2]) << 2);
      s_code[k] = (uint16_t)code;
      atomicAdd(&hist[code], 1u);
    }
    __syncthreads();
    constexpr int PER = kNumCodes / BLOCK;
    uint32_t loc[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int e = 0; e < PER; ++e) { loc[e] = hist[t * PER + e]; sum += loc[e]; }
    uint32_t incl = sum;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += y;
    }
    if (lane == kWave - 1) scan_red[w] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int q = 0; q < w; ++q) base += scan_red[q];
    uint32_t run = base + incl - sum;
#pragma unroll
    for (int e = 0; e < PER; ++e) { hist[t * PER + e] = run; run += loc[e]; }
    __syncthreads();
    for (int k = t; k < N; k += BLOCK) s_sorted[atomicAdd(&hist[s_code[k]], 1u)] = (uint16_t)k;
    __syncthreads();
  }

  float px[PPT], py[PPT], pz[PPT];
  int tb[PPT];
  uint32_t tl[PPT];
  float blx = __builtin_inff(), bly = blx, blz = blx, bhx = -blx, bhy = -blx, bhz = -blx;
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int pos = (i * NW + w) * kWave + lane;  // cell i*NW + w
    const int k = pos < N ? (int)s_sorted[pos] : N;
    float l0 = __builtin_inff(), l1 = l0, l2 = l0, h0 = -l0, h1 = -l0, h2 = -l0;
    if (k < N) {
      px[i] = P[3 * k + 0];
      py[i] = P[3 * k + 1];
      pz[i] = P[3 * k + 2];
      tb[i] = __float_as_int(kInitTemp);
      tl[i] = tie_low(k);
      l0 = h0 = px[i]; l1 = h1 = py[i]; l2 = h2 = pz[i];
    } else {  // padding: key (0, 0) never wins, min(d, 0) stays 0
      px[i] = py[i] = pz[i] = 0.0f;
      tb[i] = 0;
      tl[i] = 0u;
    }
    l0 = wave_min_f(l0); l1 = wave_min_f(l1); l2 = wave_min_f(l2);
    h0 = wave_max_f(h0); h1 = wave_max_f(h1); h2 = wave_max_f(h2);
    if (lane == i) { blx = l0; bly = l1; blz = l2; bhx = h0; bhy = h1; bhz = h2; }
  }
  __syncthreads();  // s_sorted is dead; smem_a becomes the xyz copy
  if constexpr (XYZ_LDS) {
    for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
    __syncthreads();
  }

  uint32_t bh = 0u, bl = 0u;  // this lane's best over its slots
  uint32_t wkm = 0u, wkl = 0u;  // the wave's best (uniform)
  float cx = P[0], cy = P[1], cz = P[2];
  int ring_i = 0;
  float ring_x = cx, ring_y = cy, ring_z = cz;
  constexpr uint64_t kSlotMask = PPT >= 64 ? ~0ull : ((1ull << PPT) - 1);
  if constexpr (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
  for (int j = 1; j < M; ++j) {
    // lane-parallel test of the wave's slots (lane i <-> slot i)
    const float dx = fmaxf(fmaxf(blx - cx, cx - bhx), 0.0f);
    const float dy = fmaxf(fmaxf(bly - cy, cy - bhy), 0.0f);
    const float dz = fmaxf(fmaxf(blz - cz, cz - bhz), 0.0f);
    const float lb = (dx * dx + dy * dy) + dz * dz;
    const bool far = j > 1 && lb > 1e-30f && lb * 0.99998f > __uint_as_float(wkm);
    const uint64_t active = __ballot(!far) & kSlotMask;
    if (active) {
#pragma unroll
      for (int i = 0; i < PPT; ++i)
        if ((active >> i) & 1ull)
          tb[i] = min(__float_as_int(sqdist(px[i], py[i], pz[i], cx, cy, cz)), tb[i]);
      bh = 0u; bl = 0u;
#pragma unroll
      for (int i = 0; i < PPT; ++i)
        if (pack64(tl[i], (uint32_t)tb[i]) > pack64(bl, bh)) { bh = (uint32_t)tb[i]; bl = tl[i]; }
      wkm = uniform_u32(wave_max_u32(bh));
    }
    PN2_STAMP(0)
    if (active) {  // the wave's tie word (only when the wave changed)
      const uint64_t ball = __ballot(bh == wkm);
      if (__popcll(ball) == 1)
        wkl = (uint32_t)__builtin_amdgcn_readlane((int)bl, __ffsll((unsigned long long)ball) - 1);
      else
        wkl = uniform_u32(wave_max_u32(bh == wkm ? bl : 0u));
    }
    PN2_STAMP(1)
    uint32_t kl = wkl;
    if constexpr (NW > 1) {
      if (lane == 0) red[j & 1][w] = make_uint2(wkm, wkl);
      __syncthreads();
      PN2_STAMP(2)
      const bool in = lane < NW;
      const uint2 r = in ? red[j & 1][lane] : make_uint2(0u, 0u);
      const uint32_t km = (uint32_t)__builtin_amdgcn_readlane((int)row16_max_u32(r.x), 0);
      const uint64_t ball = __ballot(in && r.x == km);
      if (__popcll(ball) == 1)
        kl = (uint32_t)__builtin_amdgcn_readlane((int)r.y, __ffsll((unsigned long long)ball) - 1);
      else
        kl = (uint32_t)__builtin_amdgcn_readlane((int)row16_max_u32(in && r.x == km ? r.y : 0u), 0);
    }
    const int old = tie_decode(kl);
    PN2_STAMP(3)
    if constexpr (XYZ_LDS) {
      cx = sxyz[3 * old + 0]; cy = sxyz[3 * old + 1]; cz = sxyz[3 * old + 2];
    } else {
      cx = P[3 * old + 0]; cy = P[3 * old + 1]; cz = P[3 * old + 2];
    }
    PN2_STAMP(4)
    {
      const int sl = j & (kWave - 1);
      const bool mine = lane == sl;
      ring_i = mine ? old : ring_i;
      ring_x = mine ? cx : ring_x;
      ring_y = mine ? cy : ring_y;
      ring_z = mine ? cz : ring_z;
      if ((sl == kWave - 1 || j == M - 1) && w == 0) {
        const int jj = (j & ~(kWave - 1)) + lane;
        if (lane <= sl) {
          I[jj] = ring_i;
          if (NX) { NX[3 * jj] = ring_x; NX[3 * jj + 1] = ring_y; NX[3 * jj + 2] = ring_z; }
        }
      }
    }
    PN2_STAMP(5)
  }
  if (M == 1 && t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }
  if constexpr (STAMP) {
    if (lane == 0 && blockIdx.x < 16)
      for (int ph = 0; ph < 6; ++ph) g_stamp[(blockIdx.x * 16 + w) * 8 + ph] = st_acc[ph];
  }
}

// The LDS copy of the cloud (12 B per point) is used whenever it fits next to the key slots
// in the 160 KiB of one CU; otherwise the winner's xyz is re-read from global memory.
template <int BLOCK, int PPT>
void launch_reg(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s) {
  if constexpr (3 * BLOCK * PPT * 4 + 256 <= 160 * 1024)
    hipLaunchKernelGGL((fps_reg_kernel<BLOCK, PPT, true>), dim3(B), dim3(BLOCK), 0, s, xyz, N, M,
                       idx, nx);
  else
    hipLaunchKernelGGL((fps_reg_kernel<BLOCK, PPT, false>), dim3(B), dim3(BLOCK), 0, s, xyz, N,
                       M, idx, nx);
}

// Variant 12 (cells): work skipping that keeps every wave equally busy. The cloud is sorted by
// a coarse Morton code (4 bits per axis, counting sort in LDS) and dealt round-robin to the 256
// threads, so slot s of EVERY thread holds one compact cell of 256 points (cell s). Per
// iteration the new centre c and the current global maximum D (the previous winner's
// distance: every running min is <= D) decide per cell, uniformly: if the cell's bounding box
// is at least D away from c (with a 2^-16 relative margin against fp32 rounding), no point of
// the cell can lower its running min, and the slot is skipped by all threads at once. Points
// are no longer in the reference's tie order, so each slot carries its tie key
// (k mod 512, k div 512) explicitly; the argmax is (max d, then min key). The lane maximum is
// kept per group of 4 slots and only groups with a scanned slot are re-reduced.
constexpr int kV12Cells = 32;
constexpr int kV12Buckets = 4096;

PN2_DEV uint32_t v12_ord(float f) {  // order-preserving float -> uint map
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
PN2_DEV float v12_unord(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}
PN2_DEV float v12_wave_max(float v) { return v12_unord(wave_max_u32(v12_ord(v))); }
PN2_DEV float v12_wave_min(float v) { return v12_unord(~wave_max_u32(~v12_ord(v))); }
PN2_DEV uint32_t v12_spread4(uint32_t v) {  // 4 bits -> every third bit
  v &= 15u;
  return (v & 1u) | ((v & 2u) << 2) | ((v & 4u) << 4) | ((v & 8u) << 6);
}

__global__ __launch_bounds__(256) void fps_v12_kernel(const float* __restrict__ xyz, int N, int M,
                                                      int32_t* __restrict__ idx,
                                                      float* __restrict__ new_xyz) {
  constexpr int BLOCK = 256, PPT = kV12Cells, NP = BLOCK * PPT, NW = BLOCK / kWave;
  constexpr int NG = PPT / 4;
  __shared__ float sxyz[3 * NP];
  __shared__ int hist[kV12Buckets + 1];
  __shared__ unsigned short order[NP];
  __shared__ unsigned short code[NP];
  __shared__ float wbox[NW][PPT][6];
  __shared__ float sbb[NW][6];
  __shared__ int wsum[NW];
  __shared__ uint2 red[2][8];
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)blockIdx.x * N * 3;
  int32_t* I = idx + (size_t)blockIdx.x * M;
  float* NX = new_xyz ? new_xyz + (size_t)blockIdx.x * M * 3 : nullptr;

  for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
  for (int e = t; e <= kV12Buckets; e += BLOCK) hist[e] = 0;
  __syncthreads();
  // bounding box of the cloud
  float lo[3] = {3e38f, 3e38f, 3e38f}, hi[3] = {-3e38f, -3e38f, -3e38f};
  for (int k = t; k < N; k += BLOCK)
    for (int a = 0; a < 3; ++a) {
      lo[a] = fminf(lo[a], sxyz[3 * k + a]);
      hi[a] = fmaxf(hi[a], sxyz[3 * k + a]);
    }
  for (int a = 0; a < 3; ++a) {
    lo[a] = v12_wave_min(lo[a]);
    hi[a] = v12_wave_max(hi[a]);
  }
  if (lane == 0)
    for (int a = 0; a < 3; ++a) { sbb[w][a] = lo[a]; sbb[w][3 + a] = hi[a]; }
  __syncthreads();
  float sc[3];
  for (int a = 0; a < 3; ++a) {
    float l = sbb[0][a], h = sbb[0][3 + a];
    for (int q = 1; q < NW; ++q) { l = fminf(l, sbb[q][a]); h = fmaxf(h, sbb[q][3 + a]); }
    lo[a] = l;
    sc[a] = 16.f / fmaxf(h - l, 1e-30f);
  }
  // coarse Morton codes, counting sort: order[] = point indices by cell-major position
  for (int k = t; k < NP; k += BLOCK) {
    uint32_t m = kV12Buckets;  // padding slots sort last
    if (k < N) {
      m = 0;
      for (int a = 0; a < 3; ++a) {
        const int q = min(15, max(0, (int)((sxyz[3 * k + a] - lo[a]) * sc[a])));
        m |= v12_spread4((uint32_t)q) << a;
      }
    }
    code[k] = (unsigned short)m;
    atomicAdd(&hist[m], 1);
  }
  __syncthreads();
  {  // exclusive scan of hist[0..4096]: 16 buckets per thread, the last one by thread 255
    int loc[16], sum = 0;
    for (int i = 0; i < 16; ++i) { loc[i] = hist[16 * t + i]; sum += loc[i]; }
    int incl = sum;
    for (int o = 1; o < kWave; o <<= 1) {
      const int v = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += v;
    }
    if (lane == kWave - 1) wsum[w] = incl;
    __syncthreads();
    int base = 0;
    for (int q = 0; q < w; ++q) base += wsum[q];
    int run = base + incl - sum;
    for (int i = 0; i < 16; ++i) { hist[16 * t + i] = run; run += loc[i]; }
    if (t == BLOCK - 1) hist[kV12Buckets] = run;
  }
  __syncthreads();
  for (int k = t; k < NP; k += BLOCK) order[atomicAdd(&hist[code[k]], 1)] = (unsigned short)k;
  __syncthreads();

  // slot s of thread t: the point at cell-major position s * 256 + t
  float px[PPT], py[PPT], pz[PPT];
  int tb[PPT], tk[PPT];
#pragma unroll
  for (int s = 0; s < PPT; ++s) {
    const int k = order[s * BLOCK + t];
    const bool in = k < N;
    const int kk = in ? k : 0;
    px[s] = sxyz[3 * kk];
    py[s] = sxyz[3 * kk + 1];
    pz[s] = sxyz[3 * kk + 2];
    tb[s] = in ? __float_as_int(kInitTemp) : -1;
    tk[s] = in ? (((k & 511) << 4) | (k >> 9)) : 0x7FFFFFFF;
  }
  // cell boxes: lane c (and c + 32) of every wave keeps cell c's box
#pragma unroll
  for (int s = 0; s < PPT; ++s) {
    const float a0 = v12_wave_min(px[s]), a1 = v12_wave_min(py[s]), a2 = v12_wave_min(pz[s]);
    const float b0 = v12_wave_max(px[s]), b1 = v12_wave_max(py[s]), b2 = v12_wave_max(pz[s]);
    if (lane == 0) {
      wbox[w][s][0] = a0; wbox[w][s][1] = a1; wbox[w][s][2] = a2;
      wbox[w][s][3] = b0; wbox[w][s][4] = b1; wbox[w][s][5] = b2;
    }
  }
  __syncthreads();
  float blo[3], bhi[3];
  {
    const int c = lane & (PPT - 1);
    for (int a = 0; a < 3; ++a) {
      float l = wbox[0][c][a], h = wbox[0][c][3 + a];
      for (int q = 1; q < NW; ++q) { l = fminf(l, wbox[q][c][a]); h = fmaxf(h, wbox[q][c][3 + a]); }
      blo[a] = l;
      bhi[a] = h;
    }
  }
  // per-group cache of the lane's (max, min key among the max)
  int gm[NG], gk[NG];
  auto regroup = [&](int g) {
    const int m = max(max(tb[4 * g], tb[4 * g + 1]), max(tb[4 * g + 2], tb[4 * g + 3]));
    int key = 0x7FFFFFFF;
#pragma unroll
    for (int q = 0; q < 4; ++q) key = (tb[4 * g + q] == m) ? min(key, tk[4 * g + q]) : key;
    gm[g] = m;
    gk[g] = key;
  };
#pragma unroll
  for (int g = 0; g < NG; ++g) regroup(g);

  float cx = sxyz[0], cy = sxyz[1], cz = sxyz[2];
  float D = kInitTemp;
  if (t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }
  constexpr float kMargin = 1.0f - 1.0f / 65536.0f;
  for (int j = 1; j < M; ++j) {
    // which cells can change: box distance below the global max D (lanes 0..31 = cells)
    float lb2;
    {
      const float gx = fmaxf(fmaxf(blo[0] - cx, cx - bhi[0]), 0.f);
      const float gy = fmaxf(fmaxf(blo[1] - cy, cy - bhi[1]), 0.f);
      const float gz = fmaxf(fmaxf(blo[2] - cz, cz - bhi[2]), 0.f);
      lb2 = (gx * gx + gy * gy) + gz * gz;
    }
    const uint32_t mask = (uint32_t)__builtin_amdgcn_ballot_w64(!(lb2 * kMargin >= D));
#pragma unroll
    for (int s = 0; s < PPT; ++s) {
      if (mask & (1u << s)) {
        const float dx = px[s] - cx, dy = py[s] - cy, dz = pz[s] - cz;
        const float d = (dx * dx + dy * dy) + dz * dz;
        tb[s] = min(tb[s], __float_as_int(d));
      }
    }
#pragma unroll
    for (int g = 0; g < NG; ++g)
      if (mask & (0xFu << (4 * g))) regroup(g);
    int bd = gm[0];
#pragma unroll
    for (int g = 1; g < NG; ++g) bd = max(bd, gm[g]);
    int bk = 0x7FFFFFFF;
#pragma unroll
    for (int g = 0; g < NG; ++g) bk = (gm[g] == bd) ? min(bk, gk[g]) : bk;
    // wave: max distance, then the smallest key among the lanes holding it
    const uint32_t hv = (uint32_t)(bd + 1);
    const uint32_t km = wave_max_u32(hv);
    const uint64_t cand = __builtin_amdgcn_ballot_w64(hv == km);
    uint32_t key;
    if (__builtin_popcountll(cand) == 1) {
      key = (uint32_t)__builtin_amdgcn_readlane(bk, (int)__builtin_ctzll(cand));
    } else {
      const uint32_t kk = (hv == km) ? (uint32_t)bk : 0xFFFFFFFFu;
      key = ~wave_max_u32(~kk);
    }
    if (lane == 0) red[j & 1][w] = make_uint2(km, key);
    __syncthreads();
    const bool inw = (lane & 7) < NW;
    const uint2 r = inw ? red[j & 1][lane & 7] : make_uint2(0u, 0xFFFFFFFFu);
    uint32_t bm = max_dpp_u32<kDppXor1>(r.x);
    bm = max_dpp_u32<kDppXor2>(bm);
    bm = max_dpp_u32<kDppHalfMirror>(bm);
    const uint64_t wins = __builtin_amdgcn_ballot_w64(r.x == bm) & 0xFFull;
    uint32_t bkey;
    if (__builtin_popcountll(wins) == 1) {
      bkey = (uint32_t)__builtin_amdgcn_readlane((int)r.y, (int)__builtin_ctzll(wins));
    } else {
      uint32_t kk = ~((r.x == bm) ? r.y : 0xFFFFFFFFu);
      kk = max_dpp_u32<kDppXor1>(kk);
      kk = max_dpp_u32<kDppXor2>(kk);
      kk = max_dpp_u32<kDppHalfMirror>(kk);
      bkey = ~(uint32_t)__builtin_amdgcn_readfirstlane((int)kk);
    }
    const int old = (int)((bkey & 15u) * 512u + (bkey >> 4));
    D = __int_as_float((int)bm - 1);
    cx = sxyz[3 * old];
    cy = sxyz[3 * old + 1];
    cz = sxyz[3 * old + 2];
    if (t == 0) {
      I[j] = old;
      if (NX) { NX[3 * j] = cx; NX[3 * j + 1] = cy; NX[3 * j + 2] = cz; }
    }
  }
}


// (variant, block, points-per-thread) launch table used by the tuner (pn2_fps_tune)
#define PN2_FPS_CONFIGS(X)                                                                      \
  X(64, 1) X(64, 2) X(64, 4) X(64, 8) X(64, 16) X(128, 4) X(128, 8) X(128, 16) X(256, 1)      \
  X(256, 2) X(256, 4) X(256, 8) X(256, 16) X(512, 2) X(512, 4) X(512, 8) X(512, 16)           \
  X(1024, 1) X(1024, 2) X(1024, 4) X(1024, 8) X(1024, 16)

template <int BLOCK, int PPT, int SUB>
void launch_cull(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s) {
  if constexpr (12 * BLOCK * PPT + 4 * 4096 + 1024 <= 160 * 1024)
    hipLaunchKernelGGL((fps_cull_kernel<BLOCK, PPT, SUB, true>), dim3(B), dim3(BLOCK), 0, s, xyz,
                       N, M, idx, nx);
  else
    hipLaunchKernelGGL((fps_cull_kernel<BLOCK, PPT, SUB, false>), dim3(B), dim3(BLOCK), 0, s,
                       xyz, N, M, idx, nx);
}

template <int BLOCK, int PPT, int SUB, bool CULL>
void launch_v5(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s) {
  hipLaunchKernelGGL((fps_v5_kernel<BLOCK, PPT, SUB, CULL>), dim3(B), dim3(BLOCK), 0, s, xyz, N,
                     M, idx, nx);
}

template <int BLOCK, int PPT, int SUB>
void launch_v6(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s) {
  hipLaunchKernelGGL((fps_v6_kernel<BLOCK, PPT, SUB>), dim3(B), dim3(BLOCK), 0, s, xyz, N, M, idx,
                     nx);
}

template <int BLOCK, int PPT>
void launch_v7(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s) {
  hipLaunchKernelGGL((fps_v7_kernel<BLOCK, PPT>), dim3(B), dim3(BLOCK), 0, s, xyz, N, M, idx, nx);
}

template <int BLOCK, int PPT>
void launch_v8(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, hipStream_t s) {
  hipLaunchKernelGGL((fps_v8_kernel<BLOCK, PPT>), dim3(B), dim3(BLOCK), 0, s, xyz, N, M, idx, nx);
}

int fps_tune_impl(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, int variant,
                  int block, int ppt, hipStream_t s) {
  if (B <= 0 || N <= 0 || M <= 0 || block * ppt < N) return PN2_EINVAL;
#define PN2_X(BL, PP)                                              \
  if (block == BL && ppt == PP && (variant == 1 || variant == 2)) {\
    if (variant == 1) launch_reg<BL, PP>(xyz, B, N, M, idx, nx, s); \
    else if (variant == 2) launch_v2<BL, PP>(xyz, B, N, M, idx, nx, s); \
    if (variant == 1 || variant == 2) PN2_RETURN_LAUNCH();         \
    return PN2_EINVAL;                                             \
  }
  PN2_FPS_CONFIGS(PN2_X)
#undef PN2_X
  if (variant == 120) {  // v12 cells: 256 threads x 32 slots, N <= 8192
    if (block != 256 || ppt != 32 || N > 8192) return PN2_EINVAL;
    hipLaunchKernelGGL(fps_v12_kernel, dim3(B), dim3(256), 0, s, xyz, N, M, idx, nx);
    PN2_RETURN_LAUNCH();
  }
  if (variant >= 111 && variant <= 114) {  // v11, variant = 110 + G
    const int G = variant - 110;
#define PN2_V11(BL, PP, GG)                                                    \
    if (block == BL && ppt == PP && G == GG) {                                 \
      launch_v11<BL, PP, GG>(xyz, B, N, M, idx, nx, s);                        \
      PN2_RETURN_LAUNCH();                                                     \
    }
    PN2_V11(64, 1, 1) PN2_V11(64, 2, 2) PN2_V11(64, 4, 4) PN2_V11(64, 8, 4) PN2_V11(256, 4, 4)
    PN2_V11(256, 8, 4) PN2_V11(256, 16, 4) PN2_V11(256, 32, 4) PN2_V11(512, 16, 4)
    PN2_V11(512, 32, 4) PN2_V11(128, 8, 4) PN2_V11(64, 16, 4) PN2_V11(128, 4, 4)
    PN2_V11(256, 32, 2) PN2_V11(512, 16, 2) PN2_V11(256, 64, 4)
#undef PN2_V11
  }
  if (variant == 97 || variant == 98) {  // v9 lane resolve + atomic block step (G = 4 / 2)
    const int G = variant == 97 ? 4 : 2;
#define PN2_V9A(BL, PP, GG)                                                    \
    if (block == BL && ppt == PP && G == GG) {                                 \
      launch_v9<BL, PP, GG, true, true>(xyz, B, N, M, idx, nx, s);             \
      PN2_RETURN_LAUNCH();                                                     \
    }
    PN2_V9A(256, 32, 4) PN2_V9A(256, 32, 2) PN2_V9A(512, 16, 4) PN2_V9A(256, 4, 4)
    PN2_V9A(256, 4, 2) PN2_V9A(256, 16, 4) PN2_V9A(256, 8, 4) PN2_V9A(256, 8, 2)
    PN2_V9A(256, 16, 2) PN2_V9A(512, 32, 4) PN2_V9A(512, 32, 2) PN2_V9A(128, 4, 2)
    PN2_V9A(128, 8, 4) PN2_V9A(512, 8, 2) PN2_V9A(512, 4, 2)
#undef PN2_V9A
  }
  if (variant == 95 || variant == 96) {  // v9 with the lane-parallel slot resolve (G = 4 / 2)
    const int G = variant == 95 ? 4 : 2;
#define PN2_V9L(BL, PP, GG)                                                    \
    if (block == BL && ppt == PP && G == GG) {                                 \
      launch_v9<BL, PP, GG, true>(xyz, B, N, M, idx, nx, s);                   \
      PN2_RETURN_LAUNCH();                                                     \
    }
    PN2_V9L(256, 32, 4) PN2_V9L(256, 32, 2) PN2_V9L(512, 16, 4) PN2_V9L(256, 4, 4)
    PN2_V9L(256, 4, 2) PN2_V9L(256, 16, 4) PN2_V9L(64, 4, 4) PN2_V9L(64, 4, 2) PN2_V9L(128, 8, 4)
    PN2_V9L(256, 8, 4) PN2_V9L(64, 16, 4) PN2_V9L(256, 64, 4) PN2_V9L(64, 8, 4) PN2_V9L(64, 8, 2)
    PN2_V9L(256, 8, 2) PN2_V9L(256, 16, 2) PN2_V9L(512, 32, 4) PN2_V9L(64, 2, 2)
    PN2_V9L(512, 32, 2) PN2_V9L(128, 4, 2)
#undef PN2_V9L
  }
  if (variant >= 91 && variant <= 94) {  // v9, variant = 90 + G (slots per max3 group)
    const int G = variant - 90;
#define PN2_V9(BL, PP, GG)                                                     \
    if (block == BL && ppt == PP && G == GG) {                                 \
      launch_v9<BL, PP, GG>(xyz, B, N, M, idx, nx, s);                         \
      PN2_RETURN_LAUNCH();                                                     \
    }
#define PN2_V9G(BL, PP) PN2_V9(BL, PP, 1) PN2_V9(BL, PP, 2) PN2_V9(BL, PP, 4)
    PN2_V9G(64, 4) PN2_V9G(64, 8) PN2_V9G(128, 4) PN2_V9G(128, 8) PN2_V9G(256, 4)
    PN2_V9G(256, 8) PN2_V9G(256, 16) PN2_V9G(512, 4) PN2_V9G(512, 8) PN2_V9G(512, 16)
    PN2_V9G(256, 32) PN2_V9(512, 32, 4) PN2_V9(256, 64, 4) PN2_V9(128, 16, 4) PN2_V9(128, 1, 1)
    PN2_V9(64, 16, 4) PN2_V9(64, 32, 4) PN2_V9(128, 32, 4)
    PN2_V9(64, 1, 1) PN2_V9(64, 2, 1) PN2_V9(64, 2, 2) PN2_V9(128, 2, 2) PN2_V9(256, 2, 2)
#undef PN2_V9G
#undef PN2_V9
  }
  if (variant == 8) {
#define PN2_V8(BL, PP)                                                         \
    if (block == BL && ppt == PP) {                                            \
      launch_v8<BL, PP>(xyz, B, N, M, idx, nx, s);                             \
      PN2_RETURN_LAUNCH();                                                     \
    }
    PN2_V8(256, 4) PN2_V8(256, 8) PN2_V8(512, 8) PN2_V8(512, 16) PN2_V8(1024, 8)
    PN2_V8(1024, 16) PN2_V8(256, 16) PN2_V8(256, 32) PN2_V8(512, 32) PN2_V8(1024, 4)
    PN2_V8(128, 8) PN2_V8(128, 16) PN2_V8(64, 16) PN2_V8(512, 4)
#undef PN2_V8
  }
  if (variant == 7) {
#define PN2_V7(BL, PP)                                                         \
    if (block == BL && ppt == PP) {                                            \
      launch_v7<BL, PP>(xyz, B, N, M, idx, nx, s);                             \
      PN2_RETURN_LAUNCH();                                                     \
    }
    PN2_FPS_CONFIGS(PN2_V7)
#undef PN2_V7
  }
  if (variant == 5) {  // v5 without culling (one cell per wave)
#define PN2_V(BL, PP)                                                          \
    if (block == BL && ppt == PP) {                                            \
      launch_v5<BL, PP, PP, false>(xyz, B, N, M, idx, nx, s);                  \
      PN2_RETURN_LAUNCH();                                                     \
    }
    PN2_FPS_CONFIGS(PN2_V)
#undef PN2_V
  }
  if (variant >= 60 && variant < 80) {  // v6, variant = 60 + SUB
    const int sub = variant - 60;
#define PN2_C6(BL, PP, SB)                                                     \
    if (block == BL && ppt == PP && sub == SB) {                                \
      launch_v6<BL, PP, SB>(xyz, B, N, M, idx, nx, s);                          \
      PN2_RETURN_LAUNCH();                                                      \
    }
    PN2_C6(256, 4, 1) PN2_C6(256, 4, 2) PN2_C6(256, 4, 4) PN2_C6(512, 8, 2) PN2_C6(512, 8, 4)
    PN2_C6(512, 16, 2) PN2_C6(512, 16, 4) PN2_C6(512, 16, 8) PN2_C6(1024, 8, 2) PN2_C6(1024, 8, 4)
    PN2_C6(256, 32, 4) PN2_C6(256, 32, 8) PN2_C6(1024, 16, 4) PN2_C6(1024, 16, 8)
    PN2_C6(128, 8, 2) PN2_C6(128, 8, 4) PN2_C6(256, 8, 2) PN2_C6(256, 16, 4) PN2_C6(64, 16, 4)
    PN2_C6(512, 32, 8) PN2_C6(256, 32, 16)
#undef PN2_C6
  }
  if (variant >= 50 && variant < 60) {  // v5 culled, variant = 50 + SUB
    const int sub = variant - 50;
#define PN2_C(BL, PP, SB)                                                      \
    if (block == BL && ppt == PP && sub == SB) {                                \
      launch_v5<BL, PP, SB, true>(xyz, B, N, M, idx, nx, s);                    \
      PN2_RETURN_LAUNCH();                                                      \
    }
    PN2_C(256, 4, 1) PN2_C(256, 4, 2) PN2_C(256, 4, 4) PN2_C(512, 8, 2) PN2_C(512, 8, 4)
    PN2_C(512, 16, 2) PN2_C(512, 16, 4) PN2_C(512, 16, 8) PN2_C(1024, 8, 2) PN2_C(1024, 8, 4)
    PN2_C(256, 32, 4) PN2_C(256, 32, 8) PN2_C(1024, 16, 4) PN2_C(1024, 16, 8) PN2_C(64, 16, 4)
    PN2_C(128, 8, 4) PN2_C(128, 16, 4) PN2_C(256, 16, 4) PN2_C(256, 8, 4) PN2_C(1024, 4, 4)
#undef PN2_C
  }
  if (variant >= 30 && variant < 50) {  // culled sampler, variant = 30 + SUB
    const int sub = variant - 30;
#define PN2_C(BL, PP, SB)                                                      \
    if (block == BL && ppt == PP && sub == SB) {                                \
      launch_cull<BL, PP, SB>(xyz, B, N, M, idx, nx, s);                        \
      PN2_RETURN_LAUNCH();                                                      \
    }
    PN2_C(256, 4, 1) PN2_C(256, 4, 2) PN2_C(256, 4, 4) PN2_C(512, 8, 2) PN2_C(512, 8, 4)
    PN2_C(512, 16, 2) PN2_C(512, 16, 4) PN2_C(512, 16, 8) PN2_C(1024, 8, 2) PN2_C(1024, 8, 4)
    PN2_C(256, 32, 4) PN2_C(256, 32, 8) PN2_C(1024, 16, 4) PN2_C(1024, 16, 8)
#undef PN2_C
  }
  return PN2_EINVAL;
}



// Hot-loop micro-benchmark (lab only): wave 0 of one workgroup runs the fps_hot.h hot-phase
// pick loop over the first 128 points of a cloud with no certification bound, `iters` picks,
// and reports s_memtime cycles per pick. VAR bits switch pieces off to price them:
// 1 = no ring write, 2 = no tie check, 4 = no readfirstlane (ballot on the DPP result).
template <int VAR>
__global__ __launch_bounds__(64) void hot_loop_bench(const float* __restrict__ xyz, int iters,
                                                     int32_t* __restrict__ out,
                                                     unsigned long long* __restrict__ cyc) {
  using f2 = float __attribute__((ext_vector_type(2)));
  __shared__ float4 scl[256];
  const int lane = threadIdx.x;
  int hv[2], hk[2];
  f2 hx, hy, hz;
  for (int q = 0; q < 2; ++q) {
    hk[q] = lane * 2 + q;
    hx[q] = xyz[3 * hk[q]]; hy[q] = xyz[3 * hk[q] + 1]; hz[q] = xyz[3 * hk[q] + 2];
    hv[q] = __float_as_int(kInitTemp);
  }
  const uint32_t hkey0 = hot_key(hk[0]), hkey1 = hot_key(hk[1]);
  int acc = 0;
  unsigned long long c0, c1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0)::"memory");
  for (int jj = 0; jj < iters; ++jj) {
    const bool b1 = hv[1] > hv[0] || (hv[1] == hv[0] && hkey1 < hkey0);
    const int cv = b1 ? hv[1] : hv[0];
    const uint32_t ck = b1 ? hkey1 : hkey0;
    const uint32_t enc = hot_enc(cv);
    const uint32_t wmv = wave_max_u32(enc);
    const uint32_t wm = (VAR & 4) ? wmv : uniform_u32(wmv);
    const uint64_t hold = __builtin_amdgcn_ballot_w64(enc == wm);
    int L;
    if ((VAR & 2) || __builtin_popcountll(hold) == 1) {
      L = (int)__builtin_ctzll(hold);
    } else {
      const uint32_t km = ~uniform_u32(wave_max_u32(enc == wm ? ~ck : 0u));
      L = (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(enc == wm && ck == km));
    }
    const uint32_t wkey = (uint32_t)__builtin_amdgcn_readlane((int)ck, L);
    acc += (int)wkey;
    const float lx = b1 ? hx[1] : hx[0], ly = b1 ? hy[1] : hy[0], lz = b1 ? hz[1] : hz[0];
    const int lk = b1 ? hk[1] : hk[0];
    if (!(VAR & 1))
      if (lane == L) scl[jj & 255] = make_float4(lx, ly, lz, __int_as_float(lk));
    const float cx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lx), L));
    const float cy = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ly), L));
    const float cz = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lz), L));
    const f2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
    const f2 dx = hx - c2x, dy = hy - c2y, dz = hz - c2z;
    const f2 d = (dx * dx + dy * dy) + dz * dz;
    hv[0] = min(hv[0], __float_as_int(d.x));
    hv[1] = min(hv[1], __float_as_int(d.y));
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1)::"memory");
  __syncthreads();
  out[lane] = acc + hv[0] + hv[1] + __float_as_int(scl[lane].x);
  if (lane == 0) cyc[0] = c1 - c0;
}
}  // namespace
}  // namespace pn2

extern "C" {

// Hot-loop micro-benchmark: cycles for `iters` picks of variant `var` (hot_loop_bench).
int pn2_hot_loop_bench(const float* xyz, int iters, int var, int32_t* out,
                       unsigned long long* cyc_dev) {
  hipStream_t s = 0;
#define PN2_HB(V) \
  if (var == V) hipLaunchKernelGGL(pn2::hot_loop_bench<V>, dim3(1), dim3(64), 0, s, xyz, iters, out, cyc_dev); else
  PN2_HB(0) PN2_HB(1) PN2_HB(2) PN2_HB(3) PN2_HB(4) PN2_HB(7) { return PN2_EINVAL; }
#undef PN2_HB
  return (int)hipDeviceSynchronize();
}

// Diagnostic entry: stamped hot-set sampler (fps_hot.h) over B clouds; out (16 clouds x 16
// waves x 8): per wave the cycles of phases 0 cold pass, 1 lane top-3, 2 row extraction,
// 3 extraction barrier, 4 hot phase (wave 0) / wait (others), 5 loop-top barrier; [6] refresh
// rounds, [7] hot picks (wave 0).
int pn2_fps_hot_stamp(const float* xyz, int B, int N, int npoint, int32_t* idx,
                      unsigned long long* out_host) {
  hipStream_t s = 0;
  if (N > 8192 || N <= 4096) return PN2_EINVAL;
  hipLaunchKernelGGL((pn2::fps_hot_kernel<256, 32, 2, 8, 256, true>), dim3(B), dim3(256), 0, s,
                     xyz, N, npoint, idx, nullptr);
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_stamp),
                          sizeof(unsigned long long) * 16 * 16 * 8);
  return (int)e;
}

// Diagnostic entry: stamped asynchronous hot-set sampler (fps_hota_kernel<8, 16, 4>); out as
// pn2_fps_hot_stamp with 9 waves: phases 0 B1 wait, 1 write-out, 2 cold catch-up, 3 top-3 +
// extraction, 4 B2 wait, 5 hot setup, 6 hot loop / cold async loop; row 12: [0] kernel
// cycles, [1] real time (10 ns), [2] rounds, [3] hot picks, [4] tie paths, [5] centres applied
// asynchronously (wave 1), [6] idle spins (wave 1).
int pn2_fps_hota_stamp(const float* xyz, int B, int N, int npoint, int32_t* idx,
                       unsigned long long* out_host) {
  hipStream_t s = 0;
  if (N > 8192) return PN2_EINVAL;
  hipLaunchKernelGGL((pn2::fps_hota_kernel<7, 20, 4, 8192, 256, true>), dim3(B), dim3(512), 0, s,
                     xyz, N, npoint, idx, nullptr);
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_stamp),
                          sizeof(unsigned long long) * 16 * 16 * 8);
  return (int)e;
}

// Diagnostic entry: stamped v2 run; out[w*8+ph] = cycles of phase ph summed over the
// iterations, for wave w of cloud 0 (ph: 0 scan, 1 wave reduce, 2 write+barrier,
// 3 cross-wave reduce, 4 centre load, 5 index store).
int pn2_fps_stamp(const float* xyz, int N, int npoint, int32_t* idx, int block, int ppt,
                  unsigned long long* out_host) {
  hipStream_t s = 0;
#define PN2_S(BL, PP)                                                                        \
  if (block == BL && ppt == PP) {                                                            \
    hipLaunchKernelGGL((pn2::fps_v2_kernel<BL, PP, (3 * BL * PP * 4 + 256 <= 160 * 1024), true>), \
                       dim3(1), dim3(BL), 0, s, xyz, N, npoint, idx, nullptr);               \
  } else
  if (block < 0) {  // v6 stamped: block = -BL, ppt = PP*100 + SUB
#define PN2_S6(BL, PP, SB)                                                                   \
    if (-block == BL && ppt == PP * 100 + SB) {                                              \
      hipLaunchKernelGGL((pn2::fps_v6_kernel<BL, PP, SB, true>), dim3(1), dim3(BL), 0, s, xyz, \
                         N, npoint, idx, nullptr);                                           \
    } else
    PN2_S6(512, 16, 4) PN2_S6(1024, 8, 4) PN2_S6(256, 4, 2) PN2_S6(512, 16, 8) { return PN2_EINVAL; }
#undef PN2_S6
  } else if (ppt >= 110000) {  // v11 (G = 4) stamped: ppt = 110000 + PP
#define PN2_S11(BL, PP)                                                                      \
    if (block == BL && ppt == 110000 + PP) {                                                 \
      hipLaunchKernelGGL((pn2::fps_v11_kernel<BL, PP, 4, true>), dim3(1), dim3(BL), 0, s,    \
                         xyz, N, npoint, idx, nullptr);                                      \
    } else
    PN2_S11(256, 32) PN2_S11(512, 16) PN2_S11(256, 4) { return PN2_EINVAL; }
#undef PN2_S11
  } else if (ppt >= 90000 && ppt < 95000) {  // v9 (G = 4) stamped: ppt = 90000 + PP
#define PN2_S9(BL, PP)                                                                       \
    if (block == BL && ppt == 90000 + PP) {                                                  \
      hipLaunchKernelGGL((pn2::fps_v9_kernel<BL, PP, 4, true, true>), dim3(1), dim3(BL), 0, s, \
                         xyz, N, npoint, idx, nullptr);                                      \
    } else
    PN2_S9(256, 32) PN2_S9(512, 16) PN2_S9(256, 4) PN2_S9(256, 16) { return PN2_EINVAL; }
#undef PN2_S9
  } else if (ppt >= 95000 && ppt < 96000) {  // v9 lane-resolve (G = 4) stamped: 95000 + PP
#define PN2_S9L(BL, PP)                                                                      \
    if (block == BL && ppt == 95000 + PP) {                                                  \
      hipLaunchKernelGGL((pn2::fps_v9_kernel<BL, PP, 4, true, true, true>), dim3(1), dim3(BL), \
                         0, s, xyz, N, npoint, idx, nullptr);                                \
    } else
    PN2_S9L(256, 32) PN2_S9L(256, 4) { return PN2_EINVAL; }
#undef PN2_S9L
  } else if (ppt >= 97000 && ppt < 98000) {  // v9 lane-resolve + atomic (G = 4): 97000 + PP
#define PN2_S9A(BL, PP)                                                                      \
    if (block == BL && ppt == 97000 + PP) {                                                  \
      hipLaunchKernelGGL((pn2::fps_v9_kernel<BL, PP, 4, true, true, true, true>), dim3(1),   \
                         dim3(BL), 0, s, xyz, N, npoint, idx, nullptr);                      \
    } else
    PN2_S9A(256, 32) PN2_S9A(256, 4) { return PN2_EINVAL; }
#undef PN2_S9A
  } else if (ppt >= 20000) {  // v8 stamped: ppt = 20000 + PP
#define PN2_S8(BL, PP)                                                                       \
    if (block == BL && ppt == 20000 + PP) {                                                  \
      hipLaunchKernelGGL((pn2::fps_v8_kernel<BL, PP, true>), dim3(1), dim3(BL), 0, s, xyz, N,  \
                         npoint, idx, nullptr);                                              \
    } else
    PN2_S8(1024, 8) PN2_S8(512, 16) PN2_S8(256, 4) PN2_S8(512, 8) { return PN2_EINVAL; }
#undef PN2_S8
  } else if (ppt >= 10000) {  // v7 stamped: ppt = 10000 + PP
#define PN2_S7(BL, PP)                                                                       \
    if (block == BL && ppt == 10000 + PP) {                                                  \
      hipLaunchKernelGGL((pn2::fps_v7_kernel<BL, PP, true>), dim3(1), dim3(BL), 0, s, xyz, N,  \
                         npoint, idx, nullptr);                                              \
    } else
    PN2_S7(64, 4) PN2_S7(256, 4) PN2_S7(512, 16) PN2_S7(1024, 8) PN2_S7(512, 8) { return PN2_EINVAL; }
#undef PN2_S7
  } else
  PN2_S(64, 4) PN2_S(256, 4) PN2_S(512, 16) PN2_S(1024, 8) PN2_S(512, 8) { return PN2_EINVAL; }
#undef PN2_S
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_stamp), sizeof(unsigned long long) * 16 * 8);
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(out_host + 16 * 8, HIP_SYMBOL(pn2::g_iter), sizeof(unsigned long long) * 4096);
  return (int)e;
}

// Tuning entry (not part of include/pn2hip.h): run one (variant, block, ppt) instantiation.
// Placement experiment: the 256 x 32 LRES sampler with `pad` s_nop at the top of its loop
// (the lab is built with -falign-loops=64, so pad * 4 bytes = the body's offset in a line).
extern "C++" {
template <int PAD>
static void launch_pad(const float* xyz, int B, int N, int M, int32_t* idx, float* nx,
                       hipStream_t s) {
  hipLaunchKernelGGL((pn2::fps_v9_kernel<256, 32, 4, true, false, true, false, PAD>), dim3(B),
                     dim3(256), 0, s, xyz, N, M, idx, nx);
}
}
int pn2_fps_pad(const float* xyz, int B, int N, int npoint, int32_t* idx, float* new_xyz, int pad,
                pn2_stream_t stream) {
  if (N > 8192 || N < 1) return PN2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  switch (pad) {
    case 0: launch_pad<0>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 1: launch_pad<1>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 2: launch_pad<2>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 3: launch_pad<3>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 4: launch_pad<4>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 5: launch_pad<5>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 6: launch_pad<6>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 7: launch_pad<7>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 8: launch_pad<8>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 9: launch_pad<9>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 10: launch_pad<10>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 11: launch_pad<11>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 12: launch_pad<12>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 13: launch_pad<13>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 14: launch_pad<14>(xyz, B, N, npoint, idx, new_xyz, s); break;
    case 15: launch_pad<15>(xyz, B, N, npoint, idx, new_xyz, s); break;
    default: return PN2_EINVAL;
  }
  PN2_RETURN_LAUNCH();
}

int pn2_fps_tune(const float* xyz, int B, int N, int npoint, int32_t* idx, float* new_xyz,
                 int variant, int block, int ppt, pn2_stream_t stream) {
  return pn2::fps_tune_impl(xyz, B, N, npoint, idx, new_xyz, variant, block, ppt,
                            (hipStream_t)stream);
}

// Diagnostic entry: stamped culled hot-set sampler (fps_cull.h); out (16 clouds x 16 waves x
// 8): per wave the cycles of phases 0 cold async apply (incl. waiting), 1 Tmax, 2 B_A,
// 3 outputs + counts, 4 B_B, 5 choice + append, 6 B_C, 7 hot phase (wave 0) + setup;
// stats (16 clouds x 8): [0] kernel cycles, [1] refreshes, [2] stalls, [3] applied (cell,
// centre) pairs of wave 1, [4] hot picks, [5] pairs of wave 2.
int pn2_fps_cull_stamp(const float* xyz, int B, int N, int npoint, int32_t* idx,
                       unsigned long long* out_host, unsigned long long* stats_host) {
  hipStream_t s = 0;
  if (N > 8192) return PN2_EINVAL;
  hipLaunchKernelGGL((pn2::fps_hotcull_kernel<16, 9, 8192, true, 3, 4>), dim3(B), dim3(1024), 0, s, xyz, N,
                     npoint, idx, nullptr);
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_stamp),
                          sizeof(unsigned long long) * 16 * 16 * 8);
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(stats_host, HIP_SYMBOL(pn2::g_cull_stats),
                          sizeof(unsigned long long) * 16 * 8);
  return (int)e;
}

// Diagnostic: the per-round trace the stamped hot-cull sampler leaves in g_iter (cloud 0).
int pn2_fps_cull_waves(unsigned long long* out_host) {
  return (int)hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_cull_wave), sizeof(unsigned long long) * 16 * 16 * 4);
}
int pn2_fps_cull_events(unsigned long long* out_host) {
  return (int)hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_cull_ev), sizeof(unsigned long long) * 64 * 16 * 8);
}

}  // extern "C"
