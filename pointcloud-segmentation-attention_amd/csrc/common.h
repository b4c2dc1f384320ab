// Shared device helpers for the gfx950 kernels of libpn2hip.so.
//
// Every translation unit is compiled with -ffp-contract=off AND starts with
// `#pragma clang fp contract(off)`: the reference's index results (FPS argmax, ball-query
// membership, three_nn order) depend on un-fused fp32 `(dx*dx+dy*dy)+dz*dz`, which is what
// the reference CPU code computes under plain `g++ -O2` (tf_interpolate_compile.sh:2,
// grouping/test/compile.sh:1). An FMA would change the rounding of d2 and therefore indices.
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pn2hip.h"

#define PN2_DEV __device__ __forceinline__

namespace pn2 {

constexpr int kWave = 64;  // CDNA wavefront

// Squared distance exactly as the reference writes it: (x2-x1)*(x2-x1)+(y2-y1)*(y2-y1)+
// (z2-z1)*(z2-z1), evaluated left to right in fp32 with no contraction
// (tf_sampling_g.cu:142, tf_grouping_g.cu:24, tf_interpolate.cpp:73).
PN2_DEV float sqdist(float ax, float ay, float az, float bx, float by, float bz) {
  const float dx = ax - bx;
  const float dy = ay - by;
  const float dz = az - bz;
  float d = __fmul_rn(dx, dx);
  d = __fadd_rn(d, __fmul_rn(dy, dy));
  d = __fadd_rn(d, __fmul_rn(dz, dz));
  return d;
}

// ---- wave-level reductions (64 lanes, result in every lane) ----------------------------
// Rows of 16 lanes are reduced with DPP (quad_perm xor1/xor2, row_half_mirror, row_mirror),
// then rows are combined with the gfx950 v_permlane16_swap / v_permlane32_swap exchanges:
// no LDS round trip, no ds_bpermute.
template <int CTRL>
PN2_DEV uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // row_half_mirror (lane i <-> 7-i within 8)
constexpr int kDppMirror = 0x140;     // row_mirror (lane i <-> 15-i within 16)

PN2_DEV uint64_t pack64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

template <int CTRL>
PN2_DEV uint64_t max_dpp_u64(uint64_t v) {
  const uint32_t lo = dpp_u32<CTRL>((uint32_t)v);
  const uint32_t hi = dpp_u32<CTRL>((uint32_t)(v >> 32));
  const uint64_t o = pack64(lo, hi);
  return o > v ? o : v;
}

// max over the 16 lanes of each DPP row (all 16 lanes get the row max)
PN2_DEV uint64_t row16_max_u64(uint64_t v) {
  v = max_dpp_u64<kDppXor1>(v);
  v = max_dpp_u64<kDppXor2>(v);
  v = max_dpp_u64<kDppHalfMirror>(v);
  v = max_dpp_u64<kDppMirror>(v);
  return v;
}

PN2_DEV uint64_t wave_max_u64(uint64_t v) {
  v = row16_max_u64(v);
  {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const uint64_t a = pack64(l[0], h[0]), b = pack64(l[1], h[1]);
    v = a > b ? a : b;
  }
  {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const uint64_t a = pack64(l[0], h[0]), b = pack64(l[1], h[1]);
    v = a > b ? a : b;
  }
  return v;
}

// 32-bit max over the 16 lanes of each DPP row / over the wave. The DPP moves fold into
// v_max_u32_dpp (one instruction per step).
template <int CTRL>
PN2_DEV uint32_t max_dpp_u32(uint32_t v) {
  const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
  return o > v ? o : v;
}
PN2_DEV uint32_t row16_max_u32(uint32_t v) {
  v = max_dpp_u32<kDppXor1>(v);
  v = max_dpp_u32<kDppXor2>(v);
  v = max_dpp_u32<kDppHalfMirror>(v);
  v = max_dpp_u32<kDppMirror>(v);
  return v;
}
PN2_DEV uint32_t wave_max_u32(uint32_t v) {
  v = row16_max_u32(v);
  {
    auto x = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = x[0] > x[1] ? x[0] : x[1];
  }
  {
    auto x = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = x[0] > x[1] ? x[0] : x[1];
  }
  return v;
}

PN2_DEV uint32_t uniform_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
PN2_DEV uint64_t uniform_u64(uint64_t v) {
  return pack64(uniform_u32((uint32_t)v), uniform_u32((uint32_t)(v >> 32)));
}

PN2_DEV int lane_id() { return (int)__lane_id(); }

// Sum / max over aligned segments of SEG lanes (SEG a power of two <= 64) using xor shuffles.
template <int SEG>
PN2_DEV float seg_sum(float v) {
#pragma unroll
  for (int o = SEG / 2; o > 0; o >>= 1) v = __fadd_rn(v, __shfl_xor(v, o, kWave));
  return v;
}
template <int SEG>
PN2_DEV float seg_max(float v) {
#pragma unroll
  for (int o = SEG / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// XCD-aware block order (MI355X_MICROARCH.md, workgroup dispatch): linear blocks are dealt
// round-robin over the 8 XCDs (blocks L and L + 8 share one XCD and its L2). Launching
// xcd_grid(n) blocks and working on logical block xcd_block(L, n) gives every XCD one
// contiguous range of logical blocks, so the blocks of one cloud share an L2 instead of each
// XCD fetching the cloud's rows. Speed only: any placement gives the same results. Logical
// blocks >= n (the padding) must return before any barrier.
constexpr int kXcds = 8;
inline unsigned xcd_grid(long long n) { return (unsigned)((n + kXcds - 1) / kXcds * kXcds); }
PN2_DEV int xcd_block(int L, int n) {
  const int per = (n + kXcds - 1) / kXcds;
  return (L % kXcds) * per + L / kXcds;
}

// Integer division by a runtime divisor via a precomputed 32-bit magic (exact when
// numerator * divisor < 2^32; the launcher checks that bound).
struct FastDiv {
  uint32_t d, magic;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  f.magic = d <= 1 ? 0u : (uint32_t)((((uint64_t)1 << 32) + d - 1) / d);
  return f;
}
PN2_DEV uint32_t fdiv(uint32_t n, FastDiv f) { return f.d == 1 ? n : __umulhi(n, f.magic); }

// pn2_fps_chain's argument check (fps.hip), shared with the plan executor (plan.hip)
int fps_chain_check(const float* xyz, int B, int N, int nstages, const int* npoint,
                    int32_t* const* idx, float* const* new_xyz);
// pn2_fps_chain without the stored-fault report (the plan executor takes the fault word once,
// before it enqueues anything, so a plan never stops part-way through a step)
int fps_chain_launch(const float* xyz, int B, int N, int nstages, const int* npoint,
                     int32_t* const* idx, float* const* new_xyz, hipStream_t s, bool take,
                     void* grid0 = nullptr, size_t grid0_bytes = 0);
// a fault stored by an earlier sampler launch, cleared (0: none)
int fps_take_fault();

}  // namespace pn2

// launch-status helper for the C ABI
#define PN2_RETURN_LAUNCH()                         \
  do {                                              \
    hipError_t e__ = hipGetLastError();             \
    return e__ == hipSuccess ? PN2_OK : (int)e__;   \
  } while (0)
