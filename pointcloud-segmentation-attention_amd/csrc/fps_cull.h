// Culled hot-set farthest-point sampler for large clouds (SA1: 8,192 -> 1,024) on gfx950.
// Reference: farthestpointsamplingKernel, pointnet2_tensorflow/tf_ops/sampling/
// tf_sampling_g.cu:105-170 -- running min distance (:139-145), argmax with the tie rule of the
// 512-thread tree (:146-163), the new centre is the argmax (:164-167).
//
// Same output as fps_v9_kernel, bit for bit; a different schedule of the same arithmetic.
//  * CELLS. The cloud is counting-sorted by a 16^3 Morton bucket, and every wave slot (64
//    consecutive sorted points) is a cell with a bounding box and the exact maximum Tmax of
//    its running mins. A centre c can lower a point of the cell only if its box lower bound
//    lb(c) < Tmax. lb is computed in fp32 with the same rounding steps as the distance, and
//    every step is monotone, so fl-dist(p, c) >= lb for every p in the box: a skipped
//    (cell, centre) pair leaves every running min unchanged, exactly.
//  * HOT SET. After each refresh the points above a threshold tau (the smallest of NT fractions
//    of the global max whose count fits K = 64 * HQ, 256 by default) form the hot set. Wave 0 picks from it alone:
//    while its best value is > tau it beats every other point (they are all <= tau, and
//    running mins only decrease), so it IS the reference's next centre; the wave updates the
//    hot values and goes on -- no block-wide argmax per pick.
//  * REFRESH. When the hot best drops to <= tau, every wave applies the batch of centres
//    picked since the last refresh to its cells (culled; two centres per packed pass), the
//    changed cells' Tmax are recomputed, and a new tau and hot set are chosen. If no fraction
//    fits (more than K points tie near the max), one exact block argmax picks the centre.
// Exactness does not depend on the sort: any cell layout gives the same picks; the sort only
// decides how much the box test skips (tools/model_fps_cull.py models it on the SA1 crops:
// ~34 refreshes for 1,023 picks at K = 128; 25 measured at K = 256, ~93 % of (cell, centre) pairs skipped).
#pragma once
#include "fps_kernels.h"
#include "grid.h"

namespace pn2 {
namespace {

__device__ unsigned long long g_cull_stats[16 * 8];  // STAMP builds: per-cloud counters
__device__ unsigned long long g_cull_wave[16 * 16 * 4];  // STAMP: per wave groups, group cycles, pairs, polls
__device__ unsigned long long g_cull_ev[64 * 16 * 8];   // STAMP: cloud 0, rounds < 64: per wave events

// float max over the wave (every lane gets it); DPP rows, then the gfx950 permlane swaps
PN2_DEV float wave_max_f32(float v) {
#define PN2_FMAX_DPP(C) v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp( \
                              __float_as_int(v), __float_as_int(v), C, 0xF, 0xF, false)))
  PN2_FMAX_DPP(kDppXor1);
  PN2_FMAX_DPP(kDppXor2);
  PN2_FMAX_DPP(kDppHalfMirror);
  PN2_FMAX_DPP(kDppMirror);
#undef PN2_FMAX_DPP
  {
    auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(x[0]), __uint_as_float(x[1]));
  }
  {
    auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(x[0]), __uint_as_float(x[1]));
  }
  return v;
}

// signed 32-bit max over the wave (every lane gets it): v_max_i32_dpp rows, permlane swaps
PN2_DEV int wave_max_i32(int v) {
// (old = 0: every lane has a valid source in these patterns, so the old value is never used,
// and the move folds into v_max_i32_dpp)
#define PN2_IMAX_DPP(C) v = max(v, __builtin_amdgcn_update_dpp(0, v, C, 0xF, 0xF, false))
  PN2_IMAX_DPP(kDppXor1);
  PN2_IMAX_DPP(kDppXor2);
  PN2_IMAX_DPP(kDppHalfMirror);
  PN2_IMAX_DPP(kDppMirror);
#undef PN2_IMAX_DPP
  {
    auto x = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
    v = max((int)x[0], (int)x[1]);
  }
  {
    auto x = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
    v = max((int)x[0], (int)x[1]);
  }
  return v;
}

// signed 32-bit max over the wave, valid in lane 63 only: the DPP row reduction, then the
// row broadcasts (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3)
PN2_DEV int wave_max_i32_l63(int v) {
#define PN2_IMAX_DPP(C, R) v = max(v, __builtin_amdgcn_update_dpp(0, v, C, R, 0xF, false))
  PN2_IMAX_DPP(kDppXor1, 0xF);
  PN2_IMAX_DPP(kDppXor2, 0xF);
  PN2_IMAX_DPP(kDppHalfMirror, 0xF);
  PN2_IMAX_DPP(kDppMirror, 0xF);
#undef PN2_IMAX_DPP
  // the broadcasts leave the rows outside row_mask unwritten (dst == src), which the
  // update_dpp builtin cannot express without an extra move: written directly, with the
  // DPP read-after-VALU-write wait states spelled out
  asm volatile(
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
      "s_nop 1"
      : "+v"(v));
  return v;
}

// tie key: smaller = earlier in the reference's order (k mod 512, k div 512); N < 2^25
PN2_DEV uint32_t cull_key(int k) { return ((uint32_t)(k & 511) << 16) | ((uint32_t)k >> 9); }

// exclusive prefix sum over the wave (Hillis-Steele on ds_swizzle-free shuffles)
PN2_DEV uint32_t wave_excl_scan(uint32_t v, int lane) {
  uint32_t s = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)s, o, kWave);
    s += lane >= o ? u : 0u;
  }
  return s - v;
}

// the box lower bound of a centre: every step rounds monotonically, so it never exceeds the
// fp32 distance (((dx*dx)+(dy*dy))+(dz*dz)) of any point inside the box
PN2_DEV float box_lb(float4 lo, float4 hi, float cx, float cy, float cz) {
  const float gx = fmaxf(fmaxf(lo.x - cx, cx - hi.x), 0.0f);
  const float gy = fmaxf(fmaxf(lo.y - cy, cy - hi.y), 0.0f);
  const float gz = fmaxf(fmaxf(lo.z - cz, cz - hi.z), 0.0f);
  return (gx * gx + gy * gy) + gz * gz;
}

// threshold fractions of the global max, ascending (chosen: the first whose count fits)
__constant__ float kCullFrac[12] = {0.6f, 0.7f, 0.75f, 0.8f, 0.84f, 0.87f,
                                    0.9f, 0.92f, 0.94f, 0.96f, 0.98f, 0.99f};


// STAMP builds: s_memtime of event K of this round, kept in SGPRs and stored for cloud 0 after
// the round's last barrier (a store before a barrier would make its s_waitcnt wait for it)
#define PN2_EV(K)                                                                          \
  if constexpr (STAMP) ev[K] = __builtin_amdgcn_s_memtime();

// bits s, s + PPT, s + 2 PPT, ... (GRP of them): the lanes that test cell s in a group
template <int PPT, int GRP>
PN2_DEV constexpr uint64_t cell_lanes(int s) {
  uint64_t m = 0;
  for (int i = 0; i < GRP; ++i) m |= 1ull << (PPT * i + s);
  return m;
}

// NPTS points at most; wave 0 is the hot wave, waves 1..NW-1 hold the cold cells (PPT cells of
// 64 sorted points per wave).
// ---- the hot wave's pick step (also run alone by tools/ubench/pick_floor.hip) -------------
using hf2 = float __attribute__((ext_vector_type(2)));

// HQ = 4 entries per lane: the lane's best entry (value desc, then entry order = tie order:
// strict '>' keeps the lower entry), its coordinates and index, interleaved with the wave max
// (DPP rows, then row_bcast:15 / :31 into lane 63): the selects fill the DPP read-after-write
// wait states (2 per step) that were s_nop before. Wait states inside the block: VALU-written
// SGPR mask -> v_cndmask 2, DPP source 2, readlane source 1. m01 / m23 / mh are the lane's
// select masks (the tie path repeats the selects on the tie keys with them).
PN2_DEV void hot_best4(const int (&hv)[4], const hf2 (&hx)[2], const hf2 (&hy)[2],
           const hf2 (&hz)[2], const int (&hk)[4], int& cv, float& lx, float& ly,
           float& lz, int& lk, int& wm, uint64_t& m01, uint64_t& m23, uint64_t& mh) {
  int v23, r, tk;
  float tx, ty, tz;
  asm volatile(
      "v_cmp_gt_i32_e64 %[m01], %[h1], %[h0]\n\t"
      "v_cmp_gt_i32_e64 %[m23], %[h3], %[h2]\n\t"
      "v_max_i32_e32 %[cv], %[h0], %[h1]\n\t"
      "v_max_i32_e32 %[v23], %[h2], %[h3]\n\t"
      "v_cmp_gt_i32_e64 %[mh], %[v23], %[cv]\n\t"
      "v_max_i32_e32 %[cv], %[cv], %[v23]\n\t"
      "v_cndmask_b32_e64 %[lx], %[x0], %[x1], %[m01]\n\t"
      "v_cndmask_b32_e64 %[tx], %[x2], %[x3], %[m23]\n\t"
      "v_max_i32_dpp %[r], %[cv], %[cv] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_e64 %[ly], %[y0], %[y1], %[m01]\n\t"
      "v_cndmask_b32_e64 %[ty], %[y2], %[y3], %[m23]\n\t"
      "v_max_i32_dpp %[r], %[r], %[r] quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_e64 %[lz], %[z0], %[z1], %[m01]\n\t"
      "v_cndmask_b32_e64 %[tz], %[z2], %[z3], %[m23]\n\t"
      "v_max_i32_dpp %[r], %[r], %[r] row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_e64 %[lk], %[k0], %[k1], %[m01]\n\t"
      "v_cndmask_b32_e64 %[tk], %[k2], %[k3], %[m23]\n\t"
      "v_max_i32_dpp %[r], %[r], %[r] row_mirror row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_e64 %[lx], %[lx], %[tx], %[mh]\n\t"
      "v_cndmask_b32_e64 %[ly], %[ly], %[ty], %[mh]\n\t"
      "v_max_i32_dpp %[r], %[r], %[r] row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "v_cndmask_b32_e64 %[lz], %[lz], %[tz], %[mh]\n\t"
      "v_cndmask_b32_e64 %[lk], %[lk], %[tk], %[mh]\n\t"
      "v_max_i32_dpp %[r], %[r], %[r] row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_readlane_b32 %[wm], %[r], 63"
      : [m01] "=&s"(m01), [m23] "=&s"(m23), [mh] "=&s"(mh), [cv] "=&v"(cv),
        [v23] "=&v"(v23), [r] "=&v"(r), [lx] "=&v"(lx), [ly] "=&v"(ly),
        [lz] "=&v"(lz), [lk] "=&v"(lk), [tx] "=&v"(tx), [ty] "=&v"(ty),
        [tz] "=&v"(tz), [tk] "=&v"(tk), [wm] "=s"(wm)
      : [h0] "v"(hv[0]), [h1] "v"(hv[1]), [h2] "v"(hv[2]), [h3] "v"(hv[3]),
        [x0] "v"(hx[0][0]), [x1] "v"(hx[0][1]), [x2] "v"(hx[1][0]), [x3] "v"(hx[1][1]),
        [y0] "v"(hy[0][0]), [y1] "v"(hy[0][1]), [y2] "v"(hy[1][0]), [y3] "v"(hy[1][1]),
        [z0] "v"(hz[0][0]), [z1] "v"(hz[0][1]), [z2] "v"(hz[1][0]), [z3] "v"(hz[1][1]),
        [k0] "v"(hk[0]), [k1] "v"(hk[1]), [k2] "v"(hk[2]), [k3] "v"(hk[3]));
}

// ---- publishing picks to the cold waves (the SA1 sampler here, the chain in fps.hip) -------
// A pick's slot is (x, y, z, w) with w = point index | pick_tag(j), j the number of the first
// pick of the slot's batch in the launch (the chain adds the earlier stages' picks). The protocol
// is the LLVM AMDGPU memory model's own mapping of a workgroup-scope release / acquire on LDS,
// not the in-order execution of a wave's DS operations (which no document promises across waves,
// and which a 16-byte centre write followed by the count did break:
// profiles/r5/chain_hot/pipe_stress_b128_publish.json):
//  * release: the count store that makes slot p visible is issued only after an
//    s_waitcnt lgkmcnt has seen slot p's writes complete (hipcc emits exactly that wait before a
//    __ATOMIC_RELEASE workgroup store to LDS). So the wait never stalls the hot wave, each pick
//    publishes the count of the picks BEFORE it: slot p is written, then lgkmcnt(4) (everything
//    but those 4 writes is complete -- slot p - 1 was written ~500 cycles earlier), then count p.
//    The batch's last pick goes out with the end flag, after lgkmcnt(0);
//  * acquire: a cold wave reads the count with __ATOMIC_ACQUIRE (ds_read, s_waitcnt lgkmcnt(0)
//    before any later LDS read), then the slots below it.
// On top, the consumer checks every slot's tag and re-polls on a mismatch. A stale slot cannot
// carry the batch's tag: a slot is written once per batch, batches start at increasing pick
// numbers (a batch that wrote a slot made a pick), and the slots are cleared (tag 0) at the
// launch's start. The tag is per batch, not per pick, so the hot entries carry it from before
// the pick loop and a pick costs no tag arithmetic (a per-pick tag OR cost the SA1 sampler ~30
// cycles a pick, 6 %: profiles/r6/pubab). The check is what a build that publishes the count
// BEFORE the centre (-DPN2_PUBLISH_BROKEN=1, csrc/Makefile target torntest) leans on: it stays
// index-exact and counts the torn reads it caught (pn2_torn_reads, tests/test_gpu_a_fullsize.py).
#ifndef PN2_PUBLISH_BROKEN
#define PN2_PUBLISH_BROKEN 0
#endif
PN2_DEV uint32_t pick_tag(int p) { return ((uint32_t)(p + 1) & 0xFFFFu) << 16; }
constexpr uint32_t kPickIdxMask = 0xFFFFu;  // point indices < 65536 (N <= 16384 here)
constexpr int kPickTagMax = 0xFFFF;         // picks per launch below this: tags never repeat
#if PN2_PUBLISH_BROKEN
__device__ unsigned int g_torn_reads;
#define PN2_TORN_SEEN() if (lane == 0) atomicAdd(&g_torn_reads, 1u)
#else
#define PN2_TORN_SEEN()
#endif

// publish pick L from the winning lane itself (exec = lane L only): its lx, ly, lz and lw (the
// point index with the batch's tag) are the slot at LDS address va_c; then, once the writes
// before them are complete, the count vcnt (the picks of this batch before this one) to va_n.
// The centre's coordinates come back to SGPRs inside the same block (v_readlane ignores exec),
// so no wait states follow the exec restore; L comes from SALU (no lane-select wait).
PN2_DEV void hot_publish(int L, int va_c, int va_n, int vcnt, float lx, float ly, float lz,
                         int lw, float& cx, float& cy, float& cz) {
#if PN2_PUBLISH_BROKEN
  // DIAGNOSTIC: the count (including this pick) first, the slot ~800 cycles later (longer than
  // a cold wave takes from reading the count to reading the slots)
  int kt;
  asm volatile("v_add_u32 %0, 1, %1\n\tds_write_b32 %2, %0\n\ts_sleep 12"
               : "=&v"(kt) : "v"(vcnt), "v"(va_n) : "memory");
#endif
  uint64_t sv;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\t"
      "s_lshl_b64 exec, 1, %[L]\n\t"
      "ds_write_b32 %[a], %[x]\n\t"
      "ds_write_b32 %[a], %[y] offset:4\n\t"
      "ds_write_b32 %[a], %[z] offset:8\n\t"
      "ds_write_b32 %[a], %[k] offset:12\n\t"
#if !PN2_PUBLISH_BROKEN
      "s_waitcnt lgkmcnt(4)\n\t"
      "ds_write_b32 %[c], %[n]\n\t"
#endif
      "v_readlane_b32 %[cx], %[x], %[L]\n\t"
      "v_readlane_b32 %[cy], %[y], %[L]\n\t"
      "v_readlane_b32 %[cz], %[z], %[L]\n\t"
      "s_mov_b64 exec, %[sv]"
      : [sv] "=&s"(sv), [cx] "=&s"(cx), [cy] "=&s"(cy), [cz] "=&s"(cz)
      : [L] "s"(L), [a] "v"(va_c), [c] "v"(va_n), [x] "v"(lx), [y] "v"(ly), [z] "v"(lz),
        [k] "v"(lw), [n] "v"(vcnt)
      : "memory", "scc");
}

// the end of a batch: every slot write complete (release), then the final count | end flag
PN2_DEV void publish_end(int* word, int value) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(word, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the hot values after the pick (cx, cy, cz): running min with the fp32 distance
// ((dx*dx + dy*dy) + dz*dz), two entries per packed instruction
template <int HP>
PN2_DEV void hot_update(int (&hv)[2 * HP], const hf2 (&hx)[HP], const hf2 (&hy)[HP],
                        const hf2 (&hz)[HP], float cx, float cy, float cz) {
  const hf2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
#pragma unroll
  for (int h = 0; h < HP; ++h) {
    const hf2 dx = hx[h] - c2x, dy = hy[h] - c2y, dz = hz[h] - c2z;
    const hf2 d = (dx * dx + dy * dy) + dz * dz;
    hv[2 * h] = min(hv[2 * h], __float_as_int(d.x));
    hv[2 * h + 1] = min(hv[2 * h + 1], __float_as_int(d.y));
  }
}

// The cold waves' wait for published centres is bounded (the hot wave always ends its batch,
// so the bound is never reached in a correct run: ~0.1 s of polling against ~25 us per batch).
// Reaching it stores PN2_FAULT_FPS_POLL into *fault (the host reports PN2_EFAULT); a build
// with a tiny bound (csrc/Makefile target polltest) exercises that path.
#ifndef PN2_FPS_POLL_LIMIT
#define PN2_FPS_POLL_LIMIT (1 << 22)
#endif

// LEAN (N <= 8192, one point per lane per cell): the cloud is NOT copied to LDS. Its
// coordinates are read from global memory (L2) at setup, the cold lanes keep x, y, z of their
// points in VGPRs, and a hot entry carries its point's coordinates (the hot wave reads no
// coordinate at a round start); the batch buffer and the hot set live in the sort histogram's
// LDS once the sort is done. ~53 KB of LDS instead of ~155 KB: with fewer VGPRs too
// (fps_hotcull_lean_kernel), a CU that side-lane workgroups partly occupy can still take a
// sampler workgroup (the 155 KB / 128-VGPR workgroup waits for a CU to drain completely).
// KG: also the picks' automatic-edge grid into kgrid (pn2_fps_chain_grid), built by the
// workgroup after its last pick (a separate instantiation: the product sampler keeps its code)
template <int NW, int PPT, int NPTS, bool STAMP = false, int PRIO = 0, int HQ = 2, int PPC = 1,
          bool LEAN = false, bool KG = false>
__device__ __attribute__((always_inline)) inline void hotcull_body(
    const float* __restrict__ xyz, int N, int M, int32_t* __restrict__ idx,
    float* __restrict__ new_xyz, int* __restrict__ fault, char* __restrict__ kgrid = nullptr) {
  constexpr int BLOCK = 64 * NW;
  constexpr int NCW = NW - 1;  // cold waves
  constexpr int NCELL = NCW * PPT;
  constexpr int GRP = kWave / PPT;      // centres per group test (lane = centre * PPT + cell)
  constexpr int K = 64 * HQ;            // hot-set capacity: HQ entries per lane of wave 0
  constexpr int NT = 12;                // thresholds
  constexpr int NWIN = 4;               // thresholds counted per refresh
  constexpr int NBK = 4096;             // sort buckets (16^3 Morton)
  constexpr int kEnd = 1 << 16;         // sj flag: the batch is complete
  constexpr int SPT = (NPTS + BLOCK - 1) / BLOCK;  // setup: points per thread
  static_assert(PPC == 1 || PPC == 2, "points per lane per cell");
  constexpr int CP = kWave * PPC;        // points per cell
  static_assert(NCELL * CP >= NPTS, "cold capacity");
  static_assert(PPT <= 32 && GRP >= 1, "slot masks");
  static_assert(NW <= 16 && NWIN == 4, "choice: lane 16 i + v = (threshold i, wave v)");
  using f2 = float __attribute__((ext_vector_type(2)));

  // the cloud's coordinates: an LDS copy when it fits beside the rest (NPTS <= 8192),
  // otherwise read from global memory (L2) -- only at setup and once per round
  static_assert(!LEAN || (PPC == 1 && NPTS <= 8192), "LEAN: one point per lane per cell");
  constexpr bool XYZ_LDS = NPTS <= 8192 && !LEAN;
  __shared__ __attribute__((aligned(16))) float sxyz[XYZ_LDS ? 3 * NPTS : 4];
  __shared__ int sperm[NPTS];         // sorted position -> point index
  // bucket counts, then offsets; LEAN: then the batch buffer and the hot set (below)
  constexpr int kLeanWords = (K + 1) * 4 + K * 4 + K;
  __shared__ __attribute__((aligned(16))) uint32_t shist[LEAN && kLeanWords > NBK ? kLeanWords : NBK];
  __shared__ float4 scell[2 * NCELL]; // cell boxes (lo, hi)
  __shared__ float4 scl_[LEAN ? 1 : K + 1];  // centres of the current batch (x, y, z, idx)
  __shared__ uint2 sh_[LEAN ? 1 : K];        // hot entries (running min bits, point index)
  float4* const scl = LEAN ? reinterpret_cast<float4*>(shist) : scl_;
  uint2* const sh = sh_;
  // LEAN hot entries: (running min bits, point index, x, y) and z
  uint4* const shx = reinterpret_cast<uint4*>(shist) + (K + 1);
  float* const shz = reinterpret_cast<float*>(shist) + (K + 1) * 4 + K * 4;
  __shared__ uint64_t swk[NW];        // per-wave (value + 1, ~key) of the exact argmax
  __shared__ float sbox[NW][8];
  __shared__ int swmax[NW];
  __shared__ int sj[2];               // published centres of a batch | kEnd once complete (by round parity)
  __shared__ uint32_t swcnt[NW][4];   // per-wave counts above the round's thresholds
  // without the LDS copy (NPTS > 8192) the cold points' z coordinates live in the freed LDS
  // instead of VGPRs (at 16 waves the kernel is held to 128 VGPRs): lane-consecutive, so a
  // cold wave's read of one slot is conflict-free
  constexpr bool ZLDS = !XYZ_LDS && !LEAN;
  __shared__ float scz[ZLDS ? NCW * PPT * PPC * kWave : 1];

  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(t / kWave);
  const int cw = w - 1;  // cold wave index (-1: the hot wave)
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0;
  unsigned long long n_refresh = 0, n_stall = 0, n_pairs = 0, n_hot = 0, clk0 = 0;
  unsigned long long n_tail_grp = 0;
  unsigned long long ev[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // STAMP: this round's events
  unsigned long long n_grp = 0, n_grp_cyc = 0, n_poll = 0;
  if constexpr (STAMP) {
    clk0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
  }

  // ---- setup: LDS copy, bounding box, counting sort by Morton bucket, cells -------------
  if constexpr (XYZ_LDS) {
    if ((((uintptr_t)P) & 15) == 0) {  // 16 B per lane: one pass of wide coalesced loads
      const int n4 = (3 * N) >> 2;
      const float4* __restrict__ P4 = reinterpret_cast<const float4*>(P);
      for (int e = t; e < n4; e += BLOCK) reinterpret_cast<float4*>(sxyz)[e] = P4[e];
      for (int e = 4 * n4 + t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
    } else {
      for (int e = t; e < 3 * N; e += BLOCK) sxyz[e] = P[e];
    }
  }
  const float* __restrict__ X = XYZ_LDS ? (const float*)sxyz : P;  // coordinates
  for (int e = t; e < NBK; e += BLOCK) shist[e] = 0u;
  // the batch slots start untagged (LEAN: they alias shist, whose counts / offsets < 65536
  // carry tag 0 too)
  if constexpr (!LEAN)
    for (int e = t; e < K + 1; e += BLOCK) scl_[e] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  if (t < NW * 4) swcnt[t / 4][t % 4] = 0u;
  // KG: the grid's address waits in LDS until the epilogue (a pointer kept in registers
  // through the pick loop made the allocator spill inside it)
  __shared__ char* s_kgrid;
  if (KG && t == 0) s_kgrid = NX && M <= NBK ? kgrid + (size_t)b * grid_stride(M) : nullptr;
  __syncthreads();
  {
    float mx[3] = {-INFINITY, -INFINITY, -INFINITY}, mn[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = t; k < N; k += BLOCK) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        mx[a] = fmaxf(mx[a], X[3 * k + a]);
        mn[a] = fmaxf(mn[a], -X[3 * k + a]);
      }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      mx[a] = wave_max_f32(mx[a]);
      mn[a] = wave_max_f32(mn[a]);
    }
    if (lane == 0) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        sbox[w][a] = mx[a];
        sbox[w][4 + a] = mn[a];
      }
    }
  }
  __syncthreads();
  float blo[3], bsc[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float hi = -INFINITY, nlo = -INFINITY;
    for (int v = 0; v < NW; ++v) {
      hi = fmaxf(hi, sbox[v][a]);
      nlo = fmaxf(nlo, sbox[v][4 + a]);
    }
    blo[a] = -nlo;
    const float ext = hi - blo[a];
    bsc[a] = ext > 0.0f ? 16.0f / ext : 0.0f;
  }
  int code[SPT], rank[SPT];
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const int k = t + i * BLOCK;
    if (k < N) {
      uint32_t c = 0;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int q = min(max((int)((X[3 * k + a] - blo[a]) * bsc[a]), 0), 15);
#pragma unroll
        for (int bit = 0; bit < 4; ++bit) c |= (uint32_t)((q >> bit) & 1) << (3 * bit + a);
      }
      code[i] = (int)c;
      rank[i] = (int)atomicAdd(&shist[c], 1u);
    } else {
      code[i] = 0;
      rank[i] = 0;
    }
  }
  __syncthreads();
  {
    constexpr int PB = (NBK + BLOCK - 1) / BLOCK;
    uint32_t c[PB], s = 0;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      c[i] = PB * t + i < NBK ? shist[PB * t + i] : 0u;
      s += c[i];
    }
    const uint32_t ex = wave_excl_scan(s, lane);
    if (lane == kWave - 1) swmax[w] = (int)(ex + s);
    __syncthreads();
    uint32_t base = 0;
    for (int v = 0; v < w; ++v) base += (uint32_t)swmax[v];
    uint32_t run = base + ex;
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      if (PB * t + i < NBK) shist[PB * t + i] = run;
      run += c[i];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const int k = t + i * BLOCK;
    if (k < N) sperm[shist[code[i]] + rank[i]] = k;
  }
  __syncthreads();
  // cell boxes: 8 lanes per cell, each folds 8 consecutive sorted points, then DPP within 8
  for (int c = t >> 3; c < NCELL; c += BLOCK / 8) {
    float lo3[3] = {INFINITY, INFINITY, INFINITY}, hi3[3] = {-INFINITY, -INFINITY, -INFINITY};
    const int base = c * CP + (t & 7) * (8 * PPC);
#pragma unroll
    for (int i = 0; i < 8 * PPC; ++i) {
      const int pos = base + i;
      if (pos < N) {
        const int k = sperm[pos];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          lo3[a] = fminf(lo3[a], X[3 * k + a]);
          hi3[a] = fmaxf(hi3[a], X[3 * k + a]);
        }
      }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#define PN2_BOX_DPP(C)                                                                       \
  lo3[a] = fminf(lo3[a], __int_as_float(__builtin_amdgcn_update_dpp(                         \
                             __float_as_int(lo3[a]), __float_as_int(lo3[a]), C, 0xF, 0xF,    \
                             false)));                                                       \
  hi3[a] = fmaxf(hi3[a], __int_as_float(__builtin_amdgcn_update_dpp(                         \
                             __float_as_int(hi3[a]), __float_as_int(hi3[a]), C, 0xF, 0xF,    \
                             false)))
      PN2_BOX_DPP(kDppXor1);
      PN2_BOX_DPP(kDppXor2);
      PN2_BOX_DPP(kDppHalfMirror);
#undef PN2_BOX_DPP
    }
    if ((t & 7) == 0) {
      scell[2 * c] = make_float4(lo3[0], lo3[1], lo3[2], 0.0f);
      scell[2 * c + 1] = make_float4(hi3[0], hi3[1], hi3[2], 0.0f);
    }
  }
  if (t == 0) {  // the first batch: centre 0 (tf_sampling_g.cu:121-125), already complete
    scl[0] = make_float4(X[0], X[1], X[2], __uint_as_float(pick_tag(0)));
    sj[0] = 1 | kEnd;
    sj[1] = 0;
    for (int v = 0; v < NW; ++v) swmax[v] = -1;  // waves without cells keep -1
  }
  __syncthreads();

  // cold registers: point h of cell s of cold lane (cw, lane) = sorted position
  // (s * NCW + cw) * CP + h * 64 + lane, held at index s * PPC + h: slot s of the cold waves
  // is cells s * NCW ... s * NCW + NCW - 1 of the Morton order, so every wave's cells spread
  // over the whole cloud and the waves get similar numbers of (cell, centre) pairs (with
  // contiguous cells the wave holding the region being sampled lagged the others)
  float px[PPT * PPC], py[PPT * PPC], pz[PPT * PPC];
  int tb[PPT * PPC];
  // The hot wave's SIMD (SIMD 0: waves 0, 4, 8, 12) holds the cold waves 4, 8 and 12 too; they
  // take issue slots from the pick chain. Those three hold kLD cells fewer than the others
  // (SA1: 7 instead of 9 at NW = 16, PPT = 9: 21 cold cells on SIMD 0 against 35-36 on SIMDs
  // 1-3; MSG: 8),
  // out of the spare slots (135 for 128 cells). Slots are ranked s-major over the valid ones
  // (valid = not a dropped slot of a light wave), the dropped ones after them (cells past N:
  // empty), so every cell is held once and the picks do not depend on it. The SA1 sampler over
  // the known grid alone: 380.8 -> 370.0 us at B = 16 (profiles/r6/light: cold waves 3 / 6
  // cells lighter or the youngest waves lighter were slower or the same).
  // (-DPN2_SA1_LIGHT_MASK / _D: other layouts for A/B builds; mask 0 = slot s of cold wave cw
  // is cell s * NCW + cw)
#ifdef PN2_SA1_LIGHT_MASK
  constexpr uint32_t kLight = PN2_SA1_LIGHT_MASK;
  constexpr int kWantD = PN2_SA1_LIGHT_D;
#else
  constexpr uint32_t kLight = [] {
    uint32_t m = 0;
    for (int c = 0; c < NCW; ++c)
      if ((c + 1) % 4 == 0) m |= 1u << c;
    return m;
  }();
  // 2 slots each with one point per lane per cell (SA1); 1 with two (MSG SA1, 16,384 points:
  // its cells hold twice the work, and 2 dropped slots made the cold SIMDs the bound, 0.341 ms
  // against 0.331 with 1 and 0.333 with none at B = 8, profiles/r6/light/msg)
  constexpr int kWantD = PPC == 1 ? 2 : 1;
#endif
  constexpr int kSpare = NCELL - (NPTS + CP - 1) / CP;  // slots beyond the cells a cloud fills
  constexpr int kNLW = __builtin_popcount(kLight);
  constexpr int kPerW = kSpare / (kNLW > 0 ? kNLW : 1);  // dropped slots each light wave can take
  constexpr int kLD = kNLW == 0 ? 0 : (kPerW < kWantD ? kPerW : kWantD);
  constexpr int kNL = kLD > 0 ? __builtin_popcount(kLight) : 0;
  static_assert(kLight < (1u << NCW), "light waves are cold waves");
  static_assert((NCELL - kNL * kLD) * CP >= NPTS, "light layout capacity");
  const int lbefore = cw >= 0 ? __builtin_popcount(kLight & ((1u << cw) - 1u)) : 0;
  const bool light = cw >= 0 && ((kLight >> cw) & 1u);
  auto cellof = [&](int s) {
    if (kNL == 0 || s < PPT - kLD) return s * NCW + cw;
    const int q = s - (PPT - kLD);
    if (!light) return s * NCW - kNL * q + cw - lbefore;
    return NCELL - kNL * kLD + q * kNL + lbefore;
  };
  auto spos = [&](int s, int h) { return cellof(s) * CP + h * kWave + lane; };
  // a cell's maximum running min (every lane gets it)
#define PN2_CELLMAX(s) wave_max_i32(PPC == 1 ? tb[(s) * PPC] : max(tb[(s) * PPC], tb[(s) * PPC + PPC - 1]))
  int Tm[PPT];  // exact max running min of each cell (wave-uniform), -1 = empty cell
  // group test: lane l tests cell (cw, l % PPT) against centre l / PPT of the group
  float4 glo = make_float4(INFINITY, INFINITY, INFINITY, 0.0f), ghi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
  int tmv = -1;
  if (cw >= 0) {
#pragma unroll
    for (int s = 0; s < PPT; ++s) {
      bool any = false;
#pragma unroll
      for (int h = 0; h < PPC; ++h) {
        const int pos = spos(s, h);
        const bool in = pos < N;
        const int k = in ? sperm[pos] : 0;
        px[s * PPC + h] = X[3 * k];
        py[s * PPC + h] = X[3 * k + 1];
        if constexpr (ZLDS) scz[(cw * PPT * PPC + s * PPC + h) * kWave + lane] = X[3 * k + 2];
        else pz[s * PPC + h] = X[3 * k + 2];
        tb[s * PPC + h] = in ? __float_as_int(kInitTemp) : -1;
        any = any || __builtin_amdgcn_ballot_w64(in) != 0;
      }
      Tm[s] = any ? __float_as_int(kInitTemp) : -1;
    }
    if (lane < GRP * PPT) {
      glo = scell[2 * cellof(lane % PPT)];
      ghi = scell[2 * cellof(lane % PPT) + 1];
    }
#pragma unroll
    for (int s = 0; s < PPT; ++s) tmv = lane % PPT == s ? Tm[s] : tmv;
  }
  PN2_STAMP(7)

  int j = 0;                // picks written to the outputs
  int rp = 0;               // round parity: sj[rp] describes this round's batch
  int tlo = 2;              // first threshold of the counted window
  int T = 0, nh = 0;        // the hot phase's threshold and hot-set size
  bool hot_turn = false;
  uint32_t dirty = 0;  // cold waves: cells whose Tmax is stale (an upper bound)
  // One round's end, after the hot phase (wave 0) or the cold application (waves 1..): three
  // barriers with the choice between them. Instantiated separately for the hot wave and the
  // cold waves, so the hot wave's loop carries none of the cold waves' point registers.
  auto round_end = [&](auto cold_tag, int round) -> bool {
    constexpr bool COLD = decltype(cold_tag)::value;
    __syncthreads();  // B1: the batch is complete and applied; Tmax and counts are current
    PN2_EV(2)
    PN2_STAMP(2)
    // (cold wave 1 stored the batch's outputs group by group, so the barriers' s_waitcnt finds
    // at most the last group's stores outstanding)
    j += sj[rp] & (kEnd - 1);
    if (j >= M) return true;
    if constexpr (STAMP) ++n_refresh;
    int top;
    {
      const int v = lane < NW ? swmax[lane] : -1;
      top = __builtin_amdgcn_readfirstlane(wave_max_i32(v));
    }
    // ---- this round's thresholds (fractions of the exact maximum; every wave computes the
    // same bits) and each wave's counts above them (cells at or below a threshold count 0)
    int tau[NWIN];
    {
      const float tf = __int_as_float(max(top, 0));
#pragma unroll
      for (int i = 0; i < NWIN; ++i)
        tau[i] = (int)uniform_u32((uint32_t)__float_as_int(tf * kCullFrac[tlo + i]));
    }
    if constexpr (COLD) {
      uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
      static_assert(NWIN == 4, "four counters");
#pragma unroll
      for (int s = 0; s < PPT; ++s) {
        if (Tm[s] > tau[0]) {
#pragma unroll
          for (int h = 0; h < PPC; ++h) {
            const int e = s * PPC + h;
            c0 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(tb[e] > tau[0]));
            c1 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(tb[e] > tau[1]));
            c2 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(tb[e] > tau[2]));
            c3 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(tb[e] > tau[3]));
          }
        }
      }
      if (lane < NWIN) swcnt[w][lane] = lane == 0 ? c0 : lane == 1 ? c1 : lane == 2 ? c2 : c3;
    }
    PN2_EV(3)
    PN2_STAMP(3)
    __syncthreads();  // B2: counts complete
    PN2_EV(4)
    PN2_STAMP(4)
    // ---- choice: the lowest window threshold whose total count is in [1, K]. Lane
    // 16 i + v holds wave v's count above tau[i]; 16-lane row sums give the totals.
    const int cvw = lane & 15, ciw = lane >> 4;
    const uint32_t cnt = cvw < NW ? swcnt[cvw][ciw] : 0u;
    uint32_t tot = cnt;
#define PN2_ADD_DPP(C) tot += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)tot, C, 0xF, 0xF, false)
    PN2_ADD_DPP(kDppXor1);
    PN2_ADD_DPP(kDppXor2);
    PN2_ADD_DPP(kDppHalfMirror);
    PN2_ADD_DPP(kDppMirror);
#undef PN2_ADD_DPP
    const uint64_t fit = __builtin_amdgcn_ballot_w64(cvw == 0 && tot >= 1u && tot <= (uint32_t)K);
    const int ti = fit ? (int)__builtin_ctzll(fit) >> 4 : -1;
    const bool stall = ti < 0;
    T = 0;
#pragma unroll
    for (int i = 0; i < NWIN; ++i) T = ti == i ? tau[i] : T;
    nh = stall ? 0 : __builtin_amdgcn_readlane((int)tot, ti * 16);
    int wbase = 0;  // this wave's first hot entry: the counts of the waves before it
    {
      uint32_t pre = ciw == ti && cvw < w ? cnt : 0u;
#define PN2_ADD_DPP(C) pre += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pre, C, 0xF, 0xF, false)
      PN2_ADD_DPP(kDppXor1);
      PN2_ADD_DPP(kDppXor2);
      PN2_ADD_DPP(kDppHalfMirror);
      PN2_ADD_DPP(kDppMirror);
#undef PN2_ADD_DPP
      if (!stall) wbase = __builtin_amdgcn_readlane((int)pre, ti * 16);
    }
    // next window: two below this choice (lower thresholds = bigger hot sets), or up; the next
    // thresholds scale with this round's maximum
    tlo = !stall ? min(max(tlo + ti - 2, 0), NT - NWIN) : min(tlo + NWIN, NT - NWIN);
    if (t == 0) sj[rp ^ 1] = 0;  // the next round's batch starts empty (last read in round - 1)
    if (!stall) {
      if constexpr (COLD) {
        // ---- hot set: every point above T, at this wave's offset
        int base = wbase;
#pragma unroll
        for (int s = 0; s < PPT; ++s) {
          if (Tm[s] > T) {
#pragma unroll
            for (int h = 0; h < PPC; ++h) {
              const int e = s * PPC + h;
              const uint64_t m = __builtin_amdgcn_ballot_w64(tb[e] > T);
              const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                  (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
              if (tb[e] > T) {
                if constexpr (LEAN) {
                  shx[base + (int)below] = make_uint4((uint32_t)tb[e], (uint32_t)sperm[spos(s, h)],
                                                      __float_as_uint(px[e]), __float_as_uint(py[e]));
                  shz[base + (int)below] = pz[e];
                } else {
                  sh[base + (int)below] = make_uint2((uint32_t)tb[e], (uint32_t)sperm[spos(s, h)]);
                }
              }
              base += __builtin_popcountll(m);
            }
          }
        }
      }
    } else {
      // ---- exact block argmax: (value desc, key asc) as one 64-bit max
      uint64_t best = 0;
      if constexpr (COLD) {
#pragma unroll
        for (int e = 0; e < PPT * PPC; ++e) {
          const uint64_t v = tb[e] < 0 ? 0ull
                                       : pack64(~cull_key(sperm[spos(e / PPC, e % PPC)]),
                                                (uint32_t)tb[e] + 1u);
          best = v > best ? v : best;
        }
        best = wave_max_u64(best);
      }
      if (lane == 0) swk[w] = best;
      if constexpr (STAMP) ++n_stall;
    }
    PN2_EV(5)
    PN2_STAMP(5)
    __syncthreads();  // B3: hot set (or the per-wave argmax) complete
    PN2_EV(6)
    PN2_STAMP(6)
    if constexpr (STAMP) {
      if (b == 0 && lane == 0 && round < 64) {
#pragma unroll
        for (int k = 0; k < 8; ++k) g_cull_ev[(round * 16 + w) * 8 + k] = ev[k];
      }
    }
    if (stall) {
      uint64_t best = lane < NW ? swk[lane] : 0ull;
      best = uniform_u64(wave_max_u64(best));
      const uint32_t key = ~(uint32_t)best;
      const int k = (int)((key >> 16) + ((key & 0xFFFFu) << 9));
      if (top <= 0) {
        // every running min is 0 and stays 0: each remaining pick is the same point
        for (int e = j + t; e < M; e += BLOCK) {
          I[e] = k;
          if (NX) {
            NX[3 * e] = X[3 * k];
            NX[3 * e + 1] = X[3 * k + 1];
            NX[3 * e + 2] = X[3 * k + 2];
          }
        }
        return true;
      }
      if (t == 0) {
        scl[0] = make_float4(X[3 * k], X[3 * k + 1], X[3 * k + 2],
                             __uint_as_float((uint32_t)k | pick_tag(j)));
        publish_end(&sj[rp ^ 1], 1 | kEnd);
      }
    }
    hot_turn = !stall;
    rp ^= 1;
    PN2_STAMP(6)
    return false;
  };
  if (w == 0) {
    for (int round = 0; round <= M; ++round) {
      if (hot_turn) {
        // ---- hot phase: certified picks while the best hot value is above T, each one
        // published to the cold waves as it is made (scl[jj] with its tag, then -- released --
        // the count sj of the picks before it; hot_publish)
        static_assert(HQ == 2 || HQ == 4, "hot entries per lane");
        int hv[HQ], hk[HQ];
        uint32_t hkey[HQ];
        float qx[HQ], qy[HQ], qz[HQ];  // LEAN: the entries' coordinates, carried in the set
#pragma unroll
        for (int q = 0; q < HQ; ++q) {
          const int e = lane + q * kWave;
          if constexpr (LEAN) {
            const uint4 en = e < nh ? shx[e] : make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
            qz[q] = e < nh ? shz[e] : 0.0f;
            hv[q] = (int)en.x;
            hk[q] = (int)en.y;
            qx[q] = __uint_as_float(en.z);
            qy[q] = __uint_as_float(en.w);
          } else {
            const uint2 en = e < nh ? sh[e] : make_uint2(0xFFFFFFFFu, 0u);
            hv[q] = (int)en.x;
            hk[q] = (int)en.y;
          }
          hkey[q] = hv[q] >= 0 ? cull_key(hk[q]) : 0xFFFFFFFFu;
        }
        // a lane's entries in tie order (odd-even transposition sort by key): then a tournament
        // of strict '>' comparisons, lower entry first, picks the reference's winner in a lane
#pragma unroll
        for (int pass = 0; pass < HQ; ++pass) {
#pragma unroll
          for (int q = pass & 1; q + 1 < HQ; q += 2) {
            if (hkey[q + 1] < hkey[q]) {
              const int v = hv[q], k = hk[q];
              const uint32_t y = hkey[q];
              hv[q] = hv[q + 1]; hk[q] = hk[q + 1]; hkey[q] = hkey[q + 1];
              hv[q + 1] = v; hk[q + 1] = k; hkey[q + 1] = y;
              if constexpr (LEAN) {
                const float ax = qx[q], ay = qy[q], az = qz[q];
                qx[q] = qx[q + 1]; qy[q] = qy[q + 1]; qz[q] = qz[q + 1];
                qx[q + 1] = ax; qy[q + 1] = ay; qz[q + 1] = az;
              }
            }
          }
        }
        constexpr int HP = HQ / 2;  // coordinate pairs
        f2 hx[HP], hy[HP], hz[HP];
#pragma unroll
        for (int q = 0; q < HQ; ++q) {
          hx[q / 2][q % 2] = LEAN ? qx[q] : X[3 * hk[q]];
          hy[q / 2][q % 2] = LEAN ? qy[q] : X[3 * hk[q] + 1];
          hz[q / 2][q % 2] = LEAN ? qz[q] : X[3 * hk[q] + 2];
          hk[q] |= (int)pick_tag(j);  // the slots' w: the point index with the batch's tag
        }
        const int lim = min(K, M - j);
        int jj = 0;
        if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO);
        // every hot-set load is complete before the loop: the wait-count pass then has no
        // pending LDS load to wait for inside it, and the picks' publishing stores stay off
        // the dependency chain (an in-loop lgkmcnt(0) would wait for the previous pick's)
        __builtin_amdgcn_s_waitcnt(0xC07F);
        // publishing addresses and the published count in VGPRs, advanced by one VALU add per
        // pick (as SGPRs they cost an SALU add and a v_mov each for the DS stores)
        // (vcnt: the picks of this batch so far, published after each pick's slot)
        int va_c, va_n, vcnt;
        asm volatile("v_mov_b32 %0, %1" : "=v"(va_c)
                     : "s"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)&scl[0]));
        asm volatile("v_mov_b32 %0, %1" : "=v"(va_n)
                     : "s"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) int*)&sj[rp]));
        asm volatile("v_mov_b32 %0, 0" : "=v"(vcnt));
        // the pick loop ends when the best hot value is no longer above T; it cannot run past
        // the nh <= K hot entries (a picked entry drops to 0 <= T), so only the last batch of
        // the cloud (fewer than K picks left) needs a count test per pick
        auto pick_loop = [&](auto checked_tag) {
          constexpr bool CHECKED = decltype(checked_tag)::value;
          for (;;) {
            int cv, lk, wm;
            float lx, ly, lz;
            uint64_t m01 = 0, m23 = 0, mh = 0;
            if constexpr (HQ == 4) {
              hot_best4(hv, hx, hy, hz, hk, cv, lx, ly, lz, lk, wm, m01, m23, mh);
            } else {
              const bool b01 = hv[1] > hv[0];
              cv = b01 ? hv[1] : hv[0];
              lx = b01 ? hx[0][1] : hx[0][0];
              ly = b01 ? hy[0][1] : hy[0][0];
              lz = b01 ? hz[0][1] : hz[0][0];
              lk = b01 ? hk[1] : hk[0];
              // the winner's coordinates are selected here, beside the reduction, not after it
              asm volatile("" ::"v"(lx), "v"(ly), "v"(lz), "v"(lk));
              wm = __builtin_amdgcn_readlane(wave_max_i32_l63(cv), 63);
            }
            if (!(wm > T)) break;
            const uint64_t hold = __builtin_amdgcn_ballot_w64(cv == wm);
            int L;
            if (__builtin_popcountll(hold) == 1) {
              L = (int)__builtin_ctzll(hold);
            } else {  // equal values: the smallest tie key among the holders
              uint32_t ck;
              if constexpr (HQ == 4) {  // the same selects as the lane's best entry
                uint32_t k23;
                asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(ck)
                             : "v"(hkey[0]), "v"(hkey[1]), "s"(m01));
                asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(k23)
                             : "v"(hkey[2]), "v"(hkey[3]), "s"(m23));
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(ck) : "v"(k23), "s"(mh));
              } else {
                ck = hv[1] > hv[0] ? hkey[1] : hkey[0];
              }
              const uint32_t km = ~uniform_u32(wave_max_u32(cv == wm ? ~ck : 0u));
              L = (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(cv == wm && ck == km));
            }
            float cx, cy, cz;
            hot_publish(L, va_c, va_n, vcnt, lx, ly, lz, lk, cx, cy, cz);
            __builtin_amdgcn_sched_barrier(0);
            hot_update<HP>(hv, hx, hy, hz, cx, cy, cz);  // the next pick depends on it
            va_c += 16;
            vcnt += 1;
            if constexpr (CHECKED)
              if (__builtin_amdgcn_readfirstlane(vcnt) >= lim) break;
          }
        };
        if (lim >= K) pick_loop(std::false_type{});
        else if (lim > 0) pick_loop(std::true_type{});
        jj = __builtin_amdgcn_readfirstlane(vcnt);
        if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(0);
        if (lane == 0) publish_end(&sj[rp], jj | kEnd);
        if constexpr (STAMP) {
          n_hot += jj;
        }
      }
      PN2_EV(0)
      PN2_STAMP(7)
      if (round_end(std::false_type{}, round)) break;
    }
  } else {
    for (int round = 0; round <= M; ++round) {
      // ---- cold waves: apply the batch's centres as the hot wave publishes them, GRP at a
      // time (the last, short group after the end flag), culled by the box test against the
      // cells' Tmax (stale within the round = larger = still a valid bound). A touched cell is
      // marked dirty; its exact Tmax is recomputed when the wave would otherwise wait, and the
      // rest at the end of the batch.
      int applied = 0;
      bool stop = false;
      unsigned long long tcnt0 = 0;
      int it = 0;
      for (; it < PN2_FPS_POLL_LIMIT; ++it) {
        const int sv = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&sj[rp], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
        const int av = sv & (kEnd - 1);
        stop = (sv & kEnd) != 0;  // set in the same word as the final count
        if (av - applied >= GRP || (stop && av > applied)) {
          const int a1 = min(av, applied + GRP);
          const int ci = applied + lane / PPT;
          const bool valid = lane < GRP * PPT && ci < a1;
          const float4 cv = scl[valid ? ci : 0];
          // every slot below the acquired count carries the batch's tag (see hot_publish)
          if (__builtin_amdgcn_ballot_w64(
                  valid && (__float_as_uint(cv.w) & ~kPickIdxMask) != pick_tag(j))) {
            PN2_TORN_SEEN();
            continue;
          }
          if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(PRIO - 1);
          if constexpr (STAMP) tcnt0 = __builtin_amdgcn_s_memtime();
          if (cw == 0 && valid && lane % PPT == 0) {  // wave 1 stores the batch's outputs
            I[j + ci] = (int)(__float_as_uint(cv.w) & kPickIdxMask);
            if (NX) {
              NX[3 * (j + ci)] = cv.x;
              NX[3 * (j + ci) + 1] = cv.y;
              NX[3 * (j + ci) + 2] = cv.z;
            }
          }
          const float lb = box_lb(glo, ghi, cv.x, cv.y, cv.z);
          const uint64_t m = __builtin_amdgcn_ballot_w64(valid && __float_as_int(lb) < tmv);
          if constexpr (STAMP) n_pairs += __builtin_popcountll(m);
          if (m) {
#pragma unroll
            for (int s = 0; s < PPT; ++s) {
              uint64_t ms = m & cell_lanes<PPT, GRP>(s);
              if (!ms) continue;
              while (ms) {  // two centres per packed pass (a lone last one is applied twice)
                const int la = (int)__builtin_ctzll(ms);
                ms &= ms - 1;
                const int lb2 = ms ? (int)__builtin_ctzll(ms) : la;
                ms &= ms ? ms - 1 : 0;
                const float ax = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(cv.x), la));
                const float ay = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(cv.y), la));
                const float az = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(cv.z), la));
                const float bx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(cv.x), lb2));
                const float by = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(cv.y), lb2));
                const float bz = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(cv.z), lb2));
                const f2 cx = {ax, bx}, cy = {ay, by}, cz = {az, bz};
#pragma unroll
                for (int h = 0; h < PPC; ++h) {
                  const int e = s * PPC + h;
                  const float zz = ZLDS ? scz[(cw * PPT * PPC + e) * kWave + lane] : pz[e];
                  const f2 qx = {px[e], px[e]}, qy = {py[e], py[e]}, qz = {zz, zz};
                  const f2 dx = qx - cx, dy = qy - cy, dz = qz - cz;
                  const f2 d = (dx * dx + dy * dy) + dz * dz;
                  tb[e] = min(min(tb[e], __float_as_int(d.x)), __float_as_int(d.y));
                }
              }
              dirty |= 1u << s;
            }
          }
          applied = a1;
          if constexpr (PRIO > 0) __builtin_amdgcn_s_setprio(0);
          if constexpr (STAMP) {
            n_tail_grp += stop ? 1 : 0;
            const unsigned long long dt = __builtin_amdgcn_s_memtime() - tcnt0;
            n_grp += 1;
            n_grp_cyc += dt;
          }
          continue;
        }
        if (stop) break;  // av is final
        if (dirty) {  // idle: refresh one dirty cell instead of waiting
          const int s0 = __builtin_ctz(dirty);
#pragma unroll
          for (int s = 0; s < PPT; ++s) {
            if (s == s0) {
              Tm[s] = __builtin_amdgcn_readfirstlane(PN2_CELLMAX(s));
              tmv = lane % PPT == s ? Tm[s] : tmv;
            }
          }
          dirty &= dirty - 1;
          continue;
        }
        if constexpr (STAMP) ++n_poll;
      }
      if (it == PN2_FPS_POLL_LIMIT && fault && lane == 0)  // centres may be missing: report
        __hip_atomic_store(fault, PN2_FAULT_FPS_POLL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      PN2_EV(0)
      PN2_STAMP(0)
      // end of the batch: this wave's exact maximum. A dirty cell is refreshed only if its
      // stale Tmax (an upper bound) exceeds the maximum of the exact ones; the others stay
      // dirty (refreshed while waiting next round) without affecting the maximum.
      int wmax = -1;
#pragma unroll
      for (int s = 0; s < PPT; ++s)
        if (!(dirty & (1u << s))) wmax = max(wmax, Tm[s]);
#pragma unroll
      for (int s = 0; s < PPT; ++s) {
        if ((dirty & (1u << s)) && Tm[s] > wmax) {
          Tm[s] = __builtin_amdgcn_readfirstlane(PN2_CELLMAX(s));
          tmv = lane % PPT == s ? Tm[s] : tmv;
          dirty &= ~(1u << s);
          wmax = max(wmax, Tm[s]);
        }
      }
      if (lane == 0) swmax[w] = wmax;
      PN2_EV(1)
      PN2_STAMP(1)
      if (round_end(std::true_type{}, round)) break;
    }
  }
  if constexpr (KG) {  // the picks' grid, from the new_xyz rows this workgroup just wrote
    __syncthreads();
    if (char* const G = s_kgrid) {  // (thread id from the wave index and mbcnt: threadIdx.x
      __shared__ GridHdr sgh;        // kept live through the loop cost registers as well)
      block_grid_build<BLOCK>(NX, M, G, shist, sbox, swmax, &sgh, w * kWave + (int)__lane_id());
    }
  }
  if constexpr (STAMP) {
    if (lane == 0 && b < 16) {
#pragma unroll
      for (int ph = 0; ph < 8; ++ph) g_stamp[(b * 16 + w) * 8 + ph] = st_acc[ph];
      g_cull_wave[(b * 16 + w) * 4 + 0] = n_grp;
      g_cull_wave[(b * 16 + w) * 4 + 1] = n_grp_cyc;
      g_cull_wave[(b * 16 + w) * 4 + 2] = n_pairs;
      g_cull_wave[(b * 16 + w) * 4 + 3] = n_poll;
      if (w == 0) {
        g_cull_stats[b * 8 + 0] = __builtin_amdgcn_s_memtime() - clk0;
        g_cull_stats[b * 8 + 1] = n_refresh;
        g_cull_stats[b * 8 + 2] = n_stall;
        g_cull_stats[b * 8 + 4] = n_hot;
      }
      if (w == 1) {
        g_cull_stats[b * 8 + 3] = n_pairs;
        g_cull_stats[b * 8 + 7] = n_tail_grp;
      }
      if (w == 2) g_cull_stats[b * 8 + 5] = n_pairs;
    }
  }
}

template <int NW, int PPT, int NPTS, bool STAMP = false, int PRIO = 0, int HQ = 2, int PPC = 1,
          bool LEAN = false>
__global__ __launch_bounds__(64 * NW) void fps_hotcull_kernel(const float* __restrict__ xyz, int N,
                                                           int M, int32_t* __restrict__ idx,
                                                           float* __restrict__ new_xyz,
                                                           int* __restrict__ fault) {
  hotcull_body<NW, PPT, NPTS, STAMP, PRIO, HQ, PPC, LEAN>(xyz, N, M, idx, new_xyz, fault);
}

template <int NW, int PPT, int NPTS, int PRIO, int HQ>
__global__ __launch_bounds__(64 * NW) void fps_hotcull_grid_kernel(const float* __restrict__ xyz,
                                                                int N, int M,
                                                                int32_t* __restrict__ idx,
                                                                float* __restrict__ new_xyz,
                                                                int* __restrict__ fault,
                                                                char* __restrict__ kgrid) {
  hotcull_body<NW, PPT, NPTS, false, PRIO, HQ, 1, false, true>(xyz, N, M, idx, new_xyz, fault,
                                                               kgrid);
}

template <int NW, int PPT, int PRIO = 0, int HQ = 2, int NPTS = 8192, int PPC = 1,
          bool LEAN = false>
void launch_hotcull(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, int* fault,
                    hipStream_t s) {
  hipLaunchKernelGGL((fps_hotcull_kernel<NW, PPT, NPTS, false, PRIO, HQ, PPC, LEAN>), dim3(B),
                     dim3(64 * NW), 0, s, xyz, N, M, idx, nx, fault);
}

// the same launch plus the picks' grid (one point per lane per cell only; kgrid non-null,
// nx non-null, M <= 4096: checked by the caller)
template <int NW, int PPT, int PRIO = 0, int HQ = 2, int NPTS = 8192>
void launch_hotcull_grid(const float* xyz, int B, int N, int M, int32_t* idx, float* nx,
                         int* fault, hipStream_t s, char* kgrid) {
  hipLaunchKernelGGL((fps_hotcull_grid_kernel<NW, PPT, NPTS, PRIO, HQ>), dim3(B), dim3(64 * NW),
                     0, s, xyz, N, M, idx, nx, fault, kgrid);
}

}  // namespace
}  // namespace pn2
