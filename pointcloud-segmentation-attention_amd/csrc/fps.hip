// Farthest-point sampling + gather_point for gfx950.
//
// Replaces FarthestPointSampleGpuOp / farthestpointsamplingKernel
// (pointnet2_tensorflow/tf_ops/sampling/tf_sampling.cpp:94-123, tf_sampling_g.cu:105-170) and
// GatherPoint(+Grad) (tf_sampling.cpp:125-178, tf_sampling_g.cu:172-192).
//
// Design (MI355X-first, not a translation of the reference's <<<32,512>>> kernel): one
// workgroup per cloud with the cloud's xyz and running min-distance in VGPRs, a register scan
// per iteration and a ballot/DPP argmax whose lane order IS the reference's tie order — see
// fps_v9_kernel in fps_kernels.h. gather_point is fused (thread 0 writes new_xyz,
// pointnet_util.py:34). Clouds beyond kMaxRegPoints keep the running min in a caller-provided
// workspace (fps_ws_kernel). The measured variants (a lab library of rounds 1-2, since removed
// from the tree) and their numbers are in DESIGN.md §3.1 and profiles/r1/.
#include <mutex>

#include "fps_kernels.h"
#ifndef PN2_SA1_PPT
#define PN2_SA1_PPT 9  // cell slots per cold wave of the SA1 sampler (A/B builds: -DPN2_SA1_PPT)
#endif
#include "fps_cull.h"

// Code placement of the SA1 (256 x 32) sampler's iteration loop. The loop runs ~6 % slower
// when it starts at an address = 0 mod 8 than at 4 mod 8 (a round-1 padding sweep, since
// removed; its log: profiles/r1/pad_fps.log). tools/place_sa1_loop.py compiles this file, reads where the
// loop landed and writes build/sa1_pad.h: the number of s_nop placed before the loop (run
// once per launch) that moves it to the measured best offset.
#ifndef PN2_SA1_PAD
#if __has_include("build/sa1_pad.h")
#include "build/sa1_pad.h"
#endif
#endif
#ifndef PN2_SA1_PAD
#define PN2_SA1_PAD -1
#endif

namespace pn2 {
namespace {

// Large clouds (N beyond the register path): running min-distance in a global workspace,
// 1024 threads, point k on thread k mod 1024 (ascending slot order = reference tie order).
__global__ __launch_bounds__(1024) void fps_ws_kernel(const float* __restrict__ xyz, int N, int M,
                                                      float* __restrict__ ws,
                                                      int32_t* __restrict__ idx,
                                                      float* __restrict__ new_xyz) {
  constexpr int BLOCK = 1024, NW = BLOCK / kWave;
  __shared__ uint64_t red[2][16];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const float* __restrict__ P = xyz + (size_t)b * N * 3;
  float* __restrict__ T = ws + (size_t)b * N;
  int32_t* __restrict__ I = idx + (size_t)b * M;
  float* __restrict__ NX = new_xyz ? new_xyz + (size_t)b * M * 3 : nullptr;
  for (int k = t; k < N; k += BLOCK) T[k] = kInitTemp;
  float cx = P[0], cy = P[1], cz = P[2];
  if (t == 0) {
    I[0] = 0;
    if (NX) { NX[0] = cx; NX[1] = cy; NX[2] = cz; }
  }
  for (int j = 1; j < M; ++j) {
    float bd = -1.0f;
    int bk = 0;
    for (int k = t; k < N; k += BLOCK) {
      const float d = sqdist(P[3 * k], P[3 * k + 1], P[3 * k + 2], cx, cy, cz);
      const float v = fminf(d, T[k]);
      T[k] = v;
      if (v > bd) { bd = v; bk = k; }
    }
    uint64_t key = bd < 0.0f ? 0ull : pack64(tie_low(bk), __float_as_uint(bd));
    key = wave_max_u64(key);
    if (lane == 0) red[j & 1][w] = key;
    __syncthreads();
    key = row16_max_u64(lane < NW ? red[j & 1][lane] : 0ull);
    const int old = tie_decode(uniform_u32((uint32_t)key));
    cx = P[3 * old + 0]; cy = P[3 * old + 1]; cz = P[3 * old + 2];
    if (t == 0) {
      I[j] = old;
      if (NX) { NX[3 * j + 0] = cx; NX[3 * j + 1] = cy; NX[3 * j + 2] = cz; }
    }
  }
}

// N == 0: the reference still emits idx 0 everywhere (tf_sampling_g.cu:125-167 with no point
// scanned leaves besti = 0); new_xyz has nothing to gather and is zero-filled.
__global__ void fps_empty_kernel(int total, int32_t* idx, float* new_xyz) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < total) {
    idx[i] = 0;
    if (new_xyz) { new_xyz[3 * i] = 0.f; new_xyz[3 * i + 1] = 0.f; new_xyz[3 * i + 2] = 0.f; }
  }
}

__global__ void gather_point_kernel(const float* __restrict__ inp, const int32_t* __restrict__ idx,
                                    int N, int M, int total, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // i = b*M + j
  if (i >= total) return;
  const int b = i / M;
  const int a = idx[i];
  const float* src = inp + ((size_t)b * N + a) * 3;
  out[3 * (size_t)i + 0] = src[0];
  out[3 * (size_t)i + 1] = src[1];
  out[3 * (size_t)i + 2] = src[2];
}

__global__ void gather_point_grad_kernel(const float* __restrict__ out_g,
                                         const int32_t* __restrict__ idx, int N, int M,
                                         int total, float* __restrict__ inp_g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int b = i / M;
  const int a = idx[i];
  float* dst = inp_g + ((size_t)b * N + a) * 3;
  atomicAdd(dst + 0, out_g[3 * (size_t)i + 0]);
  atomicAdd(dst + 1, out_g[3 * (size_t)i + 1]);
  atomicAdd(dst + 2, out_g[3 * (size_t)i + 2]);
}

constexpr int kMaxRegPoints = 1024 * 16;

constexpr int kCullGridMax = 4096;  // picks whose grid the culled sampler builds itself

// ---- device fault word ------------------------------------------------------------------
// A kernel that finds a broken invariant (the culled sampler's cold waves waiting past their
// poll bound, fps_cull.h) stores a PN2_FAULT_* code into one host-pinned, device-mapped word.
// The host reads it without synchronising: the next pn2_fps* call reports it as PN2_EFAULT
// (and clears it), and pn2_fault_status() returns it. Allocated at the first sampler launch
// (never on a machine without a GPU); nullptr if that fails (then nothing is reported).
std::once_flag g_fault_once;
int* g_fault_host = nullptr;
int* g_fault_dev = nullptr;

int* fault_word_dev() {
  std::call_once(g_fault_once, [] {
    void* h = nullptr;
    if (hipHostMalloc(&h, sizeof(int), hipHostMallocMapped | hipHostMallocPortable) != hipSuccess)
      return;
    *(volatile int*)h = 0;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      return;
    }
    g_fault_host = (int*)h;
    g_fault_dev = (int*)d;
  });
  return g_fault_dev;
}

// a fault stored by an earlier launch (visible once that launch's stream has synchronised)
int take_fault() {
  if (!g_fault_host) return 0;
  return __atomic_exchange_n(g_fault_host, 0, __ATOMIC_ACQ_REL);
}

// ---- sampler chain: SA1..SAk's samplers of one cloud, stage 2.. in ONE workgroup -----------
// The SSG stack samples 8192 -> 1024 -> 256 -> 64 -> 16, each stage from the previous stage's
// output. pn2_fps_chain runs a big first stage (N > kChainNext) as the ordinary sampler
// kernel, then every remaining stage of a cloud back to back in one workgroup (no kernel
// boundary, no event between stages): the tail kernel's first stage reads its points from
// HBM (with an LDS copy for the centre lookups), every later stage reads them from the LDS
// array the previous stage filled as it went. Each stage writes its idx and new_xyz to global
// memory exactly as pn2_fps_gather does, with the same per-size configuration as fps_impl
// (BLOCK 256, or wave 0 alone). (Fusing the 8192-point stage too was measured slower: the
// fused kernel's SA1 loop ran ~4% behind the same loop in its own kernel, more than the
// launch it saved -- profiles/r1/chain_split.log.)
constexpr int kChainMax = 4;
constexpr int kChainBlock = 256;  // 128 and 512 measured slower (profiles/r4/ab)
constexpr int kChainNext = 1024;  // points per fused stage (LDS: input copy + 2 hand-over arrays)

struct FpsChain {
  int stages;
  int verdicts;  // > 0: fps_prefix_check_kernel's verdict words at the head of each idx[0] row
  int* fault;  // the device fault word (fault_word_dev)
  int n[kChainMax], m[kChainMax];
  int32_t* idx[kChainMax];
  float* nx[kChainMax];
};

// ---- hot-set schedule of one fused chain stage (N <= kChainNext, the whole workgroup) -----
// The culled sampler's certificate (fps_cull.h, HOT SET) without its cells, with the roles
// split by wave. Waves 1-3 (the cold waves) hold the cloud's points, PPT per thread, in the
// reference's tie order (k mod 512, k div 512) (tf_sampling_g.cu:146-163); wave 0 (the hot
// wave, alone on its SIMD) holds no points. A round:
//   1. the cold waves' running mins are exact; tau = ref * frac chooses the hot set (ref: the
//      last round's tau, an upper bound of every value, else the block max; counted and
//      staged for two fractions at once, the lower one taken when at most K = 64 points lie
//      above it), which the cold waves stage, in tie order;
//   2. wave 0 takes one hot point per lane and picks from them alone while its best value is
//      > tau: every other point is <= tau and running mins only decrease, so that best IS the
//      reference's next centre. Per pick: a wave max, one ballot, the winning lane's four
//      4-byte LDS writes of the centre and the count, three readlanes -- no barrier, no LDS
//      read;
//   3. meanwhile the cold waves apply every published centre to their points (they poll the
//      count), so their mins are exact again when the round ends.
// The first picks of a stage are exact block argmaxes (the first rounds certify few picks).
// A cloud of at most 64 points is all hot (wave 0 alone, tau = -1). If no fraction fits (ties
// crowd the top) or the max is negative, one exact block argmax (fps_v9's rule: the lowest
// position holding the max, position 0 when every value is below 0) picks the centre. The
// outputs (idx, new_xyz, the next stage's LDS copy) are written from the pick list after the
// stage (bulk, coalesced). Same picks as fps_v9_body bit for bit: the same fp32 distance, the same int-bit
// running mins and tie order.
constexpr int kHotFracs = 12;  // kCullFrac (fps_cull.h): the thresholds
constexpr int kHotK = kWave;  // hot points: one per lane of wave 0
constexpr int kHotCold = kChainBlock / kWave - 1;  // cold waves
// a cold wave's polls per round: at PN2_FPS_POLL_LIMIT (fps_cull.h) it stores
// PN2_FAULT_FPS_POLL and goes on waiting (the picks stay exact: the polltest build's 4 polls
// report the fault without breaking the stage); at kHotPollHard (~2 s, a hung hot wave) it gives
// up, and the stage's picks are wrong -- reported by the same fault
constexpr int kHotPollHard = 1 << 24;
#ifndef PN2_HOT_EXACT
#define PN2_HOT_EXACT 16
#endif
#ifndef PN2_HOT_EXACT2
#define PN2_HOT_EXACT2 6
#endif
constexpr int kHotExact = PN2_HOT_EXACT;  // picks of the 1,024-point stage made one at a time
constexpr int kHotExact2 = PN2_HOT_EXACT2;  // ... of the smaller ones
struct HotLds {
  float4 pc[kChainNext];          // picks by number: x, y, z, bits(index)
  float4 hk[2][kHotCold][kHotK];  // hot staging for two thresholds, per cold wave: x, y, z, bits(index)
  int hv[2][kHotCold][kHotK];     // hot staging: running min (int bits)
  int wmax[2][kHotCold];          // per cold wave: its max (double-buffered by try)
  int cnt[2][2][kHotCold];        // [try parity][threshold][cold wave]: points above it
  uint2 red[2][kHotCold];         // exact argmax by pick parity: (max + 1, index) per cold wave
  int pub[2];                     // by round parity: picks published | kHotEnd when the round ends
};
constexpr int kHotEnd = 1 << 30;

// DIAGNOSTIC build flag (tools/stamp_chain.py): per round of cloud 0's stages, s_memtime at
// the round's start (after the block max), when the hot set fits, the hot wave's end and the
// first cold wave's end, plus the picks made and the tries; read back with pn2_hot_stamps()
#ifndef PN2_HOT_STAMP
#define PN2_HOT_STAMP 0
#endif
#if PN2_HOT_STAMP
__device__ unsigned long long g_hot_ev[3 * 64 * 8];
#define PN2_HOTEV(R, F, V)                                                            \
  if (blockIdx.x == 0 && lane == 0 && (R) < 64)                                      \
    g_hot_ev[((N > 512 ? 0 : (N > 64 ? 1 : 2)) * 64 + (R)) * 8 + (F)] = (unsigned long long)(V);
#else
#define PN2_HOTEV(R, F, V)
#endif

// tie position p -> point index: p = k below 512 points, else p = 2 (k mod 512) + k div 512
PN2_DEV int hot_point(int p, bool wide) { return wide ? (p >> 1) + ((p & 1) << 9) : p; }

using hf4 = float __attribute__((ext_vector_type(4)));

// wave 0's picks from its hot entries (e = x, y, z, bits(point index), value hv; empty lanes
// hold INT_MIN) while the best is > tau and j < M; each pick is published as it is made (its
// slot with the batch's tag pick_tag(tag0 + j), then -- released -- the count of the picks before it;
// fps_cull.h hot_publish; a cold wave acquires the count, then reads the slots). At most lim
// picks (a picked entry drops to 0 <= tau, so a round cannot outrun its hot set -- except
// through NaN distances, which the bound covers; the all-hot path, tau = -1, needs it to stop
// at M). Returns the picks made so far.
PN2_DEV int hot_picks(hf4 e, int hv, int tau, int j, int lim, int* pub, HotLds& S, int tag0) {
  j = __builtin_amdgcn_readfirstlane(j);  // (a scalar loop count: no exec-mask bookkeeping)
  // publishing addresses and the count in VGPRs, advanced by one VALU add per pick
  int va_c, va_n, vcnt;
  asm volatile("v_mov_b32 %0, %1" : "=v"(va_c)
               : "s"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)&S.pc[j]));
  asm volatile("v_mov_b32 %0, %1" : "=v"(va_n)
               : "s"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) int*)pub));
  asm volatile("v_mov_b32 %0, %1" : "=v"(vcnt) : "s"(j));
  const int lw = __float_as_int(e.w) | (int)pick_tag(tag0 + j);  // the slots' w
  int n = 0;
  // (one exit, at the bottom: the loop carries no break flags)
  int km = __builtin_amdgcn_readlane(wave_max_i32_l63(hv), kWave - 1);
  while (km > tau) {  // else the certificate fails: the round ends
    const int L = (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(hv == km));
    float cx, cy, cz;
    hot_publish(L, va_c, va_n, vcnt, e.x, e.y, e.z, lw, cx, cy, cz);
    __builtin_amdgcn_sched_barrier(0);
    ++n;
    hv = min(hv, __float_as_int(sqdist(e.x, e.y, e.z, cx, cy, cz)));
    va_c += 16;
    vcnt += 1;
    km = __builtin_amdgcn_readlane(wave_max_i32_l63(hv), kWave - 1);
    km = n >= lim ? tau : km;
  }
  return j + n;
}

// tag0: the picks of the launch's earlier stages (the slots' tags are pick_tag(tag0 + pick))
template <int PPT>
PN2_DEV void fps_hot_body(const float* CXYZ, int N, int M, int32_t* I, float* NX, float* SNEXT,
                          HotLds& S, int tag0, int* fault) {
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const bool wide = N > 512;
  const float c0x = CXYZ[0], c0y = CXYZ[1], c0z = CXYZ[2];
  if (t == 0) S.pc[0] = make_float4(c0x, c0y, c0z, __uint_as_float(pick_tag(tag0)));
  int j = 1;  // picks made (uniform)
  PN2_HOTEV(63, 0, __builtin_amdgcn_s_memtime())
  if (N <= kHotK) {
    // all hot: wave 0 alone, point k on lane k
    if (w == 0) {
      const bool in = lane < N;
      const float hx = in ? CXYZ[3 * lane + 0] : 0.0f, hy = in ? CXYZ[3 * lane + 1] : 0.0f,
                  hz = in ? CXYZ[3 * lane + 2] : 0.0f;
      int hv = in ? min(__float_as_int(kInitTemp), __float_as_int(sqdist(hx, hy, hz, c0x, c0y, c0z)))
                  : (-2147483647 - 1);
      while (j < M) {
        j = hot_picks(hf4{hx, hy, hz, __int_as_float(lane)}, hv, -1, j, M - j, &S.pub[0], S, tag0);
        if (j >= M) break;
        // every value < 0 (padding / negative NaN bits): fps_v9 picks point 0; refresh the
        // lanes' values from the centres published since (cheap: this path is degenerate)
        hv = in ? __float_as_int(kInitTemp) : (-2147483647 - 1);
        if (lane == 0) S.pc[j] = make_float4(c0x, c0y, c0z, __uint_as_float(pick_tag(tag0 + j)));
        ++j;
        for (int p = 0; p < j && in; ++p) {
          const float4 c = S.pc[p];
          hv = min(hv, __float_as_int(sqdist(hx, hy, hz, c.x, c.y, c.z)));
        }
      }
    }
  } else {
    // cold waves: tie positions p = u * PPT + s, u = t - 64
    const int u = t - kWave;
    using f2 = float __attribute__((ext_vector_type(2)));
    constexpr bool PK = PPT % 2 == 0;
    constexpr int NP = PK ? PPT / 2 : 1;
    float px[PPT], py[PPT], pz[PPT];
    int tb[PPT], pk[PPT];
    f2 vx[NP], vy[NP], vz[NP];
    if (w > 0) {
#pragma unroll
      for (int s = 0; s < PPT; ++s) {
        const int pp = u * PPT + s;
        const int k = hot_point(pp, wide);
        const bool in = pp < kChainNext && k < N;
        const int kk = in ? k : 0;
        pk[s] = k;
        px[s] = in ? CXYZ[3 * kk + 0] : 0.0f;
        py[s] = in ? CXYZ[3 * kk + 1] : 0.0f;
        pz[s] = in ? CXYZ[3 * kk + 2] : 0.0f;
        tb[s] = in ? __float_as_int(kInitTemp) : -1;  // padding never wins
        if constexpr (PK) { vx[s / 2][s % 2] = px[s]; vy[s / 2][s % 2] = py[s]; vz[s / 2][s % 2] = pz[s]; }
      }
    }
    auto apply = [&](float cx, float cy, float cz) {
      if constexpr (PK) {
        const f2 c2x = {cx, cx}, c2y = {cy, cy}, c2z = {cz, cz};
#pragma unroll
        for (int h = 0; h < NP; ++h) {
          const f2 dx = vx[h] - c2x, dy = vy[h] - c2y, dz = vz[h] - c2z;
          const f2 d = (dx * dx + dy * dy) + dz * dz;
          tb[2 * h] = min(tb[2 * h], __float_as_int(d.x));
          tb[2 * h + 1] = min(tb[2 * h + 1], __float_as_int(d.y));
        }
      } else {
#pragma unroll
        for (int s = 0; s < PPT; ++s)
          tb[s] = min(tb[s], __float_as_int(sqdist(px[s], py[s], pz[s], cx, cy, cz)));
      }
    };
    if (w > 0) apply(c0x, c0y, c0z);
    int r = 1;       // cold waves: picks applied
    int fi = 0;      // threshold fraction (kept from round to round)
    int round = 0;
    int tries = 0;   // parity of the count buffers
    // one exact block argmax over the cold waves (fps_v9's order), every thread: pick j
    auto exact_pick = [&]() {
      if (w > 0) {
        int bd = -1, bs = 0;
#pragma unroll
        for (int s = 0; s < PPT; ++s) {
          bs = tb[s] > bd ? s : bs;
          bd = max(bd, tb[s]);
        }
        const uint32_t hi = (uint32_t)(bd + 1);
        const uint32_t km = wave_max_u32(hi);
        const int L = (int)__builtin_amdgcn_readfirstlane(
            (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(hi == km)));
        const int sq = __builtin_amdgcn_readlane(bs, L);
        if (lane == 0)
          S.red[j & 1][w - 1] = make_uint2(km, (uint32_t)hot_point((u - lane + L) * PPT + sq, wide));
      }
      __syncthreads();
      uint2 best = S.red[j & 1][0];
#pragma unroll
      for (int i = 1; i < kHotCold; ++i) {
        const uint2 q = S.red[j & 1][i];
        best = q.x > best.x ? q : best;  // ties: the lowest wave
      }
      const int old = __builtin_amdgcn_readfirstlane((int)best.y);
      const float cx = CXYZ[3 * old + 0], cy = CXYZ[3 * old + 1], cz = CXYZ[3 * old + 2];
      if (t == 0) S.pc[j] = make_float4(cx, cy, cz, __uint_as_float((uint32_t)old | pick_tag(tag0 + j)));
      if (w > 0) apply(cx, cy, cz);
      ++j;
      r = j;
    };
    // the first picks one at a time: the first rounds certify only 1-4 picks each
    // (tools/stamp_chain.py), less than a round costs
    const int e0 = min(M, PPT >= 6 ? kHotExact : kHotExact2);
    while (j < e0) exact_pick();
    PN2_HOTEV(63, 2, __builtin_amdgcn_s_memtime())
    // the thresholds' fractions, lane f holding fraction f (read with one readlane per round)
    const float fracv = kCullFrac[lane < kHotFracs ? lane : kHotFracs - 1];
    int tref = -1;  // the last round's tau: every value is <= it now (-1: none)
    while (j < M) {
      // this round's publishing word reset (its last readers, two rounds ago, are past the
      // barriers since)
      if (t == 0) S.pub[(round + 1) & 1] = j;
      // 1. the reference value for the thresholds: the last round's tau (an upper bound of
      // the block max, no barrier needed), else the block max itself
      int ref = tref;
      bool exact_ref = ref < 0;
      if (exact_ref) {
        if (w > 0) {
          int lm = tb[0];
#pragma unroll
          for (int s = 1; s < PPT; ++s) lm = max(lm, tb[s]);
          lm = wave_max_i32(lm);
          if (lane == 0) S.wmax[tries & 1][w - 1] = lm;
        }
        __syncthreads();
        ref = S.wmax[tries & 1][0];
#pragma unroll
        for (int i = 1; i < kHotCold; ++i) ref = max(ref, S.wmax[tries & 1][i]);
        ref = __builtin_amdgcn_readfirstlane(ref);
      }
      PN2_HOTEV(round, 0, __builtin_amdgcn_s_memtime())
      const int tries0 = tries;
      (void)tries0;
      // 2. the hot set: counted and staged for two thresholds at once (fractions fi, fi + 1
      // of the reference), the lower one taken when it fits; both too large: two fractions
      // up; a bound as the reference and nothing fits: again with the block max (each pass
      // also publishes the cold waves' maxima)
      int tau = 0, sel = 0, c[kHotCold] = {0, 0, 0};
      bool fits = false;
      while (ref >= 0) {
        const int fa = fi, fb = min(fi + 1, kHotFracs - 1);
        const float rf = __int_as_float(ref);
        const int ta = __builtin_amdgcn_readfirstlane(
            __float_as_int(rf * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fracv), fa))));
        const int tbb = __builtin_amdgcn_readfirstlane(
            __float_as_int(rf * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fracv), fb))));
        if (w > 0) {
          int pa = 0, pb = 0, ca = 0, cb = 0, lm = tb[0];
#pragma unroll
          for (int s = 0; s < PPT; ++s) {
            const uint64_t ba = __builtin_amdgcn_ballot_w64(tb[s] > ta);
            const uint64_t bb = __builtin_amdgcn_ballot_w64(tb[s] > tbb);
            pa += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(ba >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ba, 0u));
            pb += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u));
            ca += __builtin_popcountll(ba);
            cb += __builtin_popcountll(bb);
            lm = max(lm, tb[s]);
          }
#pragma unroll
          for (int s = 0; s < PPT; ++s) {
            const float4 en = make_float4(px[s], py[s], pz[s], __int_as_float(pk[s]));
            if (tb[s] > ta) {
              if (pa < kHotK) { S.hk[0][w - 1][pa] = en; S.hv[0][w - 1][pa] = tb[s]; }
              ++pa;
            }
            if (tb[s] > tbb) {
              if (pb < kHotK) { S.hk[1][w - 1][pb] = en; S.hv[1][w - 1][pb] = tb[s]; }
              ++pb;
            }
          }
          if (!exact_ref) lm = wave_max_i32(lm);
          if (lane == 0) {
            S.cnt[tries & 1][0][w - 1] = ca;
            S.cnt[tries & 1][1][w - 1] = cb;
            if (!exact_ref) S.wmax[tries & 1][w - 1] = lm;
          }
        }
        __syncthreads();
        int ca[kHotCold], cb[kHotCold], tota = 0, totb = 0;
#pragma unroll
        for (int i = 0; i < kHotCold; ++i) {
          ca[i] = __builtin_amdgcn_readfirstlane(S.cnt[tries & 1][0][i]);
          cb[i] = __builtin_amdgcn_readfirstlane(S.cnt[tries & 1][1][i]);
          tota += ca[i];
          totb += cb[i];
        }
        const int tr = tries++;
        if (tota >= 1 && tota <= kHotK) {
          fits = true;
          tau = ta;
          sel = 0;
#pragma unroll
          for (int i = 0; i < kHotCold; ++i) c[i] = ca[i];
          if (2 * tota < kHotK && fi > 0) --fi;  // a small set: a lower fraction next round
          break;
        }
        if (totb >= 1 && totb <= kHotK) {
          fits = true;
          tau = tbb;
          sel = 1;
#pragma unroll
          for (int i = 0; i < kHotCold; ++i) c[i] = cb[i];
          fi = fb;
          break;
        }
        if (!exact_ref) {  // the bound did not serve: the block max, same fractions
          int m = S.wmax[tr & 1][0];
#pragma unroll
          for (int i = 1; i < kHotCold; ++i) m = max(m, S.wmax[tr & 1][i]);
          ref = __builtin_amdgcn_readfirstlane(m);
          exact_ref = true;
          if (tota > kHotK) fi = min(fb + 1, kHotFracs - 1);
          continue;
        }
        if (totb == 0 || fb == kHotFracs - 1) break;  // (no higher fraction fits either)
        fi = min(fb + 1, kHotFracs - 1);
      }
      tref = fits ? tau : -1;
      if (!fits) {  // ties crowd the top, or only negative values are left
        exact_pick();
        continue;
      }
      PN2_HOTEV(round, 1, __builtin_amdgcn_s_memtime())
      PN2_HOTEV(round, 4, tries - tries0)
      ++round;
      int* const pub = &S.pub[round & 1];
      if (w == 0) {
        // 2. the picks: lane l takes hot entry l (the cold waves' stagings in wave order)
        const int i1 = lane - c[0], i2 = i1 - c[1];
        const int src = lane < c[0] ? 0 : (i1 < c[1] ? 1 : 2);
        const int off = src == 0 ? lane : (src == 1 ? i1 : i2);
        const bool in = lane < c[0] + c[1] + c[2];
        const hf4 e = *reinterpret_cast<const hf4*>(&S.hk[sel][src][in ? off : 0]);
        const int hv = in ? S.hv[sel][src][off] : (-2147483647 - 1);
        j = hot_picks(e, hv, tau, j, min(M - j, kHotK), pub, S, tag0);
        PN2_HOTEV(round - 1, 2, __builtin_amdgcn_s_memtime())
        PN2_HOTEV(round - 1, 3, j)
        if (lane == 0) publish_end(pub, j | kHotEnd);
      } else {
        // 3. the cold waves apply the centres as wave 0 publishes them, up to 64 per LDS read
        for (int it = 0; it < kHotPollHard; ++it) {
          if (it == PN2_FPS_POLL_LIMIT && fault && lane == 0)
            __hip_atomic_store(fault, PN2_FAULT_FPS_POLL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          const int sv = __builtin_amdgcn_readfirstlane(
              __hip_atomic_load(pub, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
          const int av = sv & (kHotEnd - 1);
          if (av > r) {
            const int n = min(av - r, kWave);
            const int p = r + min(lane, n - 1);
            const float4 cv = S.pc[p];
            // every slot below the acquired count carries the batch's tag (fps_cull.h
            // hot_publish; j: this round's first pick)
            if (__builtin_amdgcn_ballot_w64((__float_as_uint(cv.w) & ~kPickIdxMask) !=
                                            pick_tag(tag0 + j))) {
              PN2_TORN_SEEN();
              continue;
            }
            for (int i = 0; i < n; ++i) {
              const float cx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(cv.x), i));
              const float cy = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(cv.y), i));
              const float cz = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(cv.z), i));
              apply(cx, cy, cz);
            }
            r += n;
            continue;
          }
          if (sv & kHotEnd) break;  // av is final and applied
        }
        if (w == 1) { PN2_HOTEV(round - 1, 5, __builtin_amdgcn_s_memtime()) }
        j = r;
      }
    }
  }
  __syncthreads();
  PN2_HOTEV(63, 1, __builtin_amdgcn_s_memtime())
  // the outputs from the pick list
  for (int i = t; i < M; i += kChainBlock) {
    const float4 c = S.pc[i];
    I[i] = (int)(__float_as_uint(c.w) & kPickIdxMask);
    if (NX) { NX[3 * i + 0] = c.x; NX[3 * i + 1] = c.y; NX[3 * i + 2] = c.z; }
    if (SNEXT) { SNEXT[3 * i + 0] = c.x; SNEXT[3 * i + 1] = c.y; SNEXT[3 * i + 2] = c.z; }
  }
}

// one stage (N <= kChainNext) for one cloud, every thread of the workgroup: the hot-set
// schedule (cold points per thread: 2 up to 384 points, 3 up to 512, 6 up to 1,024).
// (Measured and not kept, profiles/r5/chain: the 1,024-point stage on ONE wave, 16 points a
// lane and no barrier -- 126.5 -> 129 us for the chain, 140 us with each lane's candidate
// coordinates read speculatively; a single wave issues the pick's ~110 dependent VALU ops at
// ~8 cycles each, which costs what the 4-wave form's barrier and cross-wave step cost.)
#ifndef PN2_CHAIN_HOT
#define PN2_CHAIN_HOT 1
#endif
PN2_DEV void chain_stage(const float* P, int N, int M, const float* CXYZ, int32_t* I, float* NX,
                         float* SNEXT, uint2 (*red)[8], HotLds& hot, int tag0, int* fault) {
#if PN2_CHAIN_HOT
  // (the pick list holds kChainNext: a larger last stage takes the v9 bodies below)
  if (M <= kChainNext) {
    if (N <= 384) fps_hot_body<2>(CXYZ, N, M, I, NX, SNEXT, hot, tag0, fault);
    else if (N <= 512) fps_hot_body<3>(CXYZ, N, M, I, NX, SNEXT, hot, tag0, fault);
    else fps_hot_body<6>(CXYZ, N, M, I, NX, SNEXT, hot, tag0, fault);
    return;
  }
#else
  (void)hot;
  (void)tag0;
  (void)fault;
#endif
  const bool w0 = threadIdx.x < kWave;
  if (N <= 64) { if (w0) fps_v9_body<64, 1, 1>(P, N, M, CXYZ, I, NX, SNEXT, red); }
  else if (N <= 128) { if (w0) fps_v9_body<64, 2, 2>(P, N, M, CXYZ, I, NX, SNEXT, red); }
  else if (N <= 256) { if (w0) fps_v9_body<64, 4, 4, false, true>(P, N, M, CXYZ, I, NX, SNEXT, red); }
  else if (N <= 512) { if (w0) fps_v9_body<64, 8, 4, false, true>(P, N, M, CXYZ, I, NX, SNEXT, red); }
  else fps_v9_body<256, 4, 2, false, true>(P, N, M, CXYZ, I, NX, SNEXT, red);
}

// ---- a chain over an earlier sampler's output: its stages are prefixes ---------------------
// If P[0..n) is itself a farthest-point sampling in pick order (the fused tail's input is the
// SA1 sampler's new_xyz), FPS(P, m) picks 0, 1, ..., m - 1: pick j of P's own sampling was the
// farthest point of a superset of P from picks 0 .. j - 1, and it lies in P, so it is also the
// farthest point of P -- unless another point ties with it, where the sampler's tie order
// (tf_sampling_g.cu:131-165: strided scan, left-biased tree) decides. So the check demands a
// unique maximum at every step: with the running mins of the reference's sampler,
// temp_j(s) = min(1e38, min_{i<j} d(P_s, P_i)) (the samplers' uncontracted fp32 distance) and
// M_j = temp_j(j), the value pick j is chosen with, every s != j has temp_j(s) < M_j, for
// j = 1 .. m - 1. Then FPS(P, m) = [0, m), and every later stage of the chain (m' <= m picks of
// that prefix) is a prefix as well, by the same argument on the subset. Non-finite
// coordinates, M_j <= 0 (duplicates) and every tie fail the check; the stages then run as
// samplers. A quick test of pick 1 first (the unique farthest point from pick 0), so an
// arbitrary input (a chain whose first stage samples a raw cloud) is rejected in one pass.
//
// fps_prefix_check_kernel: one workgroup per (slice of kPrefixPts points, cloud); each checks
// its points against every M_j (computed by every workgroup: no exchange) and stores its
// verdict, 0 (holds) or -1, in word `slice` of the cloud's stage-0 idx row, which the chain
// kernel reads before it writes that row. The work is ~n x m independent distance updates per
// cloud, spread over the chip instead of the chain's one workgroup per cloud.
constexpr int kPrefixPts = 256;
using pf2 = float __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(kPrefixPts) void fps_prefix_check_kernel(
    const float* __restrict__ xyz, int n, int m, int32_t* __restrict__ verdict) {
  // picks 0 .. m - 1 as x, y, z arrays (a pair of consecutive picks from an even index is one
  // 8-byte read); smm[j + 1] = M_j (a pair M_j, M_j+1 from an odd j likewise)
  __shared__ __attribute__((aligned(16))) float sx[kChainNext + 2], sy[kChainNext + 2],
      sz[kChainNext + 2], smm[kChainNext + 4];
  const int b = blockIdx.y, slice = blockIdx.x, t = threadIdx.x;
  const float* __restrict__ P = xyz + (size_t)b * n * 3;
  for (int e = t; e < m; e += kPrefixPts) {
    sx[e] = P[3 * e];
    sy[e] = P[3 * e + 1];
    sz[e] = P[3 * e + 2];
  }
  if (t < 2) sx[m + t] = sy[m + t] = sz[m + t] = 0.0f;  // (pair tails)
  __syncthreads();
  const int s = slice * kPrefixPts + t;
  const bool in = s < n;
  // a point past n stands in as a copy of pick 0: its running min is 0 from step 1 on
  const float px = in ? P[3 * s] : sx[0], py = in ? P[3 * s + 1] : sy[0],
              pz = in ? P[3 * s + 2] : sz[0];
  bool bad = !(__builtin_isfinite(px) && __builtin_isfinite(py) && __builtin_isfinite(pz));
  {
    const float m1 = fminf(1e38f, sqdist(sx[1], sy[1], sz[1], sx[0], sy[0], sz[0]));
    bad = bad || !(m1 > 0.0f) ||
          (s != 1 && !(fminf(1e38f, sqdist(px, py, pz, sx[0], sy[0], sz[0])) < m1));
  }
  if (__syncthreads_or(bad)) {
    if (t == 0) verdict[(size_t)b * m + slice] = -1;
    return;
  }
  // M_j = temp_j(j), two picks' distances per packed step
  for (int j = t; j < m; j += kPrefixPts) {
    const pf2 qx = {sx[j], sx[j]}, qy = {sy[j], sy[j]}, qz = {sz[j], sz[j]};
    float v = 1e38f;
    int i = 0;
#pragma unroll 4
    for (; i + 1 < j; i += 2) {
      const pf2 cx = *reinterpret_cast<const pf2*>(&sx[i]),
                cy = *reinterpret_cast<const pf2*>(&sy[i]),
                cz = *reinterpret_cast<const pf2*>(&sz[i]);
      const pf2 dx = qx - cx, dy = qy - cy, dz = qz - cz;
      const pf2 d = (dx * dx + dy * dy) + dz * dz;
      v = fminf(fminf(v, d.x), d.y);
    }
    if (i < j) v = fminf(v, sqdist(qx.x, qy.x, qz.x, sx[i], sy[i], sz[i]));
    smm[j + 1] = v;
    bad = bad || (j > 0 && !(v > 0.0f));
  }
  if (t == 0) smm[m + 1] = 0.0f;  // (pair tail)
  if (__syncthreads_or(bad)) {
    if (t == 0) verdict[(size_t)b * m + slice] = -1;
    return;
  }
  // every point's running min against each M_j; the one hit allowed is s's own step (j = s,
  // where temp_s(s) is M_s bit for bit: the same distances, and min is exact)
  {
    const pf2 qx = {px, px}, qy = {py, py}, qz = {pz, pz};
    float v = 1e38f;
    int hits = in && s >= 1 && s < m ? -1 : 0;
    int j = 1;
#pragma unroll 4
    for (; j + 1 < m; j += 2) {  // steps j and j + 1: picks j - 1 and j
      const pf2 cx = *reinterpret_cast<const pf2*>(&sx[j - 1]),
                cy = *reinterpret_cast<const pf2*>(&sy[j - 1]),
                cz = *reinterpret_cast<const pf2*>(&sz[j - 1]),
                mm = *reinterpret_cast<const pf2*>(&smm[j + 1]);
      const pf2 dx = qx - cx, dy = qy - cy, dz = qz - cz;
      const pf2 d = (dx * dx + dy * dy) + dz * dz;
      v = fminf(v, d.x);
      hits += v >= mm.x ? 1 : 0;
      v = fminf(v, d.y);
      hits += v >= mm.y ? 1 : 0;
    }
    if (j < m) {
      v = fminf(v, sqdist(px, py, pz, sx[j - 1], sy[j - 1], sz[j - 1]));
      hits += v >= smm[j + 1] ? 1 : 0;
    }
    bad = hits != 0;
  }
  bad = __syncthreads_or(bad);
  if (t == 0) verdict[(size_t)b * m + slice] = bad ? -1 : 0;
}

__global__ __launch_bounds__(kChainBlock) void fps_chain_kernel(const float* __restrict__ xyz,
                                                                FpsChain c) {
  __shared__ uint2 red[2][8];
  __shared__ float sxyz[3 * kChainNext];
  __shared__ float snew[2][3 * kChainNext];
  __shared__ HotLds hot;
  const int b = blockIdx.x;
  const float* __restrict__ P = xyz + (size_t)b * c.n[0] * 3;
  if (c.verdicts > 0) {  // fps_prefix_check_kernel ran before: every stage a prefix?
    const int32_t* vw = c.idx[0] + (size_t)b * c.m[0];
    bool prefix = true;
    for (int k = 0; k < c.verdicts; ++k) prefix = prefix && vw[k] == 0;
    __syncthreads();  // (every thread has read the words before any writes the row)
    if (prefix) {
      for (int i = 0; i < c.stages; ++i) {
        int32_t* I = c.idx[i] + (size_t)b * c.m[i];
        float* NX = c.nx[i] ? c.nx[i] + (size_t)b * c.m[i] * 3 : nullptr;
        for (int e = threadIdx.x; e < c.m[i]; e += kChainBlock) I[e] = e;
        if (NX)
          for (int e = threadIdx.x; e < 3 * c.m[i]; e += kChainBlock) NX[e] = P[e];
      }
      return;
    }
  }
  for (int e = threadIdx.x; e < 3 * c.n[0]; e += kChainBlock) sxyz[e] = P[e];
  // the pick slots start untagged (an earlier workgroup on this CU left its own tags there)
  for (int e = threadIdx.x; e < kChainNext; e += kChainBlock)
    hot.pc[e] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  __syncthreads();
  int tag0 = 0;  // the picks of the earlier stages: every slot tag of the launch is distinct
  for (int i = 0; i < c.stages; ++i) {
    const float* cxyz = i == 0 ? sxyz : snew[(i - 1) & 1];
    float* next = i + 1 < c.stages ? snew[i & 1] : nullptr;
    chain_stage(cxyz, c.n[i], c.m[i], cxyz, c.idx[i] + (size_t)b * c.m[i],
                c.nx[i] ? c.nx[i] + (size_t)b * c.m[i] * 3 : nullptr, next, red, hot, tag0,
                c.fault);
    tag0 += c.m[i];
    __syncthreads();  // stage i's LDS output complete before stage i+1 reads it
  }
}

// kgrid (optional, pn2_grid_size(B, M) bytes): also the picks' automatic-edge grid, exactly
// pn2_grid_build(nx, B, M, 0, kgrid): built inside the culled sampler's workgroups (N <= 8192,
// M <= 4096), else by a pn2_grid_build launch after the sampler
int fps_impl(const float* xyz, int B, int N, int M, int32_t* idx, float* nx, void* ws,
             size_t ws_bytes, hipStream_t s, int sched = PN2_FPS_AUTO, bool take = true,
             char* kgrid = nullptr, size_t kgrid_bytes = 0) {
  if (B < 0 || N < 0 || M <= 0 || (B > 0 && (!xyz || !idx))) return PN2_EINVAL;
  if (kgrid && (!nx || kgrid_bytes < pn2_grid_size(B, M) || ((uintptr_t)kgrid & 15)))
    return PN2_EINVAL;
  // the block-scan schedule exists only where the culled sampler runs (4096 < N <= 16384)
  if (sched != PN2_FPS_AUTO && sched != PN2_FPS_BLOCKSCAN) return PN2_EINVAL;
  if (sched != PN2_FPS_AUTO && (N <= 4096 || N > kMaxRegPoints)) return PN2_EINVAL;
  if (take && take_fault()) return PN2_EFAULT;
  if (B == 0) return PN2_OK;
  if (N == 0) {
    const int total = B * M;
    hipLaunchKernelGGL(fps_empty_kernel, dim3((total + 255) / 256), dim3(256), 0, s, total, idx,
                       nx);
    PN2_RETURN_LAUNCH();
  }
  // launch table measured on MI355X (round-1 sweep, B = 16 ScanNet crops,
  // profiles/r1/tune_fps.jsonl; lane-resolve variants: profiles/r1/tune_fps_lres.jsonl)
  if (N <= 64) launch_v9<64, 1, 1>(xyz, B, N, M, idx, nx, s);
  else if (N <= 128) launch_v9<64, 2, 2>(xyz, B, N, M, idx, nx, s);
  else if (N <= 256) launch_v9<64, 4, 4, true>(xyz, B, N, M, idx, nx, s);
  else if (N <= 512) launch_v9<64, 8, 4, true>(xyz, B, N, M, idx, nx, s);
  else if (N <= 1024) {
    // the hot-set schedule of the fused chain (one stage): cfg1's 1,024 -> 256 sampler
    if (M <= kChainNext) {
      FpsChain c{};
      c.stages = 1;
      c.fault = fault_word_dev();
      c.n[0] = N;
      c.m[0] = M;
      c.idx[0] = idx;
      c.nx[0] = nx;
      hipLaunchKernelGGL(fps_chain_kernel, dim3(B), dim3(kChainBlock), 0, s, xyz, c);
    } else {
      launch_v9<256, 4, 2, true>(xyz, B, N, M, idx, nx, s);
    }
  }
  else if (N <= 2048) launch_v9<256, 8, 2, true>(xyz, B, N, M, idx, nx, s);
  else if (N <= 4096) launch_v9<256, 16, 4, true>(xyz, B, N, M, idx, nx, s);
  else if (N <= 8192) {
    // culled hot-set sampler (fps_cull.h; 0.37 vs 0.71 ms at B = 16); the v9
    // block-scan sampler stays selectable for A/B timing and parity cross-checks
    if (sched == PN2_FPS_BLOCKSCAN) {
      launch_v9<256, 32, 4, true, PN2_SA1_PAD>(xyz, B, N, M, idx, nx, s);
    } else {
      if (kgrid && M <= kCullGridMax) {
        launch_hotcull_grid<16, PN2_SA1_PPT, 3, 4>(xyz, B, N, M, idx, nx, fault_word_dev(), s, kgrid);
        kgrid = nullptr;  // (built)
      } else {
        // (the LEAN form -- 53 KB of LDS, so a CU holding a sampler can take side workgroups
        // too -- measured again in round 6: the same rate, profiles/r6/lanes20, lanes500)
        launch_hotcull<16, PN2_SA1_PPT, 3, 4>(xyz, B, N, M, idx, nx, fault_word_dev(), s);
      }
    }
  }
  else if (N <= kMaxRegPoints) {
    // MSG SA1 size (cfg5, 16384 -> 512): the culled sampler with coordinates read from L2 and
    // two points per lane per cell (135 cells of 128 points), the cold points' z in LDS: 0.33
    // vs 0.59 ms for v9 512 x 32 at B = 8 (tools/fps_hot_check.py --msg,
    // profiles/r2/fps_msg_ab.log), index-exact; 12 or 8 waves spill more (0.49, 0.66 ms)
    if (sched == PN2_FPS_BLOCKSCAN) {
      launch_v9<512, 32, 4>(xyz, B, N, M, idx, nx, s);
    } else {
      launch_hotcull<16, 9, 3, 4, 16384, 2>(xyz, B, N, M, idx, nx, fault_word_dev(), s);
    }
  }
  else {
    if (!ws || ws_bytes < (size_t)B * N * sizeof(float)) return PN2_EINVAL;
    hipLaunchKernelGGL(fps_ws_kernel, dim3(B), dim3(1024), 0, s, xyz, N, M, (float*)ws, idx, nx);
  }
  if (kgrid) {  // not built inside the sampler: the grid build launch
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    return pn2_grid_build(nx, B, M, 0.0f, kgrid, kgrid_bytes, s);
  }
  PN2_RETURN_LAUNCH();
}

}  // namespace

// pn2_fps_chain's argument check, shared with the plan executor (plan.hip), which validates
// a chain launch once when it is recorded
int fps_chain_check(const float* xyz, int B, int N, int nstages, const int* npoint,
                    int32_t* const* idx, float* const* new_xyz) {
  if (B < 0 || N <= 0 || N > kMaxRegPoints || nstages < 1 || nstages > kChainMax || !npoint ||
      !idx || !new_xyz)
    return PN2_EINVAL;
  for (int i = 0; i < nstages; ++i) {
    if (npoint[i] <= 0 || !idx[i] || !new_xyz[i]) return PN2_EINVAL;
    if (i + 1 < nstages && npoint[i] > kChainNext) return PN2_EINVAL;
  }
  if (B > 0 && (!xyz || B > 65535)) return PN2_EINVAL;
  return PN2_OK;
}
int fps_take_fault() { return take_fault(); }

int fps_chain_launch(const float* xyz, int B, int N, int nstages, const int* npoint,
                     int32_t* const* idx, float* const* new_xyz, hipStream_t s, bool take,
                     void* grid0, size_t grid0_bytes) {
  const int rc0 = fps_chain_check(xyz, B, N, nstages, npoint, idx, new_xyz);
  if (rc0 != PN2_OK || B == 0) return rc0;
  if (grid0 && (grid0_bytes < pn2_grid_size(B, npoint[0]) || ((uintptr_t)grid0 & 15)))
    return PN2_EINVAL;
  int first = 0;  // first stage of the fused tail
  if (N > kChainNext) {  // the big first stage as its own sampler launch (+ its picks' grid)
    const int rc = fps_impl(xyz, B, N, npoint[0], idx[0], new_xyz[0], nullptr, 0, s,
                            PN2_FPS_AUTO, take, (char*)grid0, grid0_bytes);
    if (rc != PN2_OK) return rc;
    if (nstages == 1) return PN2_OK;
    grid0 = nullptr;
    xyz = new_xyz[0];
    N = npoint[0];
    first = 1;
  }
  FpsChain c;
  c.stages = nstages - first;
  c.fault = fault_word_dev();
  int n = N;
  bool nested = true;  // every stage samples no more points than its input holds
  for (int i = 0; i < kChainMax; ++i) {
    const bool on = i < c.stages;
    c.n[i] = on ? n : 0;
    c.m[i] = on ? npoint[first + i] : 0;
    c.idx[i] = on ? idx[first + i] : nullptr;
    c.nx[i] = on ? new_xyz[first + i] : nullptr;
    if (on) {
      nested = nested && c.m[i] <= n;
      n = c.m[i];
    }
  }
  // the prefix check (fps_prefix_check_kernel) when the verdict words fit the stage-0 row
  const int slices = (c.n[0] + kPrefixPts - 1) / kPrefixPts;
  c.verdicts = nested && c.m[0] >= 2 && c.m[0] >= slices ? slices : 0;
  if (c.verdicts)
    hipLaunchKernelGGL(fps_prefix_check_kernel, dim3(slices, B), dim3(kPrefixPts), 0, s, xyz,
                       c.n[0], c.m[0], c.idx[0]);
  hipLaunchKernelGGL(fps_chain_kernel, dim3(B), dim3(kChainBlock), 0, s, xyz, c);
  if (grid0) {  // stage 0 ran inside the chain kernel: its picks' grid as a launch after it
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    return pn2_grid_build(new_xyz[0], B, npoint[0], 0.0f, grid0, grid0_bytes, s);
  }
  PN2_RETURN_LAUNCH();
}
}  // namespace pn2

extern "C" {

int pn2_fps_max_points(void) { return pn2::kMaxRegPoints; }

#if PN2_HOT_STAMP
int pn2_hot_stamps(unsigned long long* host_out) {  // 3 x 64 x 8 u64 (DIAGNOSTIC builds only)
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(pn2::g_hot_ev),
                                  sizeof(unsigned long long) * 3 * 64 * 8, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

#if PN2_PUBLISH_BROKEN
// DIAGNOSTIC (torntest builds only): the slot reads whose tag check failed since the last call
unsigned int pn2_torn_reads(void) {
  unsigned int v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(pn2::g_torn_reads), sizeof(v), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 0xFFFFFFFFu;
  const unsigned int zero = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(pn2::g_torn_reads), &zero, sizeof(zero), 0,
                          hipMemcpyHostToDevice);
  return v;
}
#endif

int pn2_fault_status(int clear) {
  if (!pn2::g_fault_host) return 0;
  return clear ? __atomic_exchange_n(pn2::g_fault_host, 0, __ATOMIC_ACQ_REL)
               : __atomic_load_n(pn2::g_fault_host, __ATOMIC_ACQUIRE);
}

int pn2_fps_gather_sched(const float* xyz, int B, int N, int npoint, int32_t* idx,
                         float* new_xyz, int schedule, pn2_stream_t stream) {
  return pn2::fps_impl(xyz, B, N, npoint, idx, new_xyz, nullptr, 0, (hipStream_t)stream,
                       schedule);
}

int pn2_fps_chain(const float* xyz, int B, int N, int nstages, const int* npoint,
                  int32_t* const* idx, float* const* new_xyz, pn2_stream_t stream) {
  return pn2::fps_chain_launch(xyz, B, N, nstages, npoint, idx, new_xyz, (hipStream_t)stream,
                               true, nullptr, 0);
}

int pn2_fps_chain_grid(const float* xyz, int B, int N, int nstages, const int* npoint,
                       int32_t* const* idx, float* const* new_xyz, void* grid0,
                       size_t grid0_bytes, pn2_stream_t stream) {
  if (!grid0) return PN2_EINVAL;
  return pn2::fps_chain_launch(xyz, B, N, nstages, npoint, idx, new_xyz, (hipStream_t)stream,
                               true, grid0, grid0_bytes);
}

size_t pn2_fps_workspace_size(int B, int N) {
  if (B <= 0 || N <= pn2::kMaxRegPoints) return 0;
  return (size_t)B * (size_t)N * sizeof(float);
}

int pn2_fps(const float* xyz, int B, int N, int npoint, int32_t* idx, pn2_stream_t stream) {
  return pn2::fps_impl(xyz, B, N, npoint, idx, nullptr, nullptr, 0, (hipStream_t)stream);
}

int pn2_fps_gather(const float* xyz, int B, int N, int npoint, int32_t* idx, float* new_xyz,
                   pn2_stream_t stream) {
  return pn2::fps_impl(xyz, B, N, npoint, idx, new_xyz, nullptr, 0, (hipStream_t)stream);
}

int pn2_fps_ws(const float* xyz, int B, int N, int npoint, int32_t* idx, float* new_xyz,
               void* workspace, size_t workspace_bytes, pn2_stream_t stream) {
  return pn2::fps_impl(xyz, B, N, npoint, idx, new_xyz, workspace, workspace_bytes,
                       (hipStream_t)stream);
}

int pn2_gather_point(const float* inp, const int32_t* idx, int B, int N, int M, float* out,
                     pn2_stream_t stream) {
  if (B < 0 || N < 0 || M < 0) return PN2_EINVAL;
  const long long total = (long long)B * M;
  if (total == 0) return PN2_OK;
  if (total > INT32_MAX || !inp || !idx || !out) return PN2_EINVAL;
  hipLaunchKernelGGL(pn2::gather_point_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256),
                     0, (hipStream_t)stream, inp, idx, N, M, (int)total, out);
  PN2_RETURN_LAUNCH();
}

int pn2_gather_point_grad(const float* out_g, const int32_t* idx, int B, int N, int M,
                          float* inp_g, pn2_stream_t stream) {
  if (B < 0 || N < 0 || M < 0) return PN2_EINVAL;
  const size_t bytes = (size_t)B * N * 3 * sizeof(float);
  if (bytes) {
    if (!inp_g) return PN2_EINVAL;
    hipError_t e = hipMemsetAsync(inp_g, 0, bytes, (hipStream_t)stream);
    if (e != hipSuccess) return (int)e;
  }
  const long long total = (long long)B * M;
  if (total == 0) return PN2_OK;
  if (total > INT32_MAX || !out_g || !idx) return PN2_EINVAL;
  hipLaunchKernelGGL(pn2::gather_point_grad_kernel, dim3((unsigned)((total + 255) / 256)),
                     dim3(256), 0, (hipStream_t)stream, out_g, idx, N, M, (int)total, inp_g);
  PN2_RETURN_LAUNCH();
}

}  // extern "C"
