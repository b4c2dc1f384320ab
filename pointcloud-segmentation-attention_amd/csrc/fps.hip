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
  int n[kChainMax], m[kChainMax];
  int32_t* idx[kChainMax];
  float* nx[kChainMax];
};

// one stage (N <= kChainNext) for one cloud: the configuration fps_impl uses for this N
// (Measured and not kept, profiles/r5/chain: the 1,024-point stage on ONE wave, 16 points a
// lane and no barrier -- 126.5 -> 129 us for the chain, 140 us with each lane's candidate
// coordinates read speculatively; a single wave issues the pick's ~110 dependent VALU ops at
// ~8 cycles each, which costs what the 4-wave form's barrier and cross-wave step cost.)
PN2_DEV void chain_stage(const float* P, int N, int M, const float* CXYZ, int32_t* I, float* NX,
                         float* SNEXT, uint2 (*red)[8]) {
  const bool w0 = threadIdx.x < kWave;
  if (N <= 64) { if (w0) fps_v9_body<64, 1, 1>(P, N, M, CXYZ, I, NX, SNEXT, red); }
  else if (N <= 128) { if (w0) fps_v9_body<64, 2, 2>(P, N, M, CXYZ, I, NX, SNEXT, red); }
  else if (N <= 256) { if (w0) fps_v9_body<64, 4, 4, false, true>(P, N, M, CXYZ, I, NX, SNEXT, red); }
  else if (N <= 512) { if (w0) fps_v9_body<64, 8, 4, false, true>(P, N, M, CXYZ, I, NX, SNEXT, red); }
  else fps_v9_body<256, 4, 2, false, true>(P, N, M, CXYZ, I, NX, SNEXT, red);
}

__global__ __launch_bounds__(kChainBlock) void fps_chain_kernel(const float* __restrict__ xyz,
                                                                FpsChain c) {
  __shared__ uint2 red[2][8];
  __shared__ float sxyz[3 * kChainNext];
  __shared__ float snew[2][3 * kChainNext];
  const int b = blockIdx.x;
  const float* __restrict__ P = xyz + (size_t)b * c.n[0] * 3;
  for (int e = threadIdx.x; e < 3 * c.n[0]; e += kChainBlock) sxyz[e] = P[e];
  __syncthreads();
  for (int i = 0; i < c.stages; ++i) {
    const float* cxyz = i == 0 ? sxyz : snew[(i - 1) & 1];
    float* next = i + 1 < c.stages ? snew[i & 1] : nullptr;
    chain_stage(cxyz, c.n[i], c.m[i], cxyz, c.idx[i] + (size_t)b * c.m[i],
                c.nx[i] + (size_t)b * c.m[i] * 3, next, red);
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
  else if (N <= 1024) launch_v9<256, 4, 2, true>(xyz, B, N, M, idx, nx, s);
  else if (N <= 2048) launch_v9<256, 8, 2, true>(xyz, B, N, M, idx, nx, s);
  else if (N <= 4096) launch_v9<256, 16, 4, true>(xyz, B, N, M, idx, nx, s);
  else if (N <= 8192) {
    // culled hot-set sampler (fps_cull.h; 0.37 vs 0.71 ms at B = 16); the v9
    // block-scan sampler stays selectable for A/B timing and parity cross-checks
    if (sched == PN2_FPS_BLOCKSCAN) {
      launch_v9<256, 32, 4, true, PN2_SA1_PAD>(xyz, B, N, M, idx, nx, s);
    } else {
      if (kgrid && M <= kCullGridMax) {
        launch_hotcull_grid<16, 9, 3, 4>(xyz, B, N, M, idx, nx, fault_word_dev(), s, kgrid);
        kgrid = nullptr;  // (built)
      } else {
        launch_hotcull<16, 9, 3, 4>(xyz, B, N, M, idx, nx, fault_word_dev(), s);
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
  int n = N;
  for (int i = 0; i < kChainMax; ++i) {
    const bool on = i < c.stages;
    c.n[i] = on ? n : 0;
    c.m[i] = on ? npoint[first + i] : 0;
    c.idx[i] = on ? idx[first + i] : nullptr;
    c.nx[i] = on ? new_xyz[first + i] : nullptr;
    if (on) n = c.m[i];
  }
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
