// Latency floors of the culled sampler (diagnostic, not the product): the pieces of
// fps_hotcull_kernel (csrc/fps_cull.h) run ALONE on one CU, timed with s_memtime.
//
//   pick_floor<0>  the dependent chain of one pick, one wave, nothing else on the CU: the lane's
//                  best of 4 hot entries + the 64-lane max (hot_best4, the kernel's own asm),
//                  the exit compare, ballot + first set bit, the winner's coordinates
//                  (3 v_readlane), the distance update of the 4 entries (hot_update).
//                  No publish, no tie path (unique values), no cold waves.
//   pick_floor<1>  + the publish (hot_publish: 5 LDS writes from the winning lane): the
//                  kernel's pick step exactly, still alone on the CU.
//   round_floor    the synchronisation skeleton of one round end with 16 waves: barrier,
//                  16-lane max of the waves' maxima, barrier, 64-lane DPP sums of the count
//                  table and the choice, barrier (no counting, no appending, no cold tail).
// Build: make -C tools/ubench; run: python tools/ubench/run_floor.py
#include "../../pointcloud-segmentation-attention_amd/csrc/fps_cull.h"

using namespace pn2;

template <int VAR>
__global__ __launch_bounds__(64) void pick_floor_kernel(const float* __restrict__ xyz, int reps,
                                                        int picks, int* __restrict__ out,
                                                        unsigned long long* __restrict__ cyc) {
  __shared__ __attribute__((aligned(16))) float4 scl[260];
  __shared__ int sj[2];
  const int lane = threadIdx.x;
  int hk[4];
  hf2 hx[2], hy[2], hz[2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    hk[q] = lane + 64 * q;
    hx[q / 2][q % 2] = xyz[3 * hk[q]];
    hy[q / 2][q % 2] = xyz[3 * hk[q] + 1];
    hz[q / 2][q % 2] = xyz[3 * hk[q] + 2];
  }
  const int T = -1;  // no pick ever fails the exit test: the loop runs `picks` picks
  unsigned long long total = 0;
  int acc = 0;
  for (int r = 0; r < reps; ++r) {
    int hv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) hv[q] = __float_as_int(kInitTemp) - hk[q];  // unique values
    int va_c, va_n, vcnt;
    asm volatile("v_mov_b32 %0, %1" : "=v"(va_c)
                 : "s"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) float4*)&scl[0]));
    asm volatile("v_mov_b32 %0, %1" : "=v"(va_n)
                 : "s"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) int*)&sj[0]));
    asm volatile("v_mov_b32 %0, 1" : "=v"(vcnt));
    unsigned long long c0, c1;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0)::"memory");
    for (int p = 0; p < picks; ++p) {
      int cv, lk, wm;
      float lx, ly, lz;
      uint64_t m01, m23, mh;
      hot_best4(hv, hx, hy, hz, hk, cv, lx, ly, lz, lk, wm, m01, m23, mh);
      if (!(wm > T)) break;
      const int L = (int)__builtin_ctzll(__builtin_amdgcn_ballot_w64(cv == wm));
      float cx, cy, cz;
      if constexpr (VAR == 1) {
        hot_publish(L, va_c, va_n, vcnt, vcnt << 16, lx, ly, lz, lk, cx, cy, cz);
        va_c += 16;
        vcnt += 1;
      } else {
        cx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(lx), L));
        cy = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(ly), L));
        cz = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(lz), L));
        acc += lk;
      }
      __builtin_amdgcn_sched_barrier(0);
      hot_update<2>(hv, hx, hy, hz, cx, cy, cz);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1)::"memory");
    total += c1 - c0;
    acc += hv[0] + hv[1] + hv[2] + hv[3];
  }
  if (lane == 0) cyc[0] = total;
  out[lane] = acc + sj[0];
}

__global__ __launch_bounds__(1024) void round_floor_kernel(int rounds, int* __restrict__ out,
                                                           unsigned long long* __restrict__ cyc) {
  __shared__ int swmax[16];
  __shared__ uint32_t swcnt[16][4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int acc = 0;
  if (t < 16) swmax[t] = t * 7;
  if (t < 64) swcnt[t >> 2][t & 3] = (uint32_t)(t * 13 % 50);
  __syncthreads();
  unsigned long long c0, c1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c0)::"memory");
  for (int r = 0; r < rounds; ++r) {
    __syncthreads();  // B1
    const int top = __builtin_amdgcn_readfirstlane(wave_max_i32(lane < 16 ? swmax[lane] : -1));
    if (lane == 0) swmax[w] = top + w;
    __syncthreads();  // B2
    const int cvw = lane & 15, ciw = lane >> 4;
    uint32_t tot = swcnt[cvw][ciw];
#define PN2_ADD_DPP(C) tot += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)tot, C, 0xF, 0xF, false)
    PN2_ADD_DPP(kDppXor1);
    PN2_ADD_DPP(kDppXor2);
    PN2_ADD_DPP(kDppHalfMirror);
    PN2_ADD_DPP(kDppMirror);
#undef PN2_ADD_DPP
    const uint64_t fit = __builtin_amdgcn_ballot_w64(cvw == 0 && tot >= 1u && tot <= 256u);
    const int ti = fit ? (int)__builtin_ctzll(fit) >> 4 : 0;
    acc += __builtin_amdgcn_readlane((int)tot, ti * 16) + top;
    if (lane == 0) swcnt[w][r & 3] = (uint32_t)(acc & 63);
    __syncthreads();  // B3
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c1)::"memory");
  if (t == 0) cyc[0] = c1 - c0;
  out[t] = acc;
}

extern "C" {

// cycles of `reps` x `picks` picks (xyz: >= 256 points, picks <= 200 keeps values unique)
int pn2_pick_floor(const float* xyz, int var, int reps, int picks, int* out,
                   unsigned long long* cyc) {
  if (picks > 200 || picks < 1 || reps < 1) return PN2_EINVAL;
  if (var == 0)
    hipLaunchKernelGGL(pick_floor_kernel<0>, dim3(1), dim3(64), 0, 0, xyz, reps, picks, out, cyc);
  else if (var == 1)
    hipLaunchKernelGGL(pick_floor_kernel<1>, dim3(1), dim3(64), 0, 0, xyz, reps, picks, out, cyc);
  else
    return PN2_EINVAL;
  return (int)hipDeviceSynchronize();
}

int pn2_round_floor(int rounds, int* out, unsigned long long* cyc) {
  hipLaunchKernelGGL(round_floor_kernel, dim3(1), dim3(1024), 0, 0, rounds, out, cyc);
  return (int)hipDeviceSynchronize();
}

}  // extern "C"
