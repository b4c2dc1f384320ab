// Diagnostic build (not the product): the culled SA1 sampler of csrc/fps_cull.h with its
// s_memtime phase stamps compiled in (STAMP = true), for tools/stamp_fps_cull.py.
//   pn2_fps_cull_stamp   run B <= 16 clouds (N <= 8192); per wave x phase cycles (g_stamp) and
//                        per cloud counters (g_cull_stats): [0] kernel cycles, [1] rounds,
//                        [2] stalls, [3] applied (cell, centre) pairs of wave 1, [4] hot picks,
//                        [5] pairs of wave 2
//   pn2_fps_cull_stamp_msg  the same at the MSG SA1 size (N <= 16384)
//   pn2_fps_cull_waves   per wave: groups, group cycles, pairs, idle polls (g_cull_wave)
//   pn2_fps_cull_events  cloud 0, rounds < 64: per wave the round's event stamps (g_cull_ev)
#include "../../pointcloud-segmentation-attention_amd/csrc/fps_cull.h"

extern "C" {

int pn2_fps_cull_stamp(const float* xyz, int B, int N, int npoint, int32_t* idx,
                       unsigned long long* out_host, unsigned long long* stats_host) {
  if (N > 8192 || N <= 0 || B <= 0 || B > 16) return PN2_EINVAL;
  hipLaunchKernelGGL((pn2::fps_hotcull_kernel<16, 9, 8192, true, 3, 4>), dim3(B), dim3(1024), 0,
                     (hipStream_t)0, xyz, N, npoint, idx, nullptr, nullptr);
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_stamp),
                          sizeof(unsigned long long) * 16 * 16 * 8);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemcpyFromSymbol(stats_host, HIP_SYMBOL(pn2::g_cull_stats),
                                  sizeof(unsigned long long) * 16 * 8);
}

// the MSG SA1 size (8192 < N <= 16384: coordinates read from L2, 128-point cells)
int pn2_fps_cull_stamp_msg(const float* xyz, int B, int N, int npoint, int32_t* idx,
                           unsigned long long* out_host, unsigned long long* stats_host) {
  if (N > 16384 || N <= 0 || B <= 0 || B > 16) return PN2_EINVAL;
  hipLaunchKernelGGL((pn2::fps_hotcull_kernel<16, 9, 16384, true, 3, 4, 2>), dim3(B), dim3(1024),
                     0, (hipStream_t)0, xyz, N, npoint, idx, nullptr, nullptr);
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_stamp),
                          sizeof(unsigned long long) * 16 * 16 * 8);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemcpyFromSymbol(stats_host, HIP_SYMBOL(pn2::g_cull_stats),
                                  sizeof(unsigned long long) * 16 * 8);
}

int pn2_fps_cull_waves(unsigned long long* out_host) {
  return (int)hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_cull_wave),
                                  sizeof(unsigned long long) * 16 * 16 * 4);
}

int pn2_fps_cull_events(unsigned long long* out_host) {
  return (int)hipMemcpyFromSymbol(out_host, HIP_SYMBOL(pn2::g_cull_ev),
                                  sizeof(unsigned long long) * 64 * 16 * 8);
}

}  // extern "C"
