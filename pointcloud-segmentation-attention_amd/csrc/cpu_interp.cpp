// Host (CPU) kernels of the three ops the reference registers ONLY on DEVICE_CPU:
// ThreeNN, ThreeInterpolate and ThreeInterpolateGrad (pointnet2_tensorflow/tf_ops/
// interpolation_3d/tf_interpolate.cpp:187,222,262 register the CPU kernels; the arithmetic is
// threenn_cpu :60-103, threeinterpolate_cpu :107-127, threeinterpolate_grad_cpu :131-153).
//
// These are the pn2cpu_* entry points of include/pn2hip.h: the same arguments as the GPU
// entry points minus the stream, host pointers, synchronous. They exist so that a caller that
// keeps these ops on the CPU, as the reference does, gets the reference's results; the MI355X
// path (pn2_three_nn / pn2_fp_fused, interp.hip) is what the models use. Not the oracle: this
// is product code with its own structure (block distance pass + early rejection, batch
// parallelism), and tests compare it with the oracle and the reference's own CPU code.
//
// Exactness (what the reference's loops compute, bit for bit):
//  * distance: ((dx*dx + dy*dy) + dz*dz) in fp32 without contraction (this file is built with
//    -ffp-contract=off), point minus centre; the reference stores it to a double, which is
//    exact, so comparing floats orders identically; an unfilled slot holds float(1e40) = +inf;
//  * three_nn: strict '<' insertion in index order (ties keep the earlier known point);
//  * interpolate: (p1*w1 + p2*w2) + p3*w3 in fp32;
//  * grad: zero-fill, then the scatter-adds in the reference's order within each cloud
//    (clouds write disjoint rows, so splitting the batch over threads changes no sum).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "../../include/pn2hip.h"

namespace {

// run fn(b) for b in [0, B) on up to hardware_concurrency threads when the work is large
template <class F>
void for_each_cloud(int B, double work, F fn) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int nt = (int)std::min<double>({(double)B, (double)hw, std::max(1.0, work / (1 << 22))});
  if (nt <= 1) {
    for (int b = 0; b < B; ++b) fn(b);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t)
    pool.emplace_back([=, &fn] {
      for (int b = t; b < B; b += nt) fn(b);
    });
  for (auto& th : pool) th.join();
}

void three_nn_cloud(const float* x1, const float* x2, int n, int m, float* dist, int32_t* idx) {
  constexpr int KB = 256;  // known points per distance block
  float d[KB];
  for (int j = 0; j < n; ++j) {
    const float ux = x1[3 * j], uy = x1[3 * j + 1], uz = x1[3 * j + 2];
    float b1 = INFINITY, b2 = INFINITY, b3 = INFINITY;
    int i1 = 0, i2 = 0, i3 = 0;
    for (int k0 = 0; k0 < m; k0 += KB) {
      const int kn = std::min(KB, m - k0);
      for (int q = 0; q < kn; ++q) {  // vectorisable: no dependence between known points
        const float* p = x2 + 3 * (k0 + q);
        const float dx = p[0] - ux, dy = p[1] - uy, dz = p[2] - uz;
        d[q] = (dx * dx + dy * dy) + dz * dz;
      }
      for (int q = 0; q < kn; ++q) {  // the reference's insertion, in index order
        const float v = d[q];
        if (!(v < b3)) continue;
        const int k = k0 + q;
        if (v < b1) {
          b3 = b2; i3 = i2; b2 = b1; i2 = i1; b1 = v; i1 = k;
        } else if (v < b2) {
          b3 = b2; i3 = i2; b2 = v; i2 = k;
        } else {
          b3 = v; i3 = k;
        }
      }
    }
    dist[3 * j] = b1; dist[3 * j + 1] = b2; dist[3 * j + 2] = b3;
    idx[3 * j] = i1; idx[3 * j + 1] = i2; idx[3 * j + 2] = i3;
  }
}

}  // namespace

extern "C" {

int pn2cpu_three_nn(const float* xyz1, const float* xyz2, int B, int n, int m, float* dist,
                    int32_t* idx) {
  if (B < 0 || n < 0 || m < 0) return PN2_EINVAL;
  if ((long long)B * n == 0) return PN2_OK;
  if (!xyz1 || !dist || !idx || (m > 0 && !xyz2)) return PN2_EINVAL;
  for_each_cloud(B, (double)n * m * B, [&](int b) {
    three_nn_cloud(xyz1 + (size_t)b * n * 3, xyz2 + (size_t)b * m * 3, n, m,
                   dist + (size_t)b * n * 3, idx + (size_t)b * n * 3);
  });
  return PN2_OK;
}

int pn2cpu_three_interpolate(const float* points, const int32_t* idx, const float* weight, int B,
                             int m, int C, int n, float* out) {
  if (B < 0 || m < 0 || C < 0 || n < 0) return PN2_EINVAL;
  if ((long long)B * n * C == 0) return PN2_OK;
  if (!points || !idx || !weight || !out) return PN2_EINVAL;
  for_each_cloud(B, (double)n * C * B, [&](int b) {
    const float* P = points + (size_t)b * m * C;
    const int32_t* I = idx + (size_t)b * n * 3;
    const float* W = weight + (size_t)b * n * 3;
    float* O = out + (size_t)b * n * C;
    for (int j = 0; j < n; ++j) {
      const float* p1 = P + (size_t)I[3 * j] * C;
      const float* p2 = P + (size_t)I[3 * j + 1] * C;
      const float* p3 = P + (size_t)I[3 * j + 2] * C;
      const float w1 = W[3 * j], w2 = W[3 * j + 1], w3 = W[3 * j + 2];
      float* o = O + (size_t)j * C;
      for (int l = 0; l < C; ++l) o[l] = (p1[l] * w1 + p2[l] * w2) + p3[l] * w3;
    }
  });
  return PN2_OK;
}

int pn2cpu_three_interpolate_grad(const float* grad_out, const int32_t* idx, const float* weight,
                                  int B, int n, int C, int m, float* grad_points) {
  if (B < 0 || n < 0 || C < 0 || m < 0) return PN2_EINVAL;
  if ((long long)B * m * C > 0) {
    if (!grad_points) return PN2_EINVAL;
    memset(grad_points, 0, sizeof(float) * (size_t)B * m * C);  // tf_interpolate.cpp:258
  }
  if ((long long)B * n * C == 0) return PN2_OK;
  if (!grad_out || !idx || !weight) return PN2_EINVAL;
  for_each_cloud(B, (double)n * C * B, [&](int b) {
    const float* G = grad_out + (size_t)b * n * C;
    const int32_t* I = idx + (size_t)b * n * 3;
    const float* W = weight + (size_t)b * n * 3;
    float* GP = grad_points + (size_t)b * m * C;
    for (int j = 0; j < n; ++j) {
      float* g1 = GP + (size_t)I[3 * j] * C;
      float* g2 = GP + (size_t)I[3 * j + 1] * C;
      float* g3 = GP + (size_t)I[3 * j + 2] * C;
      const float w1 = W[3 * j], w2 = W[3 * j + 1], w3 = W[3 * j + 2];
      const float* g = G + (size_t)j * C;
      for (int l = 0; l < C; ++l) {  // the reference's order: i1, i2, i3 per channel
        g1[l] += g[l] * w1;
        g2[l] += g[l] * w2;
        g3[l] += g[l] * w3;
      }
    }
  });
  return PN2_OK;
}

}  // extern "C"
