// C-ABI shim over the reference's own CPU functions, compiled unchanged from /root/reference
// by oracle/Makefile (target _ref/libref_cpu.so). TEST INFRASTRUCTURE ONLY.
//
//   query_ball_point_cpu, group_point_cpu, group_point_grad_cpu
//       pointnet2_tensorflow/tf_ops/grouping/test/query_ball_point.cpp:19-84
//   threenn_cpu (renamed pn2ref_threenn_cpu at compile time)
//       pointnet2_tensorflow/tf_ops/interpolation_3d/tf_interpolate.cpp:57-103
//       (the TensorFlow-free line range, piped from the file into g++; nothing is copied)
//   interpolate_cpu, interpolate_grad_cpu
//       pointnet2_tensorflow/tf_ops/interpolation_3d/interpolate.cpp:84-129 (identical to
//       threeinterpolate_cpu / threeinterpolate_grad_cpu of tf_interpolate.cpp:107-153)
// Only the prototypes below are ours.
#include <cstdint>

void query_ball_point_cpu(int b, int n, int m, float radius, int nsample, const float* xyz1,
                          const float* xyz2, int* idx);
void group_point_cpu(int b, int n, int c, int m, int nsample, const float* points,
                     const int* idx, float* out);
void group_point_grad_cpu(int b, int n, int c, int m, int nsample, const float* grad_out,
                          const int* idx, float* grad_points);
void pn2ref_threenn_cpu(int b, int n, int m, const float* xyz1, const float* xyz2, float* dist,
                        int* idx);
void interpolate_cpu(int b, int m, int c, int n, const float* points, const int* idx,
                     const float* weight, float* out);
void interpolate_grad_cpu(int b, int n, int c, int m, const float* grad_out, const int* idx,
                          const float* weight, float* grad_points);

extern "C" {
void pn2ref_query_ball_point(int b, int n, int m, float radius, int nsample, const float* xyz1,
                             const float* xyz2, int32_t* idx) {
  query_ball_point_cpu(b, n, m, radius, nsample, xyz1, xyz2, idx);
}
void pn2ref_group_point(int b, int n, int c, int m, int nsample, const float* points,
                        const int32_t* idx, float* out) {
  group_point_cpu(b, n, c, m, nsample, points, idx, out);
}
void pn2ref_group_point_grad(int b, int n, int c, int m, int nsample, const float* grad_out,
                             const int32_t* idx, float* grad_points) {
  group_point_grad_cpu(b, n, c, m, nsample, grad_out, idx, grad_points);
}
void pn2ref_three_nn(int b, int n, int m, const float* xyz1, const float* xyz2, float* dist,
                     int32_t* idx) {
  pn2ref_threenn_cpu(b, n, m, xyz1, xyz2, dist, idx);
}
void pn2ref_three_interpolate(int b, int m, int c, int n, const float* points,
                              const int32_t* idx, const float* weight, float* out) {
  interpolate_cpu(b, m, c, n, points, idx, weight, out);
}
void pn2ref_three_interpolate_grad(int b, int n, int c, int m, const float* grad_out,
                                   const int32_t* idx, const float* weight, float* grad_points) {
  interpolate_grad_cpu(b, n, c, m, grad_out, idx, weight, grad_points);
}
}
