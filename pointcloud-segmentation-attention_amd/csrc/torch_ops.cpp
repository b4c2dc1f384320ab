// torch_ops.cpp — the pn2hip C ABI (include/pn2hip.h) registered as PyTorch operators,
// torch.ops.pn2.*, with the reference's op names, argument order and shape checks.
//
// This is layer (2) of the drop-in boundary: the reference exposes these
// as TensorFlow custom ops loaded by tf.load_op_library (tf_sampling.py:13, tf_grouping.py:7,
// tf_interpolate.py:7) whose OP_REQUIRES checks raise InvalidArgument; here every check raises
// ValueError (TORCH_CHECK_VALUE) with the reference's message, outputs come from the caching
// allocator, and every launch goes on the current HIP stream of the input's device
// (c10::hip::getCurrentHIPStream), so the ops compose with torch streams and hipGraph capture.
// Each op has a CUDA (= HIP on ROCm) kernel and a Meta kernel (shapes only, for fake tensors
// and torch.compile). Autograd for gather_point / group_point / three_interpolate (w.r.t.
// the points only, tf_sampling.py:44-48, tf_grouping.py:42-46, tf_interpolate.py:29-34) and
// attn_reduce is registered from Python (torch.library.register_autograd, _torch_ops.py).
// CPU kernels exist only for the three ops the reference itself runs on the CPU (ThreeNN,
// ThreeInterpolate, ThreeInterpolateGrad: registered for DEVICE_CPU only,
// tf_interpolate.cpp:187,222,262), through the host twins pn2cpu_* (csrc/cpu_interp.cpp);
// every other op has no CPU kernel, so a CPU tensor fails in the dispatcher (no CPU fallback).
#include <ATen/ATen.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <string>
#include <tuple>
#include <vector>

#include "../../include/pn2hip.h"

namespace {

using at::Tensor;

pn2_stream_t stream_of(const Tensor& t) {
  return reinterpret_cast<pn2_stream_t>(c10::hip::getCurrentHIPStream(t.device().index()).stream());
}

void check_rc(int rc, const char* op) {
  TORCH_CHECK_VALUE(rc != PN2_EINVAL, op, ": invalid argument");
  TORCH_CHECK(rc != PN2_EFAULT, op, ": an earlier sampler launch reported a device fault ",
              "(its indices are not trustworthy; see pn2_fault_status)");
  TORCH_CHECK(rc == 0, op, ": HIP error ", rc, ": ", pn2_strerror(rc));
}

// A GPU input of the reference dtype, made contiguous.
Tensor dev(const Tensor& t, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), name, " is on ", t.device(),
              ": pn2hip ops run on the MI355X only (no CPU fallback)");
  TORCH_CHECK_TYPE(t.scalar_type() == dt, name, " must be ", dt, ", got ", t.scalar_type());
  return t.contiguous();
}

int I(int64_t v) { return static_cast<int>(v); }
at::TensorOptions f32(const Tensor& like) { return like.options().dtype(at::kFloat); }
at::TensorOptions i32(const Tensor& like) { return like.options().dtype(at::kInt); }
void* P(const Tensor& t) { return t.defined() ? t.data_ptr() : nullptr; }
const float* F(const Tensor& t) { return t.defined() ? t.data_ptr<float>() : nullptr; }
const int32_t* Ii(const Tensor& t) { return t.data_ptr<int32_t>(); }

// ------------------------------------------------------------------------- shape checks
// Shared by the HIP and Meta kernels (the messages are the reference's OP_REQUIRES texts).
void chk_fps(int64_t npoint, const Tensor& inp) {
  TORCH_CHECK_VALUE(npoint > 0, "FarthestPointSample expects positive npoint");  // tf_sampling.cpp:99
  TORCH_CHECK_VALUE(inp.dim() == 3 && inp.size(2) == 3,                          // :105
                    "FarthestPointSample expects (batch_size,num_points,3) inp shape");
}
void chk_gather(const Tensor& inp, const Tensor& idx, const char* name) {
  TORCH_CHECK_VALUE(inp.dim() == 3 && inp.size(2) == 3, name,                    // :131
                    " expects (batch_size,num_points,3) inp shape");
  TORCH_CHECK_VALUE(idx.dim() == 2 && idx.size(0) == inp.size(0), name,          // :135
                    " expects (batch_size,num_result) idx shape");
}
void chk_prob(const Tensor& inp, const Tensor& inpr) {
  TORCH_CHECK_VALUE(inp.dim() == 2, "ProbSample expects (batch_size,num_choices) inp shape");
  TORCH_CHECK_VALUE(inpr.dim() == 2 && inpr.size(0) == inp.size(0),               // :76-79
                    "ProbSample expects (batch_size,num_points) inpr shape");
}
void chk_ball(double radius, int64_t nsample, const Tensor& xyz1, const Tensor& xyz2) {
  TORCH_CHECK_VALUE(radius > 0, "QueryBallPoint expects positive radius");    // tf_grouping.cpp:71
  TORCH_CHECK_VALUE(nsample > 0, "QueryBallPoint expects positive nsample");  // :74
  TORCH_CHECK_VALUE(xyz1.dim() == 3 && xyz1.size(2) == 3,                      // :79
                    "QueryBallPoint expects (batch_size, ndataset, 3) xyz1 shape.");
  TORCH_CHECK_VALUE(xyz2.dim() == 3 && xyz2.size(2) == 3,                      // :84
                    "QueryBallPoint expects (batch_size, npoint, 3) xyz2 shape.");
  TORCH_CHECK_VALUE(xyz1.size(0) == xyz2.size(0),
                    "QueryBallPoint expects xyz1 and xyz2 with the same batch size");
}
void chk_group(const Tensor& points, const Tensor& idx, const char* name) {
  TORCH_CHECK_VALUE(points.dim() == 3, name,                                   // :149
                    " expects (batch_size, num_points, channel) points shape");
  TORCH_CHECK_VALUE(idx.dim() == 3 && idx.size(0) == points.size(0), name,     // :155
                    " expects (batch_size, npoints, nsample) idx shape");
}
void chk_nn(const Tensor& xyz1, const Tensor& xyz2) {
  TORCH_CHECK_VALUE(xyz1.dim() == 3 && xyz1.size(2) == 3,            // tf_interpolate.cpp:163
                    "ThreeNN expects (b,n,3) xyz1 shape.");
  TORCH_CHECK_VALUE(xyz2.dim() == 3 && xyz2.size(2) == 3,            // :168
                    "ThreeNN expects (b,m,3) xyz2 shape.");
  TORCH_CHECK_VALUE(xyz1.size(0) == xyz2.size(0), "ThreeNN expects xyz1 and xyz2 with the same b");
}
void chk_interp(const Tensor& points, const Tensor& idx, const Tensor& weight, const char* name) {
  TORCH_CHECK_VALUE(points.dim() == 3, name, " expects (b,m,c) points shape");  // :197
  const int64_t b = points.size(0);
  TORCH_CHECK_VALUE(idx.dim() == 3 && idx.size(0) == b && idx.size(2) == 3, name,  // :203
                    " expects (b,n,3) idx shape");
  TORCH_CHECK_VALUE(weight.dim() == 3 && weight.size(0) == b && weight.size(1) == idx.size(1) &&
                        weight.size(2) == 3,
                    name, " expects (b,n,3) weight shape");                       // :206
}
void chk_attn(const Tensor& Q, const Tensor& K, const Tensor& V) {
  TORCH_CHECK_VALUE(Q.dim() == 3 && K.dim() == 4 && V.sizes() == K.sizes() &&
                        K.size(0) == Q.size(0) && K.size(1) == Q.size(1) && K.size(3) == Q.size(2),
                    "attn_reduce expects Q (B,M,C) and K, V (B,M,ns,C)");
  TORCH_CHECK_VALUE(Q.size(2) % 4 == 0, "attn_reduce expects C % 4 == 0 (key_dim 4)");
}
// fused group + centre + concat (pointnet_util.py:16-58 / :180-191): every tensor must agree
// with xyz's batch and point count, or the kernel would index past idx, new_xyz or points
void chk_group_concat(const Tensor& xyz, const std::optional<Tensor>& points,
                      const Tensor& new_xyz, const Tensor& idx) {
  TORCH_CHECK_VALUE(xyz.dim() == 3 && xyz.size(2) == 3 && new_xyz.dim() == 3 &&
                        new_xyz.size(2) == 3 && idx.dim() == 3 && idx.size(1) == new_xyz.size(1),
                    "group_concat expects xyz (B,N,3), new_xyz (B,M,3), idx (B,M,ns)");
  TORCH_CHECK_VALUE(new_xyz.size(0) == xyz.size(0) && idx.size(0) == xyz.size(0),
                    "group_concat expects xyz, new_xyz and idx with the same batch size");
  if (points.has_value() && points->numel() > 0)
    TORCH_CHECK_VALUE(points->dim() == 3 && points->size(0) == xyz.size(0) &&
                          points->size(1) == xyz.size(1),
                      "group_concat expects points (B,N,C) for xyz (B,N,3)");
}
// pooling over nsample (pointnet_util.py:130-145); weighted_avg needs grouped_xyz (B,M,ns,3)
void chk_group_pool(const Tensor& x, const std::optional<Tensor>& gxyz, int64_t mode) {
  TORCH_CHECK_VALUE(x.dim() == 4, "group_pool expects (B,M,ns,C) x");
  TORCH_CHECK_VALUE(mode >= PN2_POOL_MAX && mode <= PN2_POOL_MAX_AND_AVG, "group_pool: unknown mode");
  if (mode == PN2_POOL_WEIGHTED_AVG)
    TORCH_CHECK_VALUE(gxyz.has_value() && gxyz->dim() == 4 && gxyz->size(0) == x.size(0) &&
                          gxyz->size(1) == x.size(1) && gxyz->size(2) == x.size(2) &&
                          gxyz->size(3) == 3,
                      "group_pool weighted_avg needs grouped_xyz (B,M,ns,3)");
}

// Clouds / query batches at least this large take the spatial grid (identical results;
// the same switch as tf_grouping.GRID_MIN_* and tf_interpolate.GRID_MIN_*).
constexpr int64_t kBallGridMinPoints = 2048, kBallGridMinQueries = 1024;
constexpr int64_t kNnGridMinPairs = int64_t(1) << 21, kNnGridMinKnown = 512;

Tensor grid_over(const Tensor& xyz, double cell_edge, const char* op) {
  const int B = I(xyz.size(0)), N = I(xyz.size(1));
  const size_t bytes = pn2_grid_size(B, N);
  Tensor g = at::empty({static_cast<int64_t>(bytes > 16 ? bytes : 16)}, xyz.options().dtype(at::kByte));
  check_rc(pn2_grid_build(F(xyz), B, N, static_cast<float>(cell_edge), P(g), bytes, stream_of(xyz)), op);
  return g;
}

// ------------------------------------------------------------------------- HIP kernels
std::tuple<Tensor, Tensor> fps_and_gather_hip(int64_t npoint, const Tensor& inp_) {
  chk_fps(npoint, inp_);
  Tensor inp = dev(inp_, "inp", at::kFloat);
  c10::hip::HIPGuard g(inp.device().index());
  const int B = I(inp.size(0)), N = I(inp.size(1)), M = I(npoint);
  Tensor idx = at::empty({B, M}, i32(inp));
  Tensor nx = at::empty({B, M, 3}, f32(inp));
  if (B == 0) return {idx, nx};
  const size_t ws = pn2_fps_workspace_size(B, N);
  if (ws) {
    Tensor w = at::empty({static_cast<int64_t>((ws + 3) / 4)}, f32(inp));
    check_rc(pn2_fps_ws(F(inp), B, N, M, idx.data_ptr<int32_t>(), nx.data_ptr<float>(), P(w), ws,
                        stream_of(inp)), "FarthestPointSample");
  } else {
    check_rc(pn2_fps_gather(F(inp), B, N, M, idx.data_ptr<int32_t>(), nx.data_ptr<float>(),
                            stream_of(inp)), "FarthestPointSample");
  }
  return {idx, nx};
}
Tensor fps_hip(int64_t npoint, const Tensor& inp) { return std::get<0>(fps_and_gather_hip(npoint, inp)); }

Tensor gather_point_hip(const Tensor& inp_, const Tensor& idx_) {
  chk_gather(inp_, idx_, "GatherPoint");
  Tensor inp = dev(inp_, "inp", at::kFloat), idx = dev(idx_, "idx", at::kInt);
  c10::hip::HIPGuard g(inp.device().index());
  const int B = I(inp.size(0)), N = I(inp.size(1)), M = I(idx.size(1));
  Tensor out = at::empty({B, M, 3}, f32(inp));
  check_rc(pn2_gather_point(F(inp), Ii(idx), B, N, M, out.data_ptr<float>(), stream_of(inp)),
           "GatherPoint");
  return out;
}

Tensor gather_point_grad_hip(const Tensor& inp, const Tensor& idx_, const Tensor& out_g_) {
  chk_gather(inp, idx_, "GatherPointGradGpuOp");
  const int B = I(inp.size(0)), N = I(inp.size(1)), M = I(idx_.size(1));
  TORCH_CHECK_VALUE(out_g_.dim() == 3 && out_g_.size(0) == B && out_g_.size(1) == M &&
                        out_g_.size(2) == 3,
                    "GatherPointGradGpuOp expects (batch_size,num_result,3) out_g shape");
  Tensor idx = dev(idx_, "idx", at::kInt), out_g = dev(out_g_, "out_g", at::kFloat);
  c10::hip::HIPGuard g(out_g.device().index());
  Tensor inp_g = at::empty({B, N, 3}, f32(out_g));
  check_rc(pn2_gather_point_grad(F(out_g), Ii(idx), B, N, M, inp_g.data_ptr<float>(),
                                 stream_of(out_g)), "GatherPointGrad");
  return inp_g;
}

Tensor prob_sample_hip(const Tensor& inp_, const Tensor& inpr_) {
  chk_prob(inp_, inpr_);
  Tensor inp = dev(inp_, "inp", at::kFloat), inpr = dev(inpr_, "inpr", at::kFloat);
  c10::hip::HIPGuard g(inp.device().index());
  const int B = I(inp.size(0)), N = I(inp.size(1)), M = I(inpr.size(1));
  Tensor out = at::empty({B, M}, i32(inp));
  if (B == 0 || M == 0) return out;
  const size_t ws = pn2_prob_sample_workspace_size(B, N);
  Tensor w = at::empty({static_cast<int64_t>(ws / 4 > 1 ? ws / 4 : 1)}, f32(inp));
  check_rc(pn2_prob_sample(F(inp), F(inpr), B, N, M, w.data_ptr<float>(), ws,
                           out.data_ptr<int32_t>(), stream_of(inp)), "ProbSample");
  return out;
}

std::tuple<Tensor, Tensor> query_ball_point_hip(double radius, int64_t nsample, const Tensor& xyz1_,
                                                const Tensor& xyz2_) {
  chk_ball(radius, nsample, xyz1_, xyz2_);
  Tensor xyz1 = dev(xyz1_, "xyz1", at::kFloat), xyz2 = dev(xyz2_, "xyz2", at::kFloat);
  c10::hip::HIPGuard g(xyz1.device().index());
  const int B = I(xyz1.size(0)), N = I(xyz1.size(1)), M = I(xyz2.size(1)), ns = I(nsample);
  Tensor idx = at::empty({B, M, ns}, i32(xyz1));
  Tensor cnt = at::empty({B, M}, i32(xyz1));
  const float r = static_cast<float>(radius);
  if (N >= kBallGridMinPoints && int64_t(B) * M >= kBallGridMinQueries) {
    Tensor grid = grid_over(xyz1, r, "QueryBallPoint");
    check_rc(pn2_ball_query_grid(P(grid), F(xyz2), B, N, M, r, ns, idx.data_ptr<int32_t>(),
                                 cnt.data_ptr<int32_t>(), stream_of(xyz1)), "QueryBallPoint");
  } else {
    check_rc(pn2_ball_query(F(xyz1), F(xyz2), B, N, M, r, ns, idx.data_ptr<int32_t>(),
                            cnt.data_ptr<int32_t>(), stream_of(xyz1)), "QueryBallPoint");
  }
  return {idx, cnt};
}

std::tuple<Tensor, Tensor> select_top_k_hip(int64_t k, const Tensor& dist_) {
  TORCH_CHECK_VALUE(k > 0, "SelectionSort expects positive k");                    // :113
  TORCH_CHECK_VALUE(dist_.dim() == 3, "SelectionSort expects (b,m,n) dist shape.");  // :118
  TORCH_CHECK_VALUE(k <= dist_.size(2), "SelectionSort expects k <= n");
  Tensor dist = dev(dist_, "dist", at::kFloat);
  c10::hip::HIPGuard g(dist.device().index());
  const int B = I(dist.size(0)), m = I(dist.size(1)), n = I(dist.size(2));
  Tensor outi = at::empty({B, m, n}, i32(dist));
  Tensor out = at::empty({B, m, n}, f32(dist));
  size_t ws = pn2_select_top_k_workspace_size(B, m, I(k));
  Tensor w = at::empty({static_cast<int64_t>(ws > 16 ? ws : 16)}, dist.options().dtype(at::kByte));
  check_rc(pn2_select_top_k(F(dist), B, m, n, I(k), outi.data_ptr<int32_t>(), out.data_ptr<float>(),
                            static_cast<int32_t*>(P(w)), stream_of(dist)), "SelectionSort");
  return {outi, out};
}

void chk_knn(int64_t k, const Tensor& xyz1, const Tensor& xyz2) {
  TORCH_CHECK_VALUE(xyz1.dim() == 3 && xyz2.dim() == 3 && xyz1.size(0) == xyz2.size(0) &&
                        xyz1.size(2) == xyz2.size(2),
                    "knn_point expects (b,n,c) xyz1 and (b,m,c) xyz2");
  TORCH_CHECK_VALUE(k > 0 && k <= xyz1.size(1), "SelectionSort expects positive k");
}

std::tuple<Tensor, Tensor> knn_point_hip(int64_t k, const Tensor& xyz1_, const Tensor& xyz2_) {
  chk_knn(k, xyz1_, xyz2_);
  Tensor xyz1 = dev(xyz1_, "xyz1", at::kFloat), xyz2 = dev(xyz2_, "xyz2", at::kFloat);
  c10::hip::HIPGuard g(xyz1.device().index());
  const int B = I(xyz1.size(0)), n = I(xyz1.size(1)), c = I(xyz1.size(2)), m = I(xyz2.size(1));
  Tensor val = at::empty({B, m, k}, f32(xyz1));
  Tensor idx = at::empty({B, m, k}, i32(xyz1));
  check_rc(pn2_knn_point(F(xyz1), F(xyz2), B, n, m, c, I(k), val.data_ptr<float>(),
                         idx.data_ptr<int32_t>(), stream_of(xyz1)), "knn_point");
  return {val, idx};
}

Tensor group_point_hip(const Tensor& points_, const Tensor& idx_) {
  chk_group(points_, idx_, "GroupPoint");
  Tensor points = dev(points_, "points", at::kFloat), idx = dev(idx_, "idx", at::kInt);
  c10::hip::HIPGuard g(points.device().index());
  const int B = I(points.size(0)), N = I(points.size(1)), C = I(points.size(2));
  const int M = I(idx.size(1)), ns = I(idx.size(2));
  Tensor out = at::empty({B, M, ns, C}, f32(points));
  check_rc(pn2_group_point(F(points), Ii(idx), B, N, C, M, ns, out.data_ptr<float>(),
                           stream_of(points)), "GroupPoint");
  return out;
}

Tensor group_point_grad_hip(const Tensor& points, const Tensor& idx_, const Tensor& grad_out_) {
  chk_group(points, idx_, "GroupPointGrad");
  const int B = I(points.size(0)), N = I(points.size(1)), C = I(points.size(2));
  const int M = I(idx_.size(1)), ns = I(idx_.size(2));
  TORCH_CHECK_VALUE(grad_out_.dim() == 4 && grad_out_.size(0) == B && grad_out_.size(1) == M &&
                        grad_out_.size(2) == ns && grad_out_.size(3) == C,  // tf_grouping.cpp:191
                    "GroupPointGrad expects (batch_size, npoints, nsample, channel) grad_out shape");
  Tensor idx = dev(idx_, "idx", at::kInt), grad_out = dev(grad_out_, "grad_out", at::kFloat);
  c10::hip::HIPGuard g(grad_out.device().index());
  Tensor gp = at::empty({B, N, C}, f32(grad_out));
  check_rc(pn2_group_point_grad(F(grad_out), Ii(idx), B, N, C, M, ns, gp.data_ptr<float>(),
                                stream_of(grad_out)), "GroupPointGrad");
  return gp;
}

std::tuple<Tensor, Tensor> group_concat_hip(const Tensor& xyz_, const std::optional<Tensor>& points_,
                                            const Tensor& new_xyz_, const Tensor& idx_, bool use_xyz,
                                            bool xyz_last) {
  chk_group_concat(xyz_, points_, new_xyz_, idx_);
  Tensor xyz = dev(xyz_, "xyz", at::kFloat), new_xyz = dev(new_xyz_, "new_xyz", at::kFloat);
  Tensor idx = dev(idx_, "idx", at::kInt);
  Tensor points;
  if (points_.has_value() && points_->numel() > 0) points = dev(*points_, "points", at::kFloat);
  c10::hip::HIPGuard g(xyz.device().index());
  const int B = I(xyz.size(0)), N = I(xyz.size(1)), M = I(idx.size(1)), ns = I(idx.size(2));
  const int C = points.defined() ? I(points.size(2)) : 0;
  const int cout = !points.defined() ? 3 : (use_xyz ? C + 3 : C);
  Tensor gx = at::empty({B, M, ns, 3}, f32(xyz));
  Tensor np = at::empty({B, M, ns, cout}, f32(xyz));
  const int flags = (use_xyz ? PN2_USE_XYZ : 0) | (xyz_last ? PN2_XYZ_LAST : 0);
  check_rc(pn2_group_concat(F(xyz), F(points), F(new_xyz), Ii(idx), B, N, C, M, ns, flags,
                            gx.data_ptr<float>(), np.data_ptr<float>(), stream_of(xyz)),
           "group_concat");
  return {gx, np};
}

std::tuple<Tensor, Tensor> three_nn_hip(const Tensor& xyz1_, const Tensor& xyz2_) {
  chk_nn(xyz1_, xyz2_);
  Tensor xyz1 = dev(xyz1_, "xyz1", at::kFloat), xyz2 = dev(xyz2_, "xyz2", at::kFloat);
  c10::hip::HIPGuard g(xyz1.device().index());
  const int B = I(xyz1.size(0)), n = I(xyz1.size(1)), m = I(xyz2.size(1));
  Tensor dist = at::empty({B, n, 3}, f32(xyz1));
  Tensor idx = at::empty({B, n, 3}, i32(xyz1));
  if (int64_t(n) * m >= kNnGridMinPairs && m >= kNnGridMinKnown) {
    Tensor grid = grid_over(xyz2, 0.0, "ThreeNN");
    check_rc(pn2_three_nn_grid(P(grid), nullptr, F(xyz1), B, n, m, dist.data_ptr<float>(),
                               idx.data_ptr<int32_t>(), stream_of(xyz1)), "ThreeNN");
  } else {
    check_rc(pn2_three_nn(F(xyz1), F(xyz2), B, n, m, dist.data_ptr<float>(),
                          idx.data_ptr<int32_t>(), stream_of(xyz1)), "ThreeNN");
  }
  return {dist, idx};
}

Tensor three_interpolate_hip(const Tensor& points_, const Tensor& idx_, const Tensor& weight_) {
  chk_interp(points_, idx_, weight_, "ThreeInterpolate");
  Tensor points = dev(points_, "points", at::kFloat), idx = dev(idx_, "idx", at::kInt);
  Tensor weight = dev(weight_, "weight", at::kFloat);
  c10::hip::HIPGuard g(points.device().index());
  const int B = I(points.size(0)), m = I(points.size(1)), C = I(points.size(2)), n = I(idx.size(1));
  Tensor out = at::empty({B, n, C}, f32(points));
  check_rc(pn2_three_interpolate(F(points), Ii(idx), F(weight), B, m, C, n, out.data_ptr<float>(),
                                 stream_of(points)), "ThreeInterpolate");
  return out;
}

Tensor three_interpolate_grad_hip(const Tensor& points, const Tensor& idx_, const Tensor& weight_,
                                  const Tensor& grad_out_) {
  chk_interp(points, idx_, weight_, "ThreeInterpolateGrad");
  const int B = I(points.size(0)), m = I(points.size(1)), C = I(points.size(2)), n = I(idx_.size(1));
  TORCH_CHECK_VALUE(grad_out_.dim() == 3 && grad_out_.size(0) == B && grad_out_.size(1) == n &&
                        grad_out_.size(2) == C,  // tf_interpolate.cpp:243
                    "ThreeInterpolateGrad expects (b,n,c) grad_out shape");
  Tensor idx = dev(idx_, "idx", at::kInt), weight = dev(weight_, "weight", at::kFloat);
  Tensor grad_out = dev(grad_out_, "grad_out", at::kFloat);
  c10::hip::HIPGuard g(grad_out.device().index());
  Tensor gp = at::empty({B, m, C}, f32(grad_out));
  check_rc(pn2_three_interpolate_grad(F(grad_out), Ii(idx), F(weight), B, n, C, m,
                                      gp.data_ptr<float>(), stream_of(grad_out)),
           "ThreeInterpolateGrad");
  return gp;
}

Tensor idw_weights_hip(const Tensor& dist_) {
  TORCH_CHECK_VALUE(dist_.dim() == 3 && dist_.size(2) == 3, "idw_weights expects (b,n,3) dist shape");
  Tensor dist = dev(dist_, "dist", at::kFloat);
  c10::hip::HIPGuard g(dist.device().index());
  Tensor w = at::empty_like(dist);
  check_rc(pn2_idw_weights(F(dist), I(dist.size(0)), I(dist.size(1)), w.data_ptr<float>(),
                           stream_of(dist)), "idw_weights");
  return w;
}

Tensor fp_fused_hip(const Tensor& xyz1_, const Tensor& xyz2_, const std::optional<Tensor>& points1_,
                    const Tensor& points2_) {
  chk_nn(xyz1_, xyz2_);
  TORCH_CHECK_VALUE(points2_.dim() == 3 && points2_.size(0) == xyz2_.size(0) &&
                        points2_.size(1) == xyz2_.size(1),
                    "fp_fused expects (b,m,c2) points2");
  Tensor xyz1 = dev(xyz1_, "xyz1", at::kFloat), xyz2 = dev(xyz2_, "xyz2", at::kFloat);
  Tensor points2 = dev(points2_, "points2", at::kFloat);
  Tensor points1;
  if (points1_.has_value() && points1_->numel() > 0) {
    TORCH_CHECK_VALUE(points1_->dim() == 3 && points1_->size(0) == xyz1.size(0) &&
                          points1_->size(1) == xyz1.size(1),
                      "fp_fused expects (b,n,c1) points1");
    points1 = dev(*points1_, "points1", at::kFloat);
  }
  c10::hip::HIPGuard g(xyz1.device().index());
  const int B = I(xyz1.size(0)), n = I(xyz1.size(1)), m = I(xyz2.size(1)), C2 = I(points2.size(2));
  const int C1 = points1.defined() ? I(points1.size(2)) : 0;
  Tensor out = at::empty({B, n, C2 + C1}, f32(xyz1));
  check_rc(pn2_fp_fused(F(xyz1), F(xyz2), F(points1), C1, F(points2), C2, B, n, m,
                        out.data_ptr<float>(), stream_of(xyz1)), "fp_fused");
  return out;
}

Tensor attn_reduce_hip(const Tensor& Q_, const Tensor& K_, const Tensor& V_) {
  chk_attn(Q_, K_, V_);
  Tensor Q = dev(Q_, "Q", at::kFloat), K = dev(K_, "K", at::kFloat), V = dev(V_, "V", at::kFloat);
  c10::hip::HIPGuard g(Q.device().index());
  const int B = I(K.size(0)), M = I(K.size(1)), ns = I(K.size(2)), C = I(K.size(3));
  Tensor out = at::empty({B, M, C}, f32(Q));
  check_rc(pn2_attn_reduce(F(Q), F(K), F(V), B, M, ns, C, out.data_ptr<float>(), stream_of(Q)),
           "attn_reduce");
  return out;
}

std::tuple<Tensor, Tensor, Tensor> attn_reduce_grad_hip(const Tensor& Q_, const Tensor& K_,
                                                        const Tensor& V_, const Tensor& go_) {
  chk_attn(Q_, K_, V_);
  TORCH_CHECK_VALUE(go_.sizes() == Q_.sizes(), "attn_reduce_grad expects grad_out shaped like Q");
  Tensor Q = dev(Q_, "Q", at::kFloat), K = dev(K_, "K", at::kFloat), V = dev(V_, "V", at::kFloat);
  Tensor go = dev(go_, "grad_out", at::kFloat);
  c10::hip::HIPGuard g(Q.device().index());
  const int B = I(K.size(0)), M = I(K.size(1)), ns = I(K.size(2)), C = I(K.size(3));
  Tensor gQ = at::empty_like(Q), gK = at::empty_like(K), gV = at::empty_like(V);
  check_rc(pn2_attn_reduce_grad(F(Q), F(K), F(V), F(go), B, M, ns, C, gQ.data_ptr<float>(),
                                gK.data_ptr<float>(), gV.data_ptr<float>(), stream_of(Q)),
           "attn_reduce_grad");
  return {gQ, gK, gV};
}

Tensor group_pool_hip(const Tensor& x_, const std::optional<Tensor>& gxyz_, int64_t mode) {
  chk_group_pool(x_, gxyz_, mode);
  Tensor x = dev(x_, "x", at::kFloat);
  Tensor gxyz;
  if (mode == PN2_POOL_WEIGHTED_AVG) gxyz = dev(*gxyz_, "grouped_xyz", at::kFloat);
  c10::hip::HIPGuard g(x.device().index());
  const int B = I(x.size(0)), M = I(x.size(1)), ns = I(x.size(2)), C = I(x.size(3));
  Tensor out = at::empty({B, M, mode == PN2_POOL_MAX_AND_AVG ? 2 * C : C}, f32(x));
  check_rc(pn2_group_pool(F(x), F(gxyz), B, M, ns, C, I(mode), out.data_ptr<float>(), stream_of(x)),
           "group_pool");
  return out;
}

// ------------------------------------------------------------------------- CPU kernels
// (the reference's CPU-only ops; host twins in csrc/cpu_interp.cpp)
Tensor host(const Tensor& t, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.device().is_cpu(), name, " must be a CPU tensor here");
  TORCH_CHECK_TYPE(t.scalar_type() == dt, name, " must be ", dt, ", got ", t.scalar_type());
  return t.contiguous();
}
std::tuple<Tensor, Tensor> three_nn_cpu(const Tensor& xyz1_, const Tensor& xyz2_) {
  chk_nn(xyz1_, xyz2_);
  Tensor xyz1 = host(xyz1_, "xyz1", at::kFloat), xyz2 = host(xyz2_, "xyz2", at::kFloat);
  const int B = I(xyz1.size(0)), n = I(xyz1.size(1)), m = I(xyz2.size(1));
  Tensor dist = at::empty({B, n, 3}, f32(xyz1));
  Tensor idx = at::empty({B, n, 3}, i32(xyz1));
  check_rc(pn2cpu_three_nn(F(xyz1), F(xyz2), B, n, m, dist.data_ptr<float>(),
                           idx.data_ptr<int32_t>()), "ThreeNN");
  return {dist, idx};
}
Tensor three_interpolate_cpu(const Tensor& points_, const Tensor& idx_, const Tensor& weight_) {
  chk_interp(points_, idx_, weight_, "ThreeInterpolate");
  Tensor points = host(points_, "points", at::kFloat), idx = host(idx_, "idx", at::kInt);
  Tensor weight = host(weight_, "weight", at::kFloat);
  const int B = I(points.size(0)), m = I(points.size(1)), C = I(points.size(2)), n = I(idx.size(1));
  Tensor out = at::empty({B, n, C}, f32(points));
  check_rc(pn2cpu_three_interpolate(F(points), Ii(idx), F(weight), B, m, C, n,
                                    out.data_ptr<float>()), "ThreeInterpolate");
  return out;
}
Tensor three_interpolate_grad_cpu(const Tensor& points, const Tensor& idx_, const Tensor& weight_,
                                  const Tensor& grad_out_) {
  chk_interp(points, idx_, weight_, "ThreeInterpolateGrad");
  const int B = I(points.size(0)), m = I(points.size(1)), C = I(points.size(2)), n = I(idx_.size(1));
  TORCH_CHECK_VALUE(grad_out_.dim() == 3 && grad_out_.size(0) == B && grad_out_.size(1) == n &&
                        grad_out_.size(2) == C,  // tf_interpolate.cpp:243
                    "ThreeInterpolateGrad expects (b,n,c) grad_out shape");
  Tensor idx = host(idx_, "idx", at::kInt), weight = host(weight_, "weight", at::kFloat);
  Tensor grad_out = host(grad_out_, "grad_out", at::kFloat);
  Tensor gp = at::empty({B, m, C}, f32(grad_out));
  check_rc(pn2cpu_three_interpolate_grad(F(grad_out), Ii(idx), F(weight), B, n, C, m,
                                         gp.data_ptr<float>()), "ThreeInterpolateGrad");
  return gp;
}

// ------------------------------------------------------------------------- Meta kernels
at::TensorOptions mf(const Tensor& t) { return t.options().dtype(at::kFloat); }
at::TensorOptions mi(const Tensor& t) { return t.options().dtype(at::kInt); }

std::tuple<Tensor, Tensor> fps_and_gather_meta(int64_t npoint, const Tensor& inp) {
  chk_fps(npoint, inp);
  return {at::empty({inp.size(0), npoint}, mi(inp)), at::empty({inp.size(0), npoint, 3}, mf(inp))};
}
Tensor fps_meta(int64_t npoint, const Tensor& inp) {
  chk_fps(npoint, inp);
  return at::empty({inp.size(0), npoint}, mi(inp));
}
Tensor gather_point_meta(const Tensor& inp, const Tensor& idx) {
  chk_gather(inp, idx, "GatherPoint");
  return at::empty({inp.size(0), idx.size(1), 3}, mf(inp));
}
Tensor gather_point_grad_meta(const Tensor& inp, const Tensor& idx, const Tensor& out_g) {
  chk_gather(inp, idx, "GatherPointGradGpuOp");
  return at::empty({inp.size(0), inp.size(1), 3}, mf(out_g));
}
Tensor prob_sample_meta(const Tensor& inp, const Tensor& inpr) {
  chk_prob(inp, inpr);
  return at::empty({inp.size(0), inpr.size(1)}, mi(inp));
}
std::tuple<Tensor, Tensor> query_ball_point_meta(double radius, int64_t nsample, const Tensor& xyz1,
                                                 const Tensor& xyz2) {
  chk_ball(radius, nsample, xyz1, xyz2);
  return {at::empty({xyz1.size(0), xyz2.size(1), nsample}, mi(xyz1)),
          at::empty({xyz1.size(0), xyz2.size(1)}, mi(xyz1))};
}
std::tuple<Tensor, Tensor> select_top_k_meta(int64_t k, const Tensor& dist) {
  TORCH_CHECK_VALUE(k > 0, "SelectionSort expects positive k");
  TORCH_CHECK_VALUE(dist.dim() == 3, "SelectionSort expects (b,m,n) dist shape.");
  return {at::empty(dist.sizes(), mi(dist)), at::empty(dist.sizes(), mf(dist))};
}
std::tuple<Tensor, Tensor> knn_point_meta(int64_t k, const Tensor& xyz1, const Tensor& xyz2) {
  chk_knn(k, xyz1, xyz2);
  return {at::empty({xyz1.size(0), xyz2.size(1), k}, mf(xyz1)),
          at::empty({xyz1.size(0), xyz2.size(1), k}, mi(xyz1))};
}
Tensor group_point_meta(const Tensor& points, const Tensor& idx) {
  chk_group(points, idx, "GroupPoint");
  return at::empty({points.size(0), idx.size(1), idx.size(2), points.size(2)}, mf(points));
}
Tensor group_point_grad_meta(const Tensor& points, const Tensor& idx, const Tensor& grad_out) {
  chk_group(points, idx, "GroupPointGrad");
  return at::empty(points.sizes(), mf(grad_out));
}
std::tuple<Tensor, Tensor> group_concat_meta(const Tensor& xyz, const std::optional<Tensor>& points,
                                             const Tensor& new_xyz, const Tensor& idx,
                                             bool use_xyz, bool) {
  chk_group_concat(xyz, points, new_xyz, idx);
  const bool has = points.has_value() && points->numel() > 0;
  const int64_t C = has ? points->size(2) : 0;
  const int64_t cout = !has ? 3 : (use_xyz ? C + 3 : C);
  return {at::empty({xyz.size(0), idx.size(1), idx.size(2), 3}, mf(xyz)),
          at::empty({xyz.size(0), idx.size(1), idx.size(2), cout}, mf(xyz))};
}
std::tuple<Tensor, Tensor> three_nn_meta(const Tensor& xyz1, const Tensor& xyz2) {
  chk_nn(xyz1, xyz2);
  return {at::empty({xyz1.size(0), xyz1.size(1), 3}, mf(xyz1)),
          at::empty({xyz1.size(0), xyz1.size(1), 3}, mi(xyz1))};
}
Tensor three_interpolate_meta(const Tensor& points, const Tensor& idx, const Tensor& weight) {
  chk_interp(points, idx, weight, "ThreeInterpolate");
  return at::empty({points.size(0), idx.size(1), points.size(2)}, mf(points));
}
Tensor three_interpolate_grad_meta(const Tensor& points, const Tensor& idx, const Tensor& weight,
                                   const Tensor& grad_out) {
  chk_interp(points, idx, weight, "ThreeInterpolateGrad");
  return at::empty(points.sizes(), mf(grad_out));
}
Tensor idw_weights_meta(const Tensor& dist) {
  TORCH_CHECK_VALUE(dist.dim() == 3 && dist.size(2) == 3, "idw_weights expects (b,n,3) dist shape");
  return at::empty(dist.sizes(), mf(dist));
}
Tensor fp_fused_meta(const Tensor& xyz1, const Tensor& xyz2, const std::optional<Tensor>& points1,
                     const Tensor& points2) {
  chk_nn(xyz1, xyz2);
  const int64_t C1 = (points1.has_value() && points1->numel() > 0) ? points1->size(2) : 0;
  return at::empty({xyz1.size(0), xyz1.size(1), points2.size(2) + C1}, mf(xyz1));
}
Tensor attn_reduce_meta(const Tensor& Q, const Tensor& K, const Tensor& V) {
  chk_attn(Q, K, V);
  return at::empty(Q.sizes(), mf(Q));
}
std::tuple<Tensor, Tensor, Tensor> attn_reduce_grad_meta(const Tensor& Q, const Tensor& K,
                                                         const Tensor& V, const Tensor&) {
  chk_attn(Q, K, V);
  return {at::empty(Q.sizes(), mf(Q)), at::empty(K.sizes(), mf(K)), at::empty(V.sizes(), mf(V))};
}
Tensor group_pool_meta(const Tensor& x, const std::optional<Tensor>& gxyz, int64_t mode) {
  chk_group_pool(x, gxyz, mode);
  return at::empty({x.size(0), x.size(1), mode == PN2_POOL_MAX_AND_AVG ? 2 * x.size(3) : x.size(3)},
                   mf(x));
}

}  // namespace

// Schemas: the reference op names and argument order (tf_sampling.py, tf_grouping.py,
// tf_interpolate.py), plus the fused / extension ops of the C ABI.
TORCH_LIBRARY(pn2, m) {
  m.def("farthest_point_sample(int npoint, Tensor inp) -> Tensor");
  m.def("farthest_point_sample_and_gather(int npoint, Tensor inp) -> (Tensor, Tensor)");
  m.def("gather_point(Tensor inp, Tensor idx) -> Tensor");
  m.def("gather_point_grad(Tensor inp, Tensor idx, Tensor out_g) -> Tensor");
  m.def("prob_sample(Tensor inp, Tensor inpr) -> Tensor");
  m.def("query_ball_point(float radius, int nsample, Tensor xyz1, Tensor xyz2) -> (Tensor, Tensor)");
  m.def("select_top_k(int k, Tensor dist) -> (Tensor, Tensor)");
  m.def("knn_point(int k, Tensor xyz1, Tensor xyz2) -> (Tensor, Tensor)");
  m.def("group_point(Tensor points, Tensor idx) -> Tensor");
  m.def("group_point_grad(Tensor points, Tensor idx, Tensor grad_out) -> Tensor");
  m.def("group_concat(Tensor xyz, Tensor? points, Tensor new_xyz, Tensor idx, bool use_xyz=True, "
        "bool xyz_last=False) -> (Tensor, Tensor)");
  m.def("three_nn(Tensor xyz1, Tensor xyz2) -> (Tensor, Tensor)");
  m.def("three_interpolate(Tensor points, Tensor idx, Tensor weight) -> Tensor");
  m.def("three_interpolate_grad(Tensor points, Tensor idx, Tensor weight, Tensor grad_out) -> Tensor");
  m.def("idw_weights(Tensor dist) -> Tensor");
  m.def("fp_fused(Tensor xyz1, Tensor xyz2, Tensor? points1, Tensor points2) -> Tensor");
  m.def("attn_reduce(Tensor Q, Tensor K, Tensor V) -> Tensor");
  m.def("attn_reduce_grad(Tensor Q, Tensor K, Tensor V, Tensor grad_out) -> (Tensor, Tensor, Tensor)");
  m.def("group_pool(Tensor x, Tensor? grouped_xyz, int mode) -> Tensor");
}

// ROCm builds of PyTorch dispatch HIP tensors under the CUDA key.
TORCH_LIBRARY_IMPL(pn2, CUDA, m) {
  m.impl("farthest_point_sample", &fps_hip);
  m.impl("farthest_point_sample_and_gather", &fps_and_gather_hip);
  m.impl("gather_point", &gather_point_hip);
  m.impl("gather_point_grad", &gather_point_grad_hip);
  m.impl("prob_sample", &prob_sample_hip);
  m.impl("query_ball_point", &query_ball_point_hip);
  m.impl("select_top_k", &select_top_k_hip);
  m.impl("knn_point", &knn_point_hip);
  m.impl("group_point", &group_point_hip);
  m.impl("group_point_grad", &group_point_grad_hip);
  m.impl("group_concat", &group_concat_hip);
  m.impl("three_nn", &three_nn_hip);
  m.impl("three_interpolate", &three_interpolate_hip);
  m.impl("three_interpolate_grad", &three_interpolate_grad_hip);
  m.impl("idw_weights", &idw_weights_hip);
  m.impl("fp_fused", &fp_fused_hip);
  m.impl("attn_reduce", &attn_reduce_hip);
  m.impl("attn_reduce_grad", &attn_reduce_grad_hip);
  m.impl("group_pool", &group_pool_hip);
}

TORCH_LIBRARY_IMPL(pn2, CPU, m) {
  m.impl("three_nn", &three_nn_cpu);
  m.impl("three_interpolate", &three_interpolate_cpu);
  m.impl("three_interpolate_grad", &three_interpolate_grad_cpu);
}

TORCH_LIBRARY_IMPL(pn2, Meta, m) {
  m.impl("farthest_point_sample", &fps_meta);
  m.impl("farthest_point_sample_and_gather", &fps_and_gather_meta);
  m.impl("gather_point", &gather_point_meta);
  m.impl("gather_point_grad", &gather_point_grad_meta);
  m.impl("prob_sample", &prob_sample_meta);
  m.impl("query_ball_point", &query_ball_point_meta);
  m.impl("select_top_k", &select_top_k_meta);
  m.impl("knn_point", &knn_point_meta);
  m.impl("group_point", &group_point_meta);
  m.impl("group_point_grad", &group_point_grad_meta);
  m.impl("group_concat", &group_concat_meta);
  m.impl("three_nn", &three_nn_meta);
  m.impl("three_interpolate", &three_interpolate_meta);
  m.impl("three_interpolate_grad", &three_interpolate_grad_meta);
  m.impl("idw_weights", &idw_weights_meta);
  m.impl("fp_fused", &fp_fused_meta);
  m.impl("attn_reduce", &attn_reduce_meta);
  m.impl("attn_reduce_grad", &attn_reduce_grad_meta);
  m.impl("group_pool", &group_pool_meta);
}
