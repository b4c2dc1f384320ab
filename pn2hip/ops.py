"""torch.ops.pn2.* under the reference's op names and argument order.

Each name is the registered PyTorch operator itself (csrc/torch_ops.cpp: HIP + Meta kernels,
autograd for gather_point / group_point / three_interpolate / attn_reduce), so calls are
visible to torch.compile and TorchScript:

    farthest_point_sample(npoint, inp)                tf_sampling.py:49-57
    gather_point(inp, idx)                            tf_sampling.py:30-38
    prob_sample(inp, inpr)                            tf_sampling.py:14-23
    query_ball_point(radius, nsample, xyz1, xyz2)     tf_grouping.py:8-20  -> (idx, pts_cnt)
    group_point(points, idx)                          tf_grouping.py:33-41
    select_top_k(k, dist)                             tf_grouping.py:22-31 -> (idx, dist_out)
    knn_point(k, xyz1, xyz2)                          tf_grouping.py:48-73 -> (val, idx)
    three_nn(xyz1, xyz2)                              tf_interpolate.py:8-17 -> (dist, idx)
    three_interpolate(points, idx, weight)            tf_interpolate.py:19-28
    attn_reduce(Q, K, V)                              attention_layer.py:29-45 (reduction core)
and the fused / gradient ops of the C ABI (farthest_point_sample_and_gather, group_concat,
idw_weights, fp_fused, group_pool, *_grad).
"""
import importlib

_ops = importlib.import_module("pointcloud-segmentation-attention_amd._torch_ops").ops()

NAMES = ("farthest_point_sample", "farthest_point_sample_and_gather", "gather_point",
         "gather_point_grad", "prob_sample", "query_ball_point", "select_top_k", "knn_point",
         "group_point", "group_point_grad", "group_concat", "three_nn", "three_interpolate",
         "three_interpolate_grad", "idw_weights", "fp_fused", "attn_reduce", "attn_reduce_grad",
         "group_pool")
for _n in NAMES:
    globals()[_n] = getattr(_ops, _n)

__all__ = list(NAMES)
