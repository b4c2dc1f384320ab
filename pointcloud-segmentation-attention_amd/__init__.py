"""pn2hip — MI355X-native PointNet++ geometric hot path for the attention segmentation models of
tpfeifle/pointcloud-segmentation-attention.

Drop-in modules (reference names, argument order, shapes, dtypes, error messages):
  tf_sampling     farthest_point_sample, gather_point (+grad)
  tf_grouping     query_ball_point, group_point (+grad)
  tf_interpolate  three_nn, three_interpolate (+grad)
  pointnet_util   sample_and_group(_all/_msg), group_pool, fp_interpolate,
                  pointnet_sa_module(_msg), pointnet_fp_module (fused group/interp + MLP + pool)
  tf_util         conv2d / conv1d (1x1, inference), ParamStore, SharedMLP
  data_transformation    get_subset (the ScanNet crop sampler) on the GPU
  complete_scene_loader  the whole-scene chunker (selection + gathers on the GPU)
  attention_layer attention_reduce, AttentionLayer
Everything runs the gfx950 kernels of libpn2hip.so (C ABI: include/pn2hip.h).

The directory name has hyphens, so import it with importlib:
    pn2 = importlib.import_module("pointcloud-segmentation-attention_amd")
"""
from . import attention_layer, complete_scene_loader, data_transformation, grid, plan, pointnet_util, \
    shard, stack, synth, tf_grouping, tf_interpolate, tf_sampling, tf_util
from ._lib import LIB_PATH, InvalidArgumentError, Pn2RuntimeError, lib

__all__ = ["tf_sampling", "tf_grouping", "tf_interpolate", "pointnet_util", "attention_layer", "grid", "tf_util", "data_transformation", "complete_scene_loader",
           "synth", "stack", "shard", "plan", "lib", "LIB_PATH", "InvalidArgumentError", "Pn2RuntimeError"]
