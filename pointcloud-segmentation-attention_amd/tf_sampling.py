"""Farthest point sampling, gather_point and prob_sample — drop-in for
pointnet2_tensorflow/tf_ops/sampling/tf_sampling.py (same names, argument order, shapes,
dtypes and error messages), running the gfx950 kernels of libpn2hip.so through the
torch.ops.pn2 operators (csrc/torch_ops.cpp; autograd for gather_point in _torch_ops.py).
The fused sampler chain (farthest_point_sample_chain) calls the C ABI directly.
"""
import ctypes

import torch

from ._lib import InvalidArgumentError, check, device_tensor, lib, ptr, stream_of
from ._torch_ops import call


def _fps(npoint, inp, want_xyz):
    if not isinstance(npoint, int) or npoint <= 0:  # tf_sampling.cpp:99
        raise InvalidArgumentError("FarthestPointSample expects positive npoint")
    if inp.dim() != 3 or inp.shape[2] != 3:  # tf_sampling.cpp:105
        raise InvalidArgumentError(
            "FarthestPointSample expects (batch_size,num_points,3) inp shape")
    inp = device_tensor(inp, "inp", torch.float32)
    if want_xyz:
        return tuple(call("farthest_point_sample_and_gather", npoint, inp))
    return call("farthest_point_sample", npoint, inp), None


def prob_sample(inp, inpr):
    """tf_sampling.py:14-23 (ProbSample, no gradient).

    input: (batch_size, ncategory) float32 weights, (batch_size, npoints) float32 uniform draws
    returns: (batch_size, npoints) int32 — per draw r, the first category whose inclusive
    prefix sum reaches r * (the row total), with the reference's fp32 prefix-sum order
    """
    if inp.dim() != 2:  # tf_sampling.cpp:76
        raise InvalidArgumentError("ProbSample expects (batch_size,num_choices) inp shape")
    if inpr.dim() != 2 or inpr.shape[0] != inp.shape[0]:  # tf_sampling.cpp:79
        raise InvalidArgumentError("ProbSample expects (batch_size,num_points) inpr shape")
    return call("prob_sample", device_tensor(inp, "inp", torch.float32),
                             device_tensor(inpr, "inpr", torch.float32))


def farthest_point_sample(npoint, inp):
    """tf_sampling.py:49-57.

    input: int32 npoint, (batch_size, ndataset, 3) float32
    returns: (batch_size, npoint) int32
    """
    return _fps(npoint, inp, False)[0]


def farthest_point_sample_and_gather(npoint, inp):
    """(idx, new_xyz) = (farthest_point_sample(npoint, inp), gather_point(inp, idx)) in one
    kernel (pointnet_util.py:34)."""
    return _fps(npoint, inp, True)


CHAIN_MAX_POINTS = 16384  # pn2_fps_chain: first stage's points per cloud (pn2_fps_max_points)
CHAIN_MAX_FEED = 1024     # points one stage hands to the next
CHAIN_MAX_STAGES = 4


def chain_supported(N, npoints):
    return (N <= CHAIN_MAX_POINTS and 1 <= len(npoints) <= CHAIN_MAX_STAGES
            and all(0 < m <= CHAIN_MAX_FEED for m in npoints[:-1]) and npoints[-1] > 0)


def farthest_point_sample_chain(npoints, inp, out=None, grid0=None):
    """The samplers of consecutive SA layers (pn2_fps_chain: a big first stage, then the rest
    fused in one launch): stage i samples
    npoints[i] points of stage i-1's new_xyz (stage 0 of inp (B,N,3)). Returns
    [(idx_i, new_xyz_i)], each exactly farthest_point_sample_and_gather(npoints[i], input_i).
    `out` optionally supplies those tensors (written in place, e.g. a step's fixed buffers).
    grid0: a grid.PointGrid(out[0][1], build=False) (automatic edge) that the launch fills
    with stage 0's picks (pn2_fps_chain_grid: the culled sampler grids them itself), so the
    FP layer that interpolates onto the input cloud need not sort them again."""
    if inp.dim() != 3 or inp.shape[2] != 3:  # tf_sampling.cpp:105
        raise InvalidArgumentError("FarthestPointSample expects (batch_size,num_points,3) inp shape")
    npoints = [int(m) for m in npoints]
    if any(m <= 0 for m in npoints):  # tf_sampling.cpp:99
        raise InvalidArgumentError("FarthestPointSample expects positive npoint")
    inp = device_tensor(inp, "inp", torch.float32)
    B, N = int(inp.shape[0]), int(inp.shape[1])
    if not chain_supported(N, npoints):
        raise InvalidArgumentError(
            f"farthest_point_sample_chain supports N <= {CHAIN_MAX_POINTS}, <= {CHAIN_MAX_STAGES} "
            f"stages and <= {CHAIN_MAX_FEED} points fed between stages")
    if out is None:
        outs = [(torch.empty((B, m), dtype=torch.int32, device=inp.device),
                 torch.empty((B, m, 3), dtype=torch.float32, device=inp.device)) for m in npoints]
    else:
        outs = list(out)
        for (i_, x_), m in zip(outs, npoints):
            if (i_.shape != (B, m) or i_.dtype != torch.int32 or x_.shape != (B, m, 3)
                    or x_.dtype != torch.float32 or not i_.is_contiguous()
                    or not x_.is_contiguous() or i_.device != inp.device
                    or x_.device != inp.device) or len(outs) != len(npoints):
                raise InvalidArgumentError("farthest_point_sample_chain: out tensors must be "
                                           "contiguous int32 (B,m) / float32 (B,m,3) on inp's device")
    k = len(npoints)
    arr_i = (ctypes.c_int * k)(*npoints)
    arr_idx = (ctypes.c_void_p * k)(*[o[0].data_ptr() for o in outs])
    arr_nx = (ctypes.c_void_p * k)(*[o[1].data_ptr() for o in outs])
    if grid0 is not None:
        check_grid0(grid0, outs[0][1])
        check(lib().pn2_fps_chain_grid(ptr(inp), B, N, k, ctypes.addressof(arr_i),
                                       ctypes.addressof(arr_idx), ctypes.addressof(arr_nx),
                                       ptr(grid0.buf), grid0.nbytes, stream_of(inp)),
              "FarthestPointSample")
        return outs
    check(lib().pn2_fps_chain(ptr(inp), B, N, k, ctypes.addressof(arr_i),
                              ctypes.addressof(arr_idx), ctypes.addressof(arr_nx),
                              stream_of(inp)), "FarthestPointSample")
    return outs


def check_grid0(grid0, new_xyz0):
    """grid0 must be an automatic-edge PointGrid allocated over stage 0's new_xyz tensor."""
    if (grid0.cell_edge > 0 or grid0.xyz.data_ptr() != new_xyz0.data_ptr()
            or not grid0.matches(new_xyz0)):
        raise InvalidArgumentError("farthest_point_sample_chain: grid0 must be "
                                   "PointGrid(out[0][1], build=False) (automatic edge)")


def _check_gather(inp, idx, name="GatherPoint"):
    if inp.dim() != 3 or inp.shape[2] != 3:  # tf_sampling.cpp:131
        raise InvalidArgumentError(f"{name} expects (batch_size,num_points,3) inp shape")
    if idx.dim() != 2 or idx.shape[0] != inp.shape[0]:  # tf_sampling.cpp:135
        raise InvalidArgumentError(f"{name} expects (batch_size,num_result) idx shape")


def gather_point_grad(inp, idx, out_g):
    """GatherPointGrad (tf_sampling.cpp:150-178): scatter-add of out_g into inp's shape."""
    if inp.dim() != 3 or inp.shape[2] != 3:
        raise InvalidArgumentError("GatherPointGradGpuOp expects (batch_size,num_points,3) inp")
    if idx.dim() != 2 or idx.shape[0] != inp.shape[0]:
        raise InvalidArgumentError(
            "GatherPointGradGpuOp expects (batch_size,num_result) idx shape")
    B, N, M = int(inp.shape[0]), int(inp.shape[1]), int(idx.shape[1])
    if tuple(out_g.shape) != (B, M, 3):
        raise InvalidArgumentError(
            "GatherPointGradGpuOp expects (batch_size,num_result,3) out_g shape")
    return call("gather_point_grad", inp, device_tensor(idx, "idx", torch.int32),
                                   device_tensor(out_g, "out_g", torch.float32))


def gather_point(inp, idx):
    """tf_sampling.py:30-38.

    input: (batch_size, ndataset, 3) float32, (batch_size, npoints) int32
    returns: (batch_size, npoints, 3) float32 — differentiable w.r.t. inp
    """
    _check_gather(inp, idx)
    return call("gather_point", device_tensor(inp, "inp", torch.float32),
                              device_tensor(idx, "idx", torch.int32))
