"""three_nn / three_interpolate — drop-in for
pointnet2_tensorflow/tf_ops/interpolation_3d/tf_interpolate.py (same names, argument order,
shapes, dtypes and error messages). The reference registers these ops for DEVICE_CPU only
(tf_interpolate.cpp:187,222,262); here they are gfx950 kernels and the data never leaves HBM
(CPU tensors run the host twins pn2cpu_*, as the reference does). Reference-signature calls go
through the torch.ops.pn2 operators (csrc/torch_ops.cpp; autograd for three_interpolate in
_torch_ops.py); three_nn with caller-built grids calls the C ABI directly.
"""
import torch

from ._lib import InvalidArgumentError, check, device_tensor, lib, ptr, stream_of


def _tensor(t, name, dtype):
    """An op input: on the GPU (the HIP kernels), or on the CPU -- these three ops are the
    reference's CPU-only ones (tf_interpolate.cpp:187,222,262), so CPU tensors run the host
    twins pn2cpu_* (csrc/cpu_interp.cpp) through the ops' CPU kernels."""
    if isinstance(t, torch.Tensor) and t.device.type == "cpu":
        if t.dtype != dtype:
            raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
        return t.contiguous()
    return device_tensor(t, name, dtype)
from ._torch_ops import call
from .grid import PointGrid


# three_nn searches over a grid of the known points when the brute-force scan would test at
# least this many (unknown, known) pairs per cloud and the known cloud is this large
# (identical results either way; tools/tune_nn.py measured the switch).
GRID_MIN_PAIRS = 1 << 21
GRID_MIN_KNOWN = 512


def use_grid(n, m):
    return n * m >= GRID_MIN_PAIRS and m >= GRID_MIN_KNOWN


def three_nn(xyz1, xyz2, known_grid=None, unknown_grid=None):
    """tf_interpolate.py:8-17.

    Input:
        xyz1: (b,n,3) float32 array, unknown points
        xyz2: (b,m,3) float32 array, known points
        known_grid / unknown_grid: optional grid.PointGrid over xyz2 / xyz1 (extension; the
            known grid is built here when the search is large)
    Output:
        dist: (b,n,3) float32 array, (squared) distances to known points
        idx: (b,n,3) int32 array, indices to known points
    """
    if xyz1.dim() != 3 or xyz1.shape[2] != 3:  # tf_interpolate.cpp:163
        raise InvalidArgumentError("ThreeNN expects (b,n,3) xyz1 shape.")
    if xyz2.dim() != 3 or xyz2.shape[2] != 3:  # tf_interpolate.cpp:168
        raise InvalidArgumentError("ThreeNN expects (b,m,3) xyz2 shape.")
    xyz1 = _tensor(xyz1, "xyz1", torch.float32)
    xyz2 = _tensor(xyz2, "xyz2", torch.float32)
    if xyz1.device != xyz2.device:
        raise RuntimeError("ThreeNN: xyz1 and xyz2 must be on the same device")
    if xyz1.device.type == "cpu":  # the reference's own placement (DEVICE_CPU only)
        if known_grid is not None or unknown_grid is not None:
            raise RuntimeError("ThreeNN grids are GPU structures")
        return tuple(call("three_nn", xyz1, xyz2))
    if known_grid is None and unknown_grid is None:  # the op picks the grid search itself
        return tuple(call("three_nn", xyz1, xyz2))
    B, n, m = int(xyz1.shape[0]), int(xyz1.shape[1]), int(xyz2.shape[1])
    dist = torch.empty((B, n, 3), dtype=torch.float32, device=xyz1.device)
    idx = torch.empty((B, n, 3), dtype=torch.int32, device=xyz1.device)
    if known_grid is None and use_grid(n, m):
        known_grid = PointGrid(xyz2, 0.0, name="ThreeNN")
    if known_grid is not None:
        if not known_grid.matches(xyz2) or (unknown_grid is not None and not unknown_grid.matches(xyz1)):
            raise InvalidArgumentError("ThreeNN grid was built over different points")
        check(lib().pn2_three_nn_grid(ptr(known_grid.buf),
                                      None if unknown_grid is None else ptr(unknown_grid.buf),
                                      ptr(xyz1), B, n, m, ptr(dist), ptr(idx), stream_of(xyz1)),
              "ThreeNN")
    else:
        check(lib().pn2_three_nn(ptr(xyz1), ptr(xyz2), B, n, m, ptr(dist), ptr(idx),
                                 stream_of(xyz1)), "ThreeNN")
    return dist, idx


def _check_interp(points, idx, weight, name="ThreeInterpolate"):
    if points.dim() != 3:  # tf_interpolate.cpp:197
        raise InvalidArgumentError(f"{name} expects (b,m,c) points shape")
    b = points.shape[0]
    if idx.dim() != 3 or idx.shape[0] != b or idx.shape[2] != 3:  # :203
        raise InvalidArgumentError(f"{name} expects (b,n,3) idx shape")
    if weight.dim() != 3 or tuple(weight.shape) != (b, idx.shape[1], 3):  # :206
        raise InvalidArgumentError(f"{name} expects (b,n,3) weight shape")


def three_interpolate_grad(points, idx, weight, grad_out):
    """ThreeInterpolateGrad (tf_interpolate.cpp:225-262)."""
    _check_interp(points, idx, weight, "ThreeInterpolateGrad")
    B, m, C = (int(s) for s in points.shape)
    if tuple(grad_out.shape) != (B, idx.shape[1], C):  # :243
        raise InvalidArgumentError("ThreeInterpolateGrad expects (b,n,c) grad_out shape")
    return call("three_interpolate_grad", points, _tensor(idx, "idx", torch.int32),
                                        _tensor(weight, "weight", torch.float32),
                                        _tensor(grad_out, "grad_out", torch.float32))


def three_interpolate(points, idx, weight):
    """tf_interpolate.py:19-28.

    Input:
        points: (b,m,c) float32 array, known points
        idx: (b,n,3) int32 array, indices to known points
        weight: (b,n,3) float32 array, weights on known points
    Output:
        out: (b,n,c) float32 array, interpolated point values — differentiable w.r.t. points
    """
    _check_interp(points, idx, weight)
    return call("three_interpolate", _tensor(points, "points", torch.float32),
                                   _tensor(idx, "idx", torch.int32),
                                   _tensor(weight, "weight", torch.float32))


def idw_weights(dist):
    """The inverse-distance weights of pointnet_fp_module (pointnet_util.py:219-222):
    d = max(dist, 1e-10); weight = (1/d) / sum_3(1/d)."""
    if dist.dim() != 3 or dist.shape[2] != 3:
        raise InvalidArgumentError("idw_weights expects (b,n,3) dist shape")
    return call("idw_weights", device_tensor(dist, "dist", torch.float32))
