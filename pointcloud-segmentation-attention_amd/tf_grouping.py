"""Ball-query grouping and group_point — drop-in for
pointnet2_tensorflow/tf_ops/grouping/tf_grouping.py (same names, argument order, shapes,
dtypes and error messages), running the gfx950 kernels of libpn2hip.so.

select_top_k / knn_point (tf_grouping.py:22-31,48-73) run knn.hip: one wavefront per query
row, radix select + the reference's selection-sort swaps replayed on at most 3k candidates,
so ties come out in exactly the reference's order; knn_point never builds the (b,m,n)
distance matrix.

Every reference-signature call goes through the torch.ops.pn2 operators (csrc/torch_ops.cpp;
autograd for group_point in _torch_ops.py); query_ball_point with a caller-built grid (the
benchmark step's early grid) calls the C ABI directly.
"""
import torch

from ._lib import InvalidArgumentError, check, device_tensor, lib, ptr, stream_of
from ._torch_ops import call
from .grid import PointGrid


# Clouds at least this large (and query batches at least this large) use the spatial grid
# (ball_grid.hip); smaller ones the in-order LDS scan (ball_query.hip). Both are exact and
# return identical results; the switch is purely a speed choice (tools/tune_bq.py).
GRID_MIN_POINTS = 2048
GRID_MIN_QUERIES = 1024


class BallGrid(PointGrid):
    """Spatial grid over xyz1 (B, N, 3) for query_ball_point (grid.PointGrid with cell edge =
    radius), reusable for any number of query batches and radii."""

    def __init__(self, xyz1, radius):
        if not radius > 0:
            raise InvalidArgumentError("QueryBallPoint expects positive radius")
        super().__init__(xyz1, float(radius), name="QueryBallPoint")


def query_ball_point(radius, nsample, xyz1, xyz2, grid=None):
    """tf_grouping.py:8-20.

    Input:
        radius: float32, ball search radius
        nsample: int32, number of points selected in each ball region
        xyz1: (batch_size, ndataset, 3) float32 array, input points
        xyz2: (batch_size, npoint, 3) float32 array, query points
        grid: optional BallGrid built over xyz1 (extension: lets callers build it early,
              e.g. concurrently with the sampler); built here when the cloud is large
    Output:
        idx: (batch_size, npoint, nsample) int32 array, indices to input points
        pts_cnt: (batch_size, npoint) int32 array, number of unique points in each local region
    """
    if not radius > 0:  # tf_grouping.cpp:71
        raise InvalidArgumentError("QueryBallPoint expects positive radius")
    if int(nsample) <= 0:  # tf_grouping.cpp:74
        raise InvalidArgumentError("QueryBallPoint expects positive nsample")
    if xyz1.dim() != 3 or xyz1.shape[2] != 3:  # tf_grouping.cpp:79
        raise InvalidArgumentError("QueryBallPoint expects (batch_size, ndataset, 3) xyz1 shape.")
    if xyz2.dim() != 3 or xyz2.shape[2] != 3:  # tf_grouping.cpp:84
        raise InvalidArgumentError("QueryBallPoint expects (batch_size, npoint, 3) xyz2 shape.")
    xyz1 = device_tensor(xyz1, "xyz1", torch.float32)
    xyz2 = device_tensor(xyz2, "xyz2", torch.float32)
    if grid is None:  # the op builds the grid itself when the cloud is large (same switch)
        return tuple(call("query_ball_point", float(radius), int(nsample), xyz1, xyz2))
    if not grid.matches(xyz1):
        raise InvalidArgumentError("QueryBallPoint grid was built over a different xyz1")
    B, N = int(xyz1.shape[0]), int(xyz1.shape[1])
    M, ns = int(xyz2.shape[1]), int(nsample)
    idx = torch.empty((B, M, ns), dtype=torch.int32, device=xyz1.device)
    pts_cnt = torch.empty((B, M), dtype=torch.int32, device=xyz1.device)
    check(lib().pn2_ball_query_grid(ptr(grid.buf), ptr(xyz2), B, N, M, float(radius), ns,
                                    ptr(idx), ptr(pts_cnt), stream_of(xyz1)), "QueryBallPoint")
    return idx, pts_cnt


def select_top_k(k, dist):
    """tf_grouping.py:22-31 (SelectionSort, tf_grouping_g.cu:83-123).

    Input:
        k: int32, number of k SMALLEST elements selected
        dist: (b,m,n) float32 array, distance matrix, m query points, n dataset points
    Output:
        idx: (b,m,n) int32 array, first k in n are indices to the top k
        dist_out: (b,m,n) float32 array, first k in n are the top k
    """
    if int(k) <= 0:  # tf_grouping.cpp:113
        raise InvalidArgumentError("SelectionSort expects positive k")
    if dist.dim() != 3:  # tf_grouping.cpp:118
        raise InvalidArgumentError("SelectionSort expects (b,m,n) dist shape.")
    dist = device_tensor(dist, "dist", torch.float32)
    if int(k) > int(dist.shape[2]):
        raise InvalidArgumentError("SelectionSort expects k <= n")
    return tuple(call("select_top_k", int(k), dist))


def knn_point(k, xyz1, xyz2):
    """tf_grouping.py:48-73.

    Input:
        k: int32, number of k in k-nn search
        xyz1: (batch_size, ndataset, c) float32 array, input points
        xyz2: (batch_size, npoint, c) float32 array, query points
    Output:
        val: (batch_size, npoint, k) float32 array, L2 distances (squared, as the reference's
             reduce_sum of squares)
        idx: (batch_size, npoint, k) int32 array, indices to input points
    """
    if xyz1.dim() != 3 or xyz2.dim() != 3 or xyz1.shape[0] != xyz2.shape[0] \
            or xyz1.shape[2] != xyz2.shape[2]:
        raise InvalidArgumentError("knn_point expects (b,n,c) xyz1 and (b,m,c) xyz2")
    xyz1 = device_tensor(xyz1, "xyz1", torch.float32)
    xyz2 = device_tensor(xyz2, "xyz2", torch.float32)
    if not 0 < int(k) <= int(xyz1.shape[1]):
        raise InvalidArgumentError("SelectionSort expects positive k")
    return tuple(call("knn_point", int(k), xyz1, xyz2))


def _check_group(points, idx, name="GroupPoint"):
    if points.dim() != 3:  # tf_grouping.cpp:149
        raise InvalidArgumentError(f"{name} expects (batch_size, num_points, channel) points shape")
    if idx.dim() != 3 or idx.shape[0] != points.shape[0]:  # tf_grouping.cpp:155
        raise InvalidArgumentError(f"{name} expects (batch_size, npoints, nsample) idx shape")


def group_point_grad(points, idx, grad_out):
    """GroupPointGrad (tf_grouping.cpp:174-208)."""
    _check_group(points, idx, "GroupPointGrad")
    B, N, C = (int(s) for s in points.shape)
    M, ns = int(idx.shape[1]), int(idx.shape[2])
    if tuple(grad_out.shape) != (B, M, ns, C):  # tf_grouping.cpp:191
        raise InvalidArgumentError(
            "GroupPointGrad expects (batch_size, npoints, nsample, channel) grad_out shape")
    return call("group_point_grad", points, device_tensor(idx, "idx", torch.int32),
                                  device_tensor(grad_out, "grad_out", torch.float32))


def group_point(points, idx):
    """tf_grouping.py:33-41.

    Input:
        points: (batch_size, ndataset, channel) float32 array, points to sample from
        idx: (batch_size, npoint, nsample) int32 array, indices to points
    Output:
        out: (batch_size, npoint, nsample, channel) float32 array — differentiable w.r.t. points
    """
    _check_group(points, idx)
    return call("group_point", device_tensor(points, "points", torch.float32),
                             device_tensor(idx, "idx", torch.int32))
