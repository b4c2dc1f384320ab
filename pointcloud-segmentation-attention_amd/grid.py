"""Uniform spatial grid over point clouds (csrc/grid.h, pn2_grid_build).

The grid is an acceleration structure only: the grid ball query and the grid three_nn return
exactly what the scans return. A grid can be built once, early (e.g. on a side stream while
the sampler runs), and reused by every op that searches the same points.
"""
import torch

from ._lib import InvalidArgumentError, check, device_tensor, lib, ptr, stream_of


class PointGrid:
    """Grid over xyz (B, N, 3). cell_edge > 0 sets the cell edge (the radius, for a ball
    query); cell_edge <= 0 lets the build choose ~2 points per cell of each cloud's bbox.
    build=False only allocates it: a kernel that writes xyz fills it later (the SA1 sampler,
    tf_sampling.farthest_point_sample_chain(grid0=...), grids its picks for FP4)."""

    def __init__(self, xyz, cell_edge=0.0, name="PointGrid", build=True):
        xyz = device_tensor(xyz, "xyz", torch.float32)
        if xyz.dim() != 3 or xyz.shape[2] != 3:
            raise InvalidArgumentError(f"{name} expects (batch_size, num_points, 3) xyz shape")
        self.xyz = xyz
        self.B, self.N = int(xyz.shape[0]), int(xyz.shape[1])
        self.cell_edge = float(cell_edge)
        self.nbytes = lib().pn2_grid_size(self.B, self.N)
        self.buf = torch.empty((max(self.nbytes, 16),), dtype=torch.uint8, device=xyz.device)
        if build:
            check(lib().pn2_grid_build(ptr(xyz), self.B, self.N, self.cell_edge, ptr(self.buf),
                                       self.nbytes, stream_of(xyz)), name)

    def rebuild(self):
        """Build the grid again over self.xyz (its current contents) on the current stream."""
        check(lib().pn2_grid_build(ptr(self.xyz), self.B, self.N, self.cell_edge, ptr(self.buf),
                                   self.nbytes, stream_of(self.xyz)), "PointGrid")

    def matches(self, xyz):
        return int(xyz.shape[0]) == self.B and int(xyz.shape[1]) == self.N
