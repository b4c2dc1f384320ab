"""Uniform spatial grid over point clouds (csrc/grid.h, pn2_grid_build).

The grid is an acceleration structure only: the grid ball query and the grid three_nn return
exactly what the scans return. A grid can be built once, early (e.g. on a side stream while
the sampler runs), and reused by every op that searches the same points.
"""
import torch

from ._lib import InvalidArgumentError, check, device_tensor, lib, ptr, stream_of


class PointGrid:
    """Grid over xyz (B, N, 3). cell_edge > 0 sets the cell edge (the radius, for a ball
    query); cell_edge <= 0 lets the build choose ~2 points per cell of each cloud's bbox."""

    def __init__(self, xyz, cell_edge=0.0, name="PointGrid"):
        xyz = device_tensor(xyz, "xyz", torch.float32)
        if xyz.dim() != 3 or xyz.shape[2] != 3:
            raise InvalidArgumentError(f"{name} expects (batch_size, num_points, 3) xyz shape")
        self.xyz = xyz
        self.B, self.N = int(xyz.shape[0]), int(xyz.shape[1])
        nbytes = lib().pn2_grid_size(self.B, self.N)
        self.buf = torch.empty((max(nbytes, 16),), dtype=torch.uint8, device=xyz.device)
        check(lib().pn2_grid_build(ptr(xyz), self.B, self.N, float(cell_edge), ptr(self.buf),
                                   nbytes, stream_of(xyz)), name)

    def matches(self, xyz):
        return int(xyz.shape[0]) == self.B and int(xyz.shape[1]) == self.N
