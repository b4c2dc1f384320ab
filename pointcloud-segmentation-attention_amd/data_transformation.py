"""The crop sampler of attention_points/scannet_dataset/data_transformation.py on gfx950.

get_subset (:70-154) picks a random 1.5 m x 1.5 m column of a ScanNet scene (ten tries,
validity test, the last try when none is valid) and draws npoints of its points with
replacement. Here the whole sampler runs on the GPU (csrc/scene.hip: pn2_scene_bbox,
pn2_crop_sample), for a batch of crops of one scene at once. The reference draws its random
numbers with tf.random_uniform; here the draws are explicit inputs (centres, u) or taken from a
torch.Generator, and for the same draws the result is the reference's.

Reference quirk kept: the validity test divides the labelled-point count by
reduce_sum(ones_like(cur_points)) = 3 n (the (n, 3) tensor, :113), so no try is ever valid and
every crop is the LAST try's column.
"""
import torch

from ._lib import InvalidArgumentError, check, device_tensor, lib, ptr, stream_of

LABEL_WEIGHTS = [0, 2.743064592944318, 3.0830506790927132, 4.785754459526457, 4.9963745147506184,
                 4.372710774561782, 5.039124880965811, 4.86451825464344, 4.717751595568025,
                 4.809412839311939, 5.052097251455304, 5.389129668645318, 5.390614085649042,
                 5.127458225110977, 5.086056870814752, 5.3831185190895265, 5.422684124268539,
                 5.422955391988761, 5.433705358072363, 5.417426773812747,
                 4.870172044153657]  # data_transformation.py:82-86
TRIES = 10  # :138-141


def scene_bbox(points):
    """[min xyz, max xyz] of a (N,3) scene on the GPU (reduce_min / reduce_max, :90-91)."""
    points = device_tensor(points, "points", torch.float32)
    N = int(points.shape[0])
    ws = torch.empty(int(lib().pn2_scene_workspace_size(N)) // 4 + 1, dtype=torch.float32,
                     device=points.device)
    bbox = torch.empty(6, dtype=torch.float32, device=points.device)
    check(lib().pn2_scene_bbox(ptr(points), N, ptr(bbox), ptr(ws), ws.numel() * 4,
                               stream_of(points)), "scene_bbox")
    return bbox


def get_subsets(points, labels, colors, normals, batch, npoints=8192, centres=None, u=None,
                generator=None, label_weights=None, bbox=None):
    """`batch` crops of one scene: get_subset (:70-154) batched. centres (batch, TRIES) int32
    point indices and u (batch, npoints) uniform draws default to draws from `generator`
    (the reference's tf.random_uniform((1,), 0, len) and ((npoints,), 0, cur_len)).
    Returns points (batch,npoints,3), labels (batch,npoints), colors (batch,npoints,3) int32,
    normals (batch,npoints,3), sample_weights (batch,npoints); colors / normals may be None."""
    points = device_tensor(points, "points", torch.float32)
    labels = device_tensor(labels, "labels", torch.int32)
    dev = points.device
    N = int(points.shape[0])
    if points.dim() != 2 or points.shape[1] != 3 or tuple(labels.shape) != (N,):
        raise InvalidArgumentError("get_subset expects points (N,3) and labels (N)")
    colors = None if colors is None else device_tensor(colors, "colors", torch.int32)
    normals = None if normals is None else device_tensor(normals, "normals", torch.float32)
    if centres is None:
        r = torch.rand((batch, TRIES), generator=generator, device=dev)
        centres = (r * float(N)).to(torch.int32).clamp_(0, N - 1)
    if u is None:
        u = torch.rand((batch, npoints), generator=generator, device=dev)
    # the draws may come from the host (numpy / CPU tensors): they are inputs, not compute
    centres = device_tensor(torch.as_tensor(centres).to(dev), "centres", torch.int32)
    u = device_tensor(torch.as_tensor(u).to(dev), "u", torch.float32)
    T = int(centres.shape[1])
    lw = torch.tensor(LABEL_WEIGHTS if label_weights is None else label_weights,
                      dtype=torch.float32, device=dev)
    if bbox is None:
        bbox = scene_bbox(points)
    ws = torch.empty(int(lib().pn2_crop_workspace_size(batch, N, T)) // 4 + 1,
                     dtype=torch.float32, device=dev)
    op = torch.empty((batch, npoints, 3), dtype=torch.float32, device=dev)
    ol = torch.empty((batch, npoints), dtype=torch.int32, device=dev)
    oc = None if colors is None else torch.empty((batch, npoints, 3), dtype=torch.int32, device=dev)
    on = None if normals is None else torch.empty((batch, npoints, 3), dtype=torch.float32,
                                                  device=dev)
    ow = torch.empty((batch, npoints), dtype=torch.float32, device=dev)
    check(lib().pn2_crop_sample(ptr(points), ptr(labels), ptr(colors), ptr(normals), N, ptr(bbox),
                                ptr(centres), batch, T, ptr(u), npoints, ptr(lw), lw.numel(),
                                ptr(ws), ws.numel() * 4, ptr(op), ptr(ol), ptr(oc), ptr(on),
                                ptr(ow), stream_of(points)), "get_subset")
    return op, ol, oc, on, ow


def get_subset(points, labels, colors, normals, npoints=8192, centres=None, u=None,
               generator=None):
    """data_transformation.py:70-154 for one crop: (points (K,3), labels (K), colors (K,3),
    normals (K,3), sample_weights (K))."""
    if centres is not None:
        centres = torch.as_tensor(centres).reshape(1, -1)
    if u is not None:
        u = torch.as_tensor(u).reshape(1, -1)
    outs = get_subsets(points, labels, colors, normals, 1, npoints, centres, u, generator)
    return tuple(None if o is None else o[0] for o in outs)
