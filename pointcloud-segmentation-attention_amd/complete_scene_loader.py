"""The whole-scene chunker of attention_points/scannet_dataset/complete_scene_loader.py.

get_all_subsets_with_all_points_for_scene_features (:4-117) cuts a scene into 1.5 m x 1.5 m
columns (0.2 m margin), shuffles each column's points and splits them into chunks of 8192
(the last one filled up with random repeats), keeping every point's original index so that
predictions map back. Here the O(points x columns) selection (box tests + ordered compaction,
pn2_subvolume_select) and the chunk gathers (pn2_gather_rows) run on the GPU; the random
shuffles and fill-up draws stay on the host, drawn from numpy's global RandomState in the
reference's call order, so under the same np.random seed the results are the reference's
exactly (tests/golden/scene_chunks_*.npz were made by the reference function itself).

Reference quirks kept: a full chunk's sample weights are multiplied by its mask but the last
(filled-up) chunk's are not (:98-101 vs :67-71); chunks whose mask is all zero are skipped.
"""
import numpy as np
import torch

from ._lib import check, lib, ptr, stream_of
from .data_transformation import scene_bbox

NPOINTS = 8192  # :13


def _to_device(a, dev):
    t = torch.as_tensor(np.ascontiguousarray(a)) if isinstance(a, np.ndarray) else a
    return t.to(dev).contiguous()


def get_all_subsets_with_all_points_for_scene_features(points, features, get_sample_weights,
                                                       device="cuda"):
    """:4-117. points (N,3) float32 (numpy or tensor), features: list of (N, ...) arrays.
    Returns numpy (point_sets (X,8192,3), feature_sets [(X,8192,...)], sample_weights
    (X,8192) float64, masks_sets (X,8192) bool, points_orig_idxs_sets (X,8192) int64)."""
    npoints = NPOINTS
    label_weights = np.ones(21)
    label_weights[0] = 0
    dev = torch.device(device)
    P = _to_device(np.asarray(points, np.float32) if isinstance(points, np.ndarray) else
                   points.to(torch.float32), dev)
    N = int(P.shape[0])
    feats_np = [np.asarray(f) if not isinstance(f, torch.Tensor) else f.cpu().numpy()
                for f in features]
    bbox = scene_bbox(P).cpu().numpy()
    coordmin, coordmax = bbox[:3], bbox[3:]
    nsubvolume_x = np.ceil((coordmax[0] - coordmin[0]) / 1.5).astype(np.int32)  # :25-26
    nsubvolume_y = np.ceil((coordmax[1] - coordmin[1]) / 1.5).astype(np.int32)
    bounds = []
    for i in range(nsubvolume_x):
        for j in range(nsubvolume_y):
            curmin = coordmin + [i * 1.5, j * 1.5, 0]  # float64, as the reference (:34-35)
            curmax = coordmin + [(i + 1) * 1.5, (j + 1) * 1.5, coordmax[2] - coordmin[2]]
            bounds.append(np.concatenate([curmin, curmax]))
    S = len(bounds)
    point_sets, feature_sets, sample_weights, masks_sets, orig_sets = [], [[] for _ in features], \
        [], [], []
    if S and N:
        nsl = int(lib().pn2_subvolume_slices(N))
        bd = torch.from_numpy(np.asarray(bounds, np.float64)).to(dev)
        cnt = torch.empty((S, nsl), dtype=torch.int32, device=dev)
        sel = torch.empty((S, N), dtype=torch.int32, device=dev)
        inner = torch.empty((S, N), dtype=torch.uint8, device=dev)
        check(lib().pn2_subvolume_select(ptr(P), N, ptr(bd), S, 0.2, ptr(cnt), ptr(sel),
                                         ptr(inner), stream_of(P)), "subvolume_select")
        counts = cnt.sum(dim=1).cpu().numpy()
        sel_h, inner_h = sel.cpu().numpy(), inner.cpu().numpy()
    rows_all = []
    for s in range(S):
        n = int(counts[s])
        if n == 0:  # :37-39
            continue
        cur_sel, cur_mask = sel_h[s, :n], inner_h[s, :n].astype(bool)
        order = list(range(n))  # shuffle_forward (:16-19): the same RandomState call
        np.random.shuffle(order)
        cur_sel, cur_mask = cur_sel[order], cur_mask[order]
        k = 0
        for k in range(int(n / npoints)):  # :53-72
            offset = k * npoints
            rows, m = cur_sel[offset:offset + npoints], cur_mask[offset:offset + npoints]
            if sum(m) == 0:
                continue
            w = label_weights[feats_np[0][rows]] if get_sample_weights else np.ones(len(rows))
            w = w * m
            rows_all.append(rows)
            sample_weights.append(w[None])
            masks_sets.append(m[None])
            orig_sets.append(rows.astype(int)[None])
        rest = n % npoints
        if n > npoints:  # :76-79
            k = k + 1
        offset = k * npoints
        fill = np.random.choice(n, npoints - rest, replace=True)  # :87
        rows = np.concatenate((cur_sel[offset:offset + rest], cur_sel[fill]))
        m = np.concatenate((cur_mask[offset:offset + rest], np.zeros(npoints - rest, dtype=bool)))
        orig = np.concatenate((cur_sel[offset:offset + rest], np.zeros(npoints - rest, dtype=int)))
        if sum(m) == 0:
            continue
        w = label_weights[feats_np[0][rows]] if get_sample_weights else np.ones(len(rows))
        rows_all.append(rows)
        sample_weights.append(w[None])
        masks_sets.append(m[None])
        orig_sets.append(orig.astype(int)[None])
    X = len(rows_all)
    idx = torch.from_numpy(np.concatenate(rows_all).astype(np.int32)).to(dev) if X else None

    def gather(src, shape_tail, dtype_np):
        src_t = src if isinstance(src, torch.Tensor) else _to_device(np.ascontiguousarray(src), dev)
        out = torch.empty((X * npoints,) + shape_tail, dtype=src_t.dtype, device=dev)
        row_bytes = src_t[0].numel() * src_t.element_size() if src_t.dim() > 1 else src_t.element_size()
        if row_bytes % 4:
            raise ValueError("gather_rows needs rows of a multiple of 4 bytes")
        check(lib().pn2_gather_rows(ptr(src_t), N, row_bytes, ptr(idx), X * npoints, ptr(out),
                                    stream_of(src_t)), "gather_rows")
        return out.cpu().numpy().reshape((X, npoints) + shape_tail).astype(dtype_np, copy=False)

    if X == 0:  # the reference's np.concatenate of an empty tuple raises here too
        raise ValueError("need at least one array to concatenate")
    point_sets = gather(P, (3,), np.float32)
    feature_sets = [gather(f, tuple(f.shape[1:]), f.dtype) for f in feats_np]
    return (point_sets, feature_sets, np.concatenate(sample_weights, axis=0),
            np.concatenate(masks_sets, axis=0), np.concatenate(orig_sets, axis=0))


def get_all_subsets_with_all_points_for_scene_numpy(points, labels, colors, normals):
    """:120-124."""
    point_sets, feature_sets, sample_weights, masks_sets, points_orig_idxs_sets = \
        get_all_subsets_with_all_points_for_scene_features(points, [labels, colors, normals], True)
    return point_sets, feature_sets[0], feature_sets[1], feature_sets[2], \
        sample_weights, masks_sets, points_orig_idxs_sets


def get_all_subsets_with_all_points_for_scene_numpy_test(points, colors, normals):
    """:127-131."""
    point_sets, feature_sets, sample_weights, masks_sets, points_orig_idxs_sets = \
        get_all_subsets_with_all_points_for_scene_features(points, [colors, normals], False)
    return point_sets, feature_sets[0], feature_sets[1], masks_sets, points_orig_idxs_sets
