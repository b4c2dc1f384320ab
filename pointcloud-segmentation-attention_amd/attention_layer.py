"""Per-group attention reduction of attention_points/attention_scannet/attention_layer.py.

attention_reduce is the reduction core of AttentionLayer.call (:35-42) as one gfx950 kernel.
AttentionLayer mirrors the reference layer (:10-45): its Dense query/key/value projections
(:24-26) are plain torch Linear layers (dense contractions are outside the hot path), the
reduction is the kernel. The reference instantiates it with key_dim = output_dim = 4 and
num_heads = C/4 (:256-258, :313-315); that is the configuration the kernel implements.
"""
import ctypes

import torch

from . import pointnet_util, tf_grouping, tf_sampling, tf_util
from ._lib import (PN2_ATTN_MAX_LAYERS, AttnLayer, InvalidArgumentError, check, device_tensor,
                   lib, ptr, stream_of)
from ._torch_ops import call


def attention_reduce(Q, K, V):
    """Q (B,M,C), K,V (B,M,ns,C) -> (B,M,C), C = 4*heads.

    Per group and head h: K_h = the contiguous block [4*ns*h, 4*ns*(h+1)) of the group's
    flattened K (the tf.reshape reinterpretation of :35-36), s = K_h q_h / 2 (:37-38),
    a = softmax(s) (:39), out[4h:4h+4] = a^T V_h (:40-42).
    """
    if Q.dim() == 4 and Q.shape[2] == 1:  # the reference's (B,M,1,C) query vectors (:259)
        Q = Q.squeeze(2)
    if Q.dim() != 3 or K.dim() != 4 or tuple(V.shape) != tuple(K.shape):
        raise InvalidArgumentError("attention_reduce expects Q (B,M,C), K and V (B,M,ns,C)")
    B, M, ns, C = (int(s) for s in K.shape)
    if tuple(Q.shape) != (B, M, C) or C % 4 != 0:
        raise InvalidArgumentError("attention_reduce expects Q (B,M,C) with C a multiple of 4")
    # torch.ops.pn2.attn_reduce (autograd: pn2_attn_reduce_grad, _torch_ops.py)
    return call("attn_reduce", device_tensor(Q, "Q", torch.float32),
                             device_tensor(K, "K", torch.float32),
                             device_tensor(V, "V", torch.float32))


def attention_reduce_layers(qkvs):
    """attention_reduce of several layers that share nsample (the SSG stack's four SA layers)
    in ONE launch (pn2_attn_reduce_layers): qkvs = [(Q, K, V)], returns [out] per layer,
    each exactly attention_reduce(Q, K, V) (an nsample outside {8, 16, 32, 64, 128}, or a layer
    too large for the one-launch task arithmetic, runs as attention_reduce runs it). All layers
    share one nsample. Inference only (no autograd)."""
    if not 1 <= len(qkvs) <= PN2_ATTN_MAX_LAYERS:
        raise InvalidArgumentError(f"attention_reduce_layers: 1..{PN2_ATTN_MAX_LAYERS} layers")
    arr = (AttnLayer * len(qkvs))()
    outs, keep, B, ns = [], [], None, None
    for i, (Q, K, V) in enumerate(qkvs):
        if Q.dim() == 4 and Q.shape[2] == 1:
            Q = Q.squeeze(2)
        Q = device_tensor(Q, "Q", torch.float32)
        K = device_tensor(K, "K", torch.float32)
        V = device_tensor(V, "V", torch.float32)
        if Q.dim() != 3 or K.dim() != 4 or tuple(V.shape) != tuple(K.shape):
            raise InvalidArgumentError("attention_reduce_layers expects Q (B,M,C), K and V "
                                       "(B,M,ns,C)")
        b, M, n, C = (int(s) for s in K.shape)
        if tuple(Q.shape) != (b, M, C) or C % 4 != 0 or (B is not None and (b, n) != (B, ns)):
            raise InvalidArgumentError("attention_reduce_layers: Q (B,M,C), C % 4 == 0, one B "
                                       "and one nsample for all layers")
        B, ns = b, n
        out = torch.empty((B, M, C), dtype=torch.float32, device=Q.device)
        arr[i] = AttnLayer(Q.data_ptr(), K.data_ptr(), V.data_ptr(), M, n, C, out.data_ptr())
        outs.append(out)
        keep += [Q, K, V]
    check(lib().pn2_attn_reduce_layers(ctypes.addressof(arr), len(qkvs), B,
                                       stream_of(outs[0])), "attention_reduce_layers")
    return outs


def attention_reduce_grad(Q, K, V, grad_out):
    """(dQ, dK, dV) of attention_reduce for the incoming gradient grad_out (B,M,C): the
    gradient TF's autodiff takes through attention_layer.py:35-42 (pn2_attn_reduce_grad)."""
    return tuple(call("attn_reduce_grad", device_tensor(Q, "Q", torch.float32),
                                        device_tensor(K, "K", torch.float32),
                                        device_tensor(V, "V", torch.float32),
                                        device_tensor(grad_out, "grad_out", torch.float32)))


class AttentionLayer(torch.nn.Module):
    """attention_layer.py:10-45 with output_dim = key_dim = 4 (the reference's only use).

    forward([input, query]): input (B,M,ns,Cin), query (B,M,1,Cin) -> (B,M,num_heads*4).
    """

    def __init__(self, output_dim, key_dim, num_heads=16, in_dim=None):
        super().__init__()
        if output_dim != 4 or key_dim != 4:
            raise NotImplementedError("the reference uses AttentionLayer(4, 4, heads) only")
        self.output_dim, self.key_dim, self.num_heads = output_dim, key_dim, num_heads
        width = key_dim * num_heads
        in_dim = in_dim if in_dim is not None else width
        self.query_net = torch.nn.Linear(in_dim, width)  # tf.layers.Dense (:24)
        self.key_net = torch.nn.Linear(in_dim, width)    # (:25)
        self.value_net = torch.nn.Linear(in_dim, width)  # (:26)

    def forward(self, inputs):
        x, query = inputs
        Q = self.query_net(query)
        K = self.key_net(x).contiguous()
        V = self.value_net(x).contiguous()
        return attention_reduce(Q.reshape(Q.shape[0], Q.shape[1], -1).contiguous(), K, V)


def _attention_scopes(scope):
    # tf.layers.Dense names inside the Keras layer, in build order (:24-26)
    base = f"{scope}/ScannetAttentionLayer"
    return f"{base}/dense", f"{base}/dense_1", f"{base}/dense_2"


def pointnet_sa_module_attention(xyz, points, npoint, radius, nsample, mlp, mlp2, group_all,
                                 is_training, bn_decay, scope, bn=True, pooling='max', knn=False,
                                 use_xyz=True, use_nchw=False, params=None, and_pooling=False):
    """attention_layer.py:229-276 (and_pooling=True: :279-338, attention + max pool).

    Returns (new_xyz, new_points (B, npoint, mlp[-1] or mlp2[-1]), idx). Variables:
    '<scope>/conv<i>/...' (the MLP), '<scope>/ScannetAttentionLayer/dense{,_1,_2}/{kernel,bias}'
    (query, key, value), '<scope>/<scope>/{gamma,beta,moving_mean,moving_variance}' (the batch
    norm after the attention, :261), '<scope>/conv_post_<i>/...' (mlp2)."""
    store = params if params is not None else tf_util.default_store()
    pu = pointnet_util
    xyz = device_tensor(xyz, "xyz", torch.float32)
    C = int(mlp[-1])
    if C % 4:
        raise InvalidArgumentError("attention SA needs mlp[-1] % 4 == 0 (heads of 4)")
    scopes = [f"{scope}/conv{i}" for i in range(len(mlp))]
    qs, ks, vs = _attention_scopes(scope)
    empty = pu._is_empty_points(points)
    cin = (0 if empty else int(points.shape[2])) + (3 if (use_xyz or empty) else 0)
    training = is_training or pu._needs_grad(xyz, points)
    if group_all:
        new_xyz, grouped, idx, _ = pu.sample_and_group_all(xyz, points, use_xyz)
    elif training or knn:
        new_xyz, grouped, idx, _ = pu.sample_and_group(npoint, radius, nsample, xyz, points, knn,
                                                       use_xyz)
    else:
        _, new_xyz = tf_sampling.farthest_point_sample_and_gather(npoint, xyz)
        idx, _ = tf_grouping.query_ball_point(radius, nsample, xyz, new_xyz)
    if training:
        X = tf_util.mlp_torch(grouped, tf_util.torch_layers(store, scopes, cin, mlp, bn=bn),
                              is_training, bn_decay)
        dense = lambda sc, x: x @ store.dense(sc, C, C)["weights"].to(x.device) + \
            store.dense(sc, C, C)["biases"].to(x.device)  # noqa: E731
        Q = dense(qs, X[:, :, 0])
        out = attention_reduce(Q.contiguous(), dense(ks, X).contiguous(), dense(vs, X).contiguous())
        p = store.bn(f"{scope}/{scope}", C)
        layer = tf_util.TorchLayer({"weights": torch.eye(C), "biases": None, **p}, relu=False)
        out = tf_util.mlp_torch(out, [layer], is_training, bn_decay)
        if and_pooling:
            out = out + X.max(dim=2).values
    else:
        fused = tf_util.packed_mlp(store, scopes, cin, mlp, bn=bn)
        out = group_mlp_attention(xyz, points, new_xyz, idx, fused, store, scope, and_pooling,
                                  use_xyz=use_xyz)
    if mlp2:
        post = [f"{scope}/conv_post_{i}" for i in range(len(mlp2))]
        if training:
            out = tf_util.mlp_torch(out, tf_util.torch_layers(store, post, C, mlp2, bn=bn),
                                    is_training, bn_decay)
        else:
            out = tf_util.packed_mlp(store, post, C, mlp2, bn=bn)(out)
    return new_xyz, out, idx


def group_mlp_attention(xyz, points, new_xyz, idx, mlp, store, scope, and_pooling=False,
                        use_xyz=True):
    """The whole inference SA-attention layer after sampling and ball query in ONE kernel
    (pn2_group_mlp_attention): group + MLP `mlp`, Dense q/k/v, the reduction per head, the
    batch norm '<scope>/<scope>' and (and_pooling) + max pool; the per-point features never
    leave the chip. -> (B, M, C)."""
    pu = pointnet_util
    xyz = device_tensor(xyz, "xyz", torch.float32)
    new_xyz = device_tensor(new_xyz, "new_xyz", torch.float32)
    idx = device_tensor(idx, "idx", torch.int32)
    B, N = int(xyz.shape[0]), int(xyz.shape[1])
    M, ns = int(idx.shape[1]), int(idx.shape[2])
    if pu._is_empty_points(points):
        points, Cin = None, 0
    else:
        points = device_tensor(points, "points", torch.float32)
        Cin = int(points.shape[2])
    C = mlp.cout
    qkv = [tf_util.packed_dense(store, d, C, C) for d in _attention_scopes(scope)]
    table = (type(mlp.table()[0][0]) * 3)(*[d.layers[0].struct() for d in qkv])
    scale, shift = tf_util.bn_affine(store, f"{scope}/{scope}", C, xyz.device)
    out = torch.empty((B, M, C), dtype=torch.float32, device=xyz.device)
    flags = pu.PN2_USE_XYZ if use_xyz else 0
    tab, n = mlp.table()
    check(lib().pn2_group_mlp_attention(ptr(xyz), ptr(points), ptr(new_xyz), ptr(idx), B, N, Cin,
                                        M, ns, flags, n, tab, table, ptr(scale), ptr(shift),
                                        1 if and_pooling else 0, ptr(out), stream_of(xyz)),
          "group_mlp_attention")
    return out


def sa_attention_tail(X, store, scope, C, and_pooling=False):
    """Inference tail of the attention SA layers on the per-point MLP output X (B,M,ns,C):
    the Dense query (first neighbour, :259), key and value projections on the matrix cores,
    the reduction kernel, the batch norm (:261) and, for _and_pooling, + max over ns (:303)."""
    qs, ks, vs = _attention_scopes(scope)
    K = tf_util.packed_dense(store, ks, C, C)(X)
    V = tf_util.packed_dense(store, vs, C, C)(X)
    Q = tf_util.packed_dense(store, qs, C, C)(X[:, :, 0].contiguous())
    out = attention_reduce(Q, K, V)
    scale, shift = tf_util.bn_affine(store, f"{scope}/{scope}", C, X.device)
    out = out * scale + shift
    if and_pooling:  # pooling='max' only (:296-299)
        out = out + pointnet_util.group_pool(X, "max").squeeze(2)
    return out


def pointnet_sa_module_attention_and_pooling(xyz, points, npoint, radius, nsample, mlp, mlp2,
                                             group_all, is_training, bn_decay, scope, bn=True,
                                             pooling='max', knn=False, use_xyz=True,
                                             use_nchw=False, params=None):
    """attention_layer.py:279-338: attention output (after its batch norm) + max pool."""
    if pooling != 'max':
        raise ValueError("Pooling must be max for this implementation")
    return pointnet_sa_module_attention(xyz, points, npoint, radius, nsample, mlp, mlp2,
                                        group_all, is_training, bn_decay, scope, bn, pooling, knn,
                                        use_xyz, use_nchw, params, and_pooling=True)
