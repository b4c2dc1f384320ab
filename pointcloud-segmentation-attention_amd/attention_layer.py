"""Per-group attention reduction of attention_points/attention_scannet/attention_layer.py.

attention_reduce is the reduction core of AttentionLayer.call (:35-42) as one gfx950 kernel.
AttentionLayer mirrors the reference layer (:10-45): its Dense query/key/value projections
(:24-26) are plain torch Linear layers (dense contractions are outside the hot path), the
reduction is the kernel. The reference instantiates it with key_dim = output_dim = 4 and
num_heads = C/4 (:256-258, :313-315); that is the configuration the kernel implements.
"""
import torch

from ._lib import InvalidArgumentError, check, device_tensor, lib, ptr, stream_of


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
    Q = device_tensor(Q, "Q", torch.float32)
    K = device_tensor(K, "K", torch.float32)
    V = device_tensor(V, "V", torch.float32)
    if torch.is_grad_enabled() and (Q.requires_grad or K.requires_grad or V.requires_grad):
        return _AttentionReduce.apply(Q, K, V)
    return _attn_fwd(Q, K, V)


def _attn_fwd(Q, K, V):
    B, M, ns, C = (int(s) for s in K.shape)
    out = torch.empty((B, M, C), dtype=torch.float32, device=Q.device)
    check(lib().pn2_attn_reduce(ptr(Q), ptr(K), ptr(V), B, M, ns, C, ptr(out), stream_of(Q)),
          "attention_reduce")
    return out


def attention_reduce_grad(Q, K, V, grad_out):
    """(dQ, dK, dV) of attention_reduce for the incoming gradient grad_out (B,M,C): the
    gradient TF's autodiff takes through attention_layer.py:35-42 (pn2_attn_reduce_grad)."""
    B, M, ns, C = (int(s) for s in K.shape)
    grad_out = device_tensor(grad_out, "grad_out", torch.float32)
    dQ = torch.empty_like(Q)
    dK = torch.empty_like(K)
    dV = torch.empty_like(V)
    check(lib().pn2_attn_reduce_grad(ptr(Q), ptr(K), ptr(V), ptr(grad_out), B, M, ns, C,
                                     ptr(dQ), ptr(dK), ptr(dV), stream_of(Q)),
          "attention_reduce_grad")
    return dQ, dK, dV


class _AttentionReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Q, K, V):
        ctx.save_for_backward(Q, K, V)
        return _attn_fwd(Q, K, V)

    @staticmethod
    def backward(ctx, grad_out):
        Q, K, V = ctx.saved_tensors
        return attention_reduce_grad(Q, K, V, grad_out.contiguous())


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
