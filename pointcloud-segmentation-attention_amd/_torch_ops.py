"""torch.ops.pn2.* — the C ABI registered as PyTorch operators (csrc/torch_ops.cpp, built into
libpn2torch.so next to libpn2hip.so): TORCH_LIBRARY schemas with the reference's op names and
argument order, HIP kernels that launch on the current HIP stream, Meta kernels for fake
tensors / torch.compile. This module loads the library and registers autograd for the ops the
reference registers gradients for, w.r.t. the points only (tf_sampling.py:44-48 GatherPoint,
tf_grouping.py:42-46 GroupPoint, tf_interpolate.py:29-34 ThreeInterpolate), plus the attention
reduction (TF autodiff through attention_layer.py:35-42, all of Q, K, V).

The mirror modules (tf_sampling, tf_grouping, tf_interpolate, attention_layer) call these ops
for every reference-signature call; the pn2hip alias package re-exports them as pn2hip.ops.
"""
import os

import torch

from ._lib import _HERE, InvalidArgumentError

TORCH_LIB_PATH = os.environ.get("PN2TORCH_LIB") or os.path.join(_HERE, "libpn2torch.so")
_loaded = False


def ops():
    """torch.ops.pn2, loading libpn2torch.so on first use (raises if it was not built)."""
    global _loaded
    if not _loaded:
        if not os.path.exists(TORCH_LIB_PATH):
            raise RuntimeError(
                f"{TORCH_LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ "
                "as g; g.build()'`. pn2hip has no CPU fallback.")
        torch.ops.load_library(TORCH_LIB_PATH)
        _register_autograd()
        _loaded = True
    return torch.ops.pn2


def call(name, *args):
    """torch.ops.pn2.<name>(*args) for the mirror modules: the op's reference-text ValueError
    (TORCH_CHECK_VALUE, or PN2_EINVAL from the C ABI) surfaces as InvalidArgumentError, the
    mirror's stand-in for tf.errors.InvalidArgumentError (a ValueError too)."""
    try:
        return getattr(ops(), name)(*args)
    except InvalidArgumentError:
        raise
    except ValueError as e:
        raise InvalidArgumentError(str(e).splitlines()[0]) from e


def _register_autograd():
    reg = torch.library.register_autograd

    def save_all(ctx, inputs, output):
        ctx.save_for_backward(*inputs)

    def gather_bwd(ctx, grad):
        inp, idx = ctx.saved_tensors
        return torch.ops.pn2.gather_point_grad(inp, idx, grad.contiguous()), None

    def group_bwd(ctx, grad):
        points, idx = ctx.saved_tensors
        return torch.ops.pn2.group_point_grad(points, idx, grad.contiguous()), None

    def interp_bwd(ctx, grad):
        points, idx, weight = ctx.saved_tensors
        return torch.ops.pn2.three_interpolate_grad(points, idx, weight, grad.contiguous()), \
            None, None

    def attn_bwd(ctx, grad):
        Q, K, V = ctx.saved_tensors
        return tuple(torch.ops.pn2.attn_reduce_grad(Q, K, V, grad.contiguous()))

    reg("pn2::gather_point", gather_bwd, setup_context=save_all)
    reg("pn2::group_point", group_bwd, setup_context=save_all)
    reg("pn2::three_interpolate", interp_bwd, setup_context=save_all)
    reg("pn2::attn_reduce", attn_bwd, setup_context=save_all)
