"""Shared-MLP layers of pointnet2_tensorflow/utils/tf_util.py, inference mode, on gfx950.

tf_util.conv2d / conv1d with a 1x1 kernel (tf_util.py:52-117, :120-185) are per-point dense
layers: conv, bias_add, batch_norm (tf.contrib.layers.batch_norm, :512-531), activation. In
inference mode (is_training=False) the batch norm is the per-channel affine map
    bn(x) = (x - moving_mean) * gamma / sqrt(moving_variance + eps) + beta,  eps = 1e-3
so a layer is  y = act((x W + b) * scale + shift). Layers are packed once (pn2_mlp_pack) into
the matrix-core operand layout of csrc/mlp.hip and then run fused with the grouping / the
interpolation before them and the pooling after them (pointnet_util.pointnet_sa_module,
pointnet_fp_module) or on plain rows (conv2d / conv1d here).

Parameters live in a ParamStore keyed by the reference's TF variable names
("layer1/conv0/weights", ".../biases", ".../bn/gamma", ".../bn/beta", ".../bn/moving_mean",
".../bn/moving_variance"), so a TF checkpoint's variables, exported to a dict of arrays, load
unchanged. Missing variables are created with the reference's initialisers (xavier weights,
zero biases, gamma 1, beta 0, moving mean 0, moving variance 1; tf_util.py:24-49).
"""
import math

import numpy as np
import torch

from ._lib import (PN2_MLP_MAX_LAYERS, PN2_MLP_RELU, InvalidArgumentError, MlpLayer, check,
                   device_tensor, lib, ptr, stream_of)

BN_EPSILON = 1e-3  # tf.contrib.layers.batch_norm's default epsilon


class ParamStore(dict):
    """TF variable name -> float32 tensor, with the reference's initialisers for misses."""

    def __init__(self, *args, seed=0, device="cuda", **kw):
        super().__init__()
        self.seed = seed
        self.device = device
        self._packed = {}
        for k, v in dict(*args, **kw).items():
            self[k] = v

    def __setitem__(self, name, value):
        # checkpoint arrays (numpy or torch) are kept as float32 CPU tensors
        super().__setitem__(name, torch.as_tensor(value, dtype=torch.float32).detach().cpu())

    def _init(self, name, shape, kind):
        if kind == "xavier":  # tf.contrib.layers.xavier_initializer(): glorot uniform
            fan_in = int(np.prod(shape[:-1]))
            fan_out = int(np.prod(shape[:-2])) * int(shape[-1])
            lim = math.sqrt(6.0 / (fan_in + fan_out))
            # deterministic per variable name
            g = np.random.default_rng([self.seed] + [ord(c) for c in name])
            return g.uniform(-lim, lim, size=shape).astype(np.float32)
        value = {"zeros": 0.0, "ones": 1.0}[kind]
        return np.full(shape, value, dtype=np.float32)

    def get(self, name, shape, kind):
        if name not in self:
            self[name] = torch.from_numpy(self._init(name, shape, kind))
        t = self[name]
        if tuple(t.shape) != tuple(shape):
            t = t.reshape(shape)
        return t

    def conv(self, scope, cin, cout, bn=True):
        """The variables tf_util.conv2d(..., scope) creates (kernel [1,1,cin,cout])."""
        p = {"weights": self.get(f"{scope}/weights", (1, 1, cin, cout), "xavier").reshape(
            cin, cout), "biases": self.get(f"{scope}/biases", (cout,), "zeros")}
        if bn:
            p["gamma"] = self.get(f"{scope}/bn/gamma", (cout,), "ones")
            p["beta"] = self.get(f"{scope}/bn/beta", (cout,), "zeros")
            p["moving_mean"] = self.get(f"{scope}/bn/moving_mean", (cout,), "zeros")
            p["moving_variance"] = self.get(f"{scope}/bn/moving_variance", (cout,), "ones")
        return p

    def dense(self, scope, cin, cout):
        """The variables of a tf.layers.Dense(cout) built under `scope` (glorot-uniform kernel,
        zero bias: the Keras defaults)."""
        return {"weights": self.get(f"{scope}/kernel", (cin, cout), "xavier"),
                "biases": self.get(f"{scope}/bias", (cout,), "zeros")}

    def bn(self, scope, c):
        """The variables of a standalone batch_norm_template(scope) (tf_util.py:512-531)."""
        return {"gamma": self.get(f"{scope}/gamma", (c,), "ones"),
                "beta": self.get(f"{scope}/beta", (c,), "zeros"),
                "moving_mean": self.get(f"{scope}/moving_mean", (c,), "zeros"),
                "moving_variance": self.get(f"{scope}/moving_variance", (c,), "ones")}

    def invalidate(self):
        """Drop packed copies (call after changing parameters in place)."""
        self._packed.clear()


_default_store = None


def default_store():
    """The process-wide store (the analogue of TF's default graph variables)."""
    global _default_store
    if _default_store is None:
        _default_store = ParamStore()
    return _default_store


class PackedLayer:
    """One conv layer in pn2_mlp_pack's layout (device buffer) + its struct pn2_mlp_layer."""

    def __init__(self, weights, biases=None, gamma=None, beta=None, moving_mean=None,
                 moving_variance=None, relu=True, eps=BN_EPSILON, device="cuda"):
        w = torch.as_tensor(weights, dtype=torch.float32)
        if w.dim() == 4:  # TF conv2d kernel [1,1,cin,cout]
            w = w.reshape(w.shape[-2], w.shape[-1])
        if w.dim() != 2:
            raise InvalidArgumentError("weights must be (cin, cout) or [1, 1, cin, cout]")
        self.cin, self.cout = int(w.shape[0]), int(w.shape[1])
        self.relu = bool(relu)
        dev = torch.device(device)
        w = w.to(dev).contiguous()
        b = None if biases is None else torch.as_tensor(biases, dtype=torch.float32).to(dev)
        scale = shift = None
        if gamma is not None:
            # inference batch norm (tf_util.py:512-531): (x - mean) * gamma / sqrt(var + eps) + beta
            g = torch.as_tensor(gamma, dtype=torch.float64)
            var = torch.as_tensor(moving_variance, dtype=torch.float64)
            mean = torch.as_tensor(moving_mean, dtype=torch.float64)
            bt = torch.as_tensor(beta, dtype=torch.float64)
            s64 = g / torch.sqrt(var + eps)
            scale = s64.to(torch.float32).to(dev).contiguous()
            shift = (bt - mean * s64).to(torch.float32).to(dev).contiguous()
        nbytes = int(lib().pn2_mlp_packed_size(self.cin, self.cout))
        self.buf = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev)
        check(lib().pn2_mlp_pack(ptr(w), ptr(b), ptr(scale), ptr(shift), self.cin, self.cout,
                                 ptr(self.buf), nbytes, stream_of(self.buf)), "mlp_pack")
        self.scale, self.shift, self.bias = scale, shift, b  # kept for the training path

    def struct(self):
        return MlpLayer(self.buf.data_ptr(), self.cin, self.cout,
                        PN2_MLP_RELU if self.relu else 0)


class SharedMLP:
    """A chain of PackedLayers run as one fused kernel (at most PN2_MLP_MAX_LAYERS)."""

    def __init__(self, layers):
        if not 1 <= len(layers) <= PN2_MLP_MAX_LAYERS:
            raise InvalidArgumentError(f"1..{PN2_MLP_MAX_LAYERS} layers per fused MLP")
        for a, b in zip(layers, layers[1:]):
            if a.cout != b.cin:
                raise InvalidArgumentError("consecutive layers must chain cout -> cin")
        self.layers = list(layers)
        self.cin, self.cout = layers[0].cin, layers[-1].cout
        self._table = (MlpLayer * len(layers))(*[l.struct() for l in layers])

    def table(self):
        return self._table, len(self.layers)

    def __call__(self, x):
        """Per-point MLP over the last axis: x (..., cin) -> (..., cout) (pn2_shared_mlp)."""
        x = device_tensor(x, "inputs", torch.float32)
        if int(x.shape[-1]) != self.cin:
            raise InvalidArgumentError(f"inputs have {int(x.shape[-1])} channels, the MLP "
                                       f"expects {self.cin}")
        rows = x.numel() // self.cin
        out = torch.empty(tuple(x.shape[:-1]) + (self.cout,), dtype=torch.float32,
                          device=x.device)
        tab, n = self.table()
        check(lib().pn2_shared_mlp(ptr(x), rows, self.cin, n, tab, ptr(out), stream_of(x)),
              "shared_mlp")
        return out


def packed_mlp(store, scopes, cin, widths, bn=True, relu=True):
    """SharedMLP over the store's variables for conv scopes `scopes` (one per width), cached
    per scope tuple. `relu` applies to every layer (tf_util.conv2d's activation_fn)."""
    key = (tuple(scopes), cin, tuple(widths), bn, relu)
    hit = store._packed.get(key)
    if hit is not None:
        return hit
    layers, c = [], cin
    for scope, w in zip(scopes, widths):
        p = store.conv(scope, c, w, bn=bn)
        layers.append(PackedLayer(p["weights"], p["biases"], p.get("gamma"), p.get("beta"),
                                  p.get("moving_mean"), p.get("moving_variance"), relu=relu,
                                  device=store.device))
        c = w
    mlp = SharedMLP(layers)
    store._packed[key] = mlp
    return mlp


def packed_dense(store, scope, cin, cout):
    """SharedMLP of one tf.layers.Dense (no activation) over the store's variables, cached."""
    key = ("dense", scope, cin, cout)
    hit = store._packed.get(key)
    if hit is None:
        p = store.dense(scope, cin, cout)
        hit = SharedMLP([PackedLayer(p["weights"], p["biases"], relu=False, device=store.device)])
        store._packed[key] = hit
    return hit


def bn_affine(store, scope, c, device):
    """Inference batch norm as (scale, shift) device tensors: x * scale + shift."""
    key = ("bn", scope, c)
    hit = store._packed.get(key)
    if hit is None:
        p = store.bn(scope, c)
        s64 = p["gamma"].double() / torch.sqrt(p["moving_variance"].double() + BN_EPSILON)
        shift = p["beta"].double() - p["moving_mean"].double() * s64
        hit = (s64.float().to(device), shift.float().to(device))
        store._packed[key] = hit
    return hit


def conv2d(inputs, num_output_channels, kernel_size, scope, stride=[1, 1], padding='SAME',
           data_format='NHWC', use_xavier=True, stddev=1e-3, weight_decay=None,
           activation_fn=torch.relu, bn=False, bn_decay=None, is_training=None, params=None):
    """tf_util.conv2d (tf_util.py:120-185) for the 1x1 kernels PointNet++ uses, NHWC,
    inference mode. Extra keyword `params`: the ParamStore (default: default_store())."""
    if list(kernel_size) != [1, 1] or list(stride) != [1, 1] or data_format != 'NHWC':
        raise NotImplementedError("pn2hip's conv2d is the 1x1 NHWC shared MLP of PointNet++")
    if is_training:
        raise NotImplementedError("conv2d: the fused layer is inference-mode batch norm; "
                                  "use pointnet_util.*(is_training=True) for training")
    if activation_fn not in (None, torch.relu, torch.nn.functional.relu):
        raise NotImplementedError("conv2d: activation must be relu or None")
    store = params if params is not None else default_store()
    mlp = packed_mlp(store, [scope], int(inputs.shape[-1]), [num_output_channels], bn=bn,
                     relu=activation_fn is not None)
    return mlp(inputs)


def conv1d(inputs, num_output_channels, kernel_size, scope, stride=1, padding='SAME',
           data_format='NHWC', use_xavier=True, stddev=1e-3, weight_decay=None,
           activation_fn=torch.relu, bn=False, bn_decay=None, is_training=None, params=None):
    """tf_util.conv1d (tf_util.py:52-117) with kernel 1 (the segmentation heads' fc layers)."""
    if kernel_size != 1 or stride != 1:
        raise NotImplementedError("pn2hip's conv1d is the kernel-1 per-point layer")
    return conv2d(inputs, num_output_channels, [1, 1], scope, data_format=data_format,
                  activation_fn=activation_fn, bn=bn, bn_decay=bn_decay,
                  is_training=is_training, params=params)


def mlp_torch(x, layers, is_training=False, bn_decay=None):
    """The same layers composed from differentiable torch ops (the training path; batch norm
    with batch statistics over every axis but the channel axis when is_training, as
    tf.contrib.layers.batch_norm does, moving averages updated with decay bn_decay or 0.9)."""
    for L in layers:
        p = L.params
        y = x @ p["weights"].to(x.device)
        if p.get("biases") is not None:
            y = y + p["biases"].to(x.device)
        if p.get("gamma") is not None:
            gamma, beta = p["gamma"].to(x.device), p["beta"].to(x.device)
            if is_training:
                dims = tuple(range(y.dim() - 1))
                mean = y.mean(dim=dims)
                var = y.var(dim=dims, unbiased=False)
                decay = 0.9 if bn_decay is None else float(bn_decay)
                with torch.no_grad():
                    p["moving_mean"].mul_(decay).add_((1 - decay) * mean.detach().cpu())
                    p["moving_variance"].mul_(decay).add_((1 - decay) * var.detach().cpu())
            else:
                mean = p["moving_mean"].to(x.device)
                var = p["moving_variance"].to(x.device)
            y = (y - mean) * (gamma / torch.sqrt(var + BN_EPSILON)) + beta
        x = torch.relu(y) if L.relu else y
    return x


class TorchLayer:
    """A conv layer's raw variables for mlp_torch."""

    def __init__(self, params, relu=True):
        self.params, self.relu = params, relu


def torch_layers(store, scopes, cin, widths, bn=True, relu=True):
    layers, c = [], cin
    for scope, w in zip(scopes, widths):
        layers.append(TorchLayer(store.conv(scope, c, w, bn=bn), relu=relu))
        c = w
    return layers
