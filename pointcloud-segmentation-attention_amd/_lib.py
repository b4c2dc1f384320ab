"""ctypes binding of libpn2hip.so — the C ABI declared in include/pn2hip.h.

The product path is the HIP library: if it is missing, every op raises; there is no CPU
fallback. `torch` is imported first on purpose: torch ships its own libamdhip64.so (SONAME
libamdhip64.so.7) and libpn2hip.so links the same SONAME, so loading it after torch binds it
to torch's HIP runtime — one runtime per process, torch's streams and allocations are valid
inside the library.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# PN2HIP_LIB: an alternative build of the same ABI (A/B measurements in tools/)
LIB_PATH = os.environ.get("PN2HIP_LIB") or os.path.join(_HERE, "libpn2hip.so")

PN2_EINVAL = -22
PN2_BQ_MAX_RADII = 3  # include/pn2hip.h
PN2_EFAULT = -14
PN2_FAULT_FPS_POLL = 1
PN2_ENOTSUP = -95  # include/pn2hip.h
PN2_FPS_AUTO, PN2_FPS_BLOCKSCAN = 0, 1
PN2_USE_XYZ = 1
PN2_XYZ_LAST = 2
POOL_MODES = {"max": 0, "avg": 1, "weighted_avg": 2, "max_and_avg": 3}
PN2_POOL_NONE = -1
PN2_MLP_MAX_LAYERS = 6
PN2_MLP_RELU = 1


class InvalidArgumentError(ValueError):
    """Raised where the reference's OP_REQUIRES raises tf.errors.InvalidArgumentError."""


class Pn2RuntimeError(RuntimeError):
    """A HIP launch error reported by the C ABI."""


_P, _I, _F, _S = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
_LL = ctypes.c_longlong


class MlpLayer(ctypes.Structure):
    """struct pn2_mlp_layer (include/pn2hip.h)."""
    _fields_ = [("packed", ctypes.c_void_p), ("cin", ctypes.c_int), ("cout", ctypes.c_int),
                ("flags", ctypes.c_int)]

class SaLayer(ctypes.Structure):
    """struct pn2_sa_layer (include/pn2hip.h)."""
    _fields_ = [("xyz", ctypes.c_void_p), ("points", ctypes.c_void_p),
                ("new_xyz", ctypes.c_void_p), ("N", ctypes.c_int), ("C", ctypes.c_int),
                ("M", ctypes.c_int), ("nsample", ctypes.c_int), ("radius", ctypes.c_float),
                ("flags", ctypes.c_int), ("idx", ctypes.c_void_p), ("pts_cnt", ctypes.c_void_p),
                ("grouped_xyz", ctypes.c_void_p), ("new_points", ctypes.c_void_p)]


PN2_SA_MAX_LAYERS = 4


class FpLayer(ctypes.Structure):
    """struct pn2_fp_layer (include/pn2hip.h)."""
    _fields_ = [("xyz1", ctypes.c_void_p), ("xyz2", ctypes.c_void_p),
                ("points1", ctypes.c_void_p), ("points2", ctypes.c_void_p), ("C1", ctypes.c_int),
                ("C2", ctypes.c_int), ("n", ctypes.c_int), ("m", ctypes.c_int),
                ("out", ctypes.c_void_p)]


PN2_FP_MAX_LAYERS = 4


class AttnLayer(ctypes.Structure):
    """struct pn2_attn_layer (include/pn2hip.h)."""
    _fields_ = [("Q", ctypes.c_void_p), ("K", ctypes.c_void_p), ("V", ctypes.c_void_p),
                ("M", ctypes.c_int), ("ns", ctypes.c_int), ("C", ctypes.c_int),
                ("out", ctypes.c_void_p)]


PN2_ATTN_MAX_LAYERS = 4

# name -> (restype, argtypes); mirrors include/pn2hip.h and include/pn2plan.h (tests/test_capi.py checks the header)
SIGNATURES = {
    "pn2_version": (ctypes.c_char_p, []),
    "pn2_strerror": (ctypes.c_char_p, [_I]),
    "pn2_copy_f4": (_I, [_P, _P, _S, _I, _P]),
    "pn2_fps": (_I, [_P, _I, _I, _I, _P, _P]),
    "pn2_fps_gather": (_I, [_P, _I, _I, _I, _P, _P, _P]),
    "pn2_fps_max_points": (_I, []),
    "pn2_fps_gather_sched": (_I, [_P, _I, _I, _I, _P, _P, _I, _P]),
    "pn2_fault_status": (_I, [_I]),
    "pn2_prob_sample_workspace_size": (_S, [_I, _I]),
    "pn2_prob_sample": (_I, [_P, _P, _I, _I, _I, _P, _S, _P, _P]),
    "pn2_fps_workspace_size": (_S, [_I, _I]),
    "pn2_fps_chain": (_I, [_P, _I, _I, _I, _P, _P, _P, _P]),
    "pn2_fps_chain_grid": (_I, [_P, _I, _I, _I, _P, _P, _P, _P, _S, _P]),
    "pn2_fps_ws": (_I, [_P, _I, _I, _I, _P, _P, _P, _S, _P]),
    "pn2_gather_point": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "pn2_gather_point_grad": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "pn2_ball_query": (_I, [_P, _P, _I, _I, _I, _F, _I, _P, _P, _P]),
    "pn2_ball_threshold": (_F, [_F]),
    "pn2_select_top_k": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "pn2_select_top_k_workspace_size": (_S, [_I, _I, _I]),
    "pn2_knn_point": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "pn2_grid_size": (_S, [_I, _I]),
    "pn2_grid_build": (_I, [_P, _I, _I, _F, _P, _S, _P]),
    "pn2_ball_query_grid": (_I, [_P, _P, _I, _I, _I, _F, _I, _P, _P, _P]),
    "pn2_ball_group_xyz_grid": (_I, [_P, _P, _P, _I, _I, _I, _F, _I, _P, _P, _P, _P]),
    "pn2_ball_group_grid": (_I, [_P, _P, _P, _I, _I, _P, _I, _I, _I, _F, _I, _P, _P, _P, _P]),
    "pn2_ball_group_xyz_grid_radii": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "pn2_three_nn_grid": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "pn2_fp_apply": (_I, [_P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _P, _P]),
    "pn2_fp_grid_fused": (_I, [_P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "pn2_fp_grid_fused_known": (_I, [_P, _P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _P, _P, _P,
                                     _P]),
    "pn2_group_point": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "pn2_group_point_grad": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "pn2_group_concat": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "pn2_ball_group_layers": (_I, [_P, _I, _I, _P]),
    "pn2_sample_and_group": (_I, [_P, _P, _I, _I, _I, _I, _F, _I, _I, _P, _P, _P, _P, _P, _P,
                                  _P]),
    "pn2_three_nn": (_I, [_P, _P, _I, _I, _I, _P, _P, _P]),
    "pn2_three_interpolate": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "pn2_three_interpolate_grad": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "pn2_idw_weights": (_I, [_P, _I, _I, _P, _P]),
    "pn2cpu_three_nn": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "pn2cpu_three_interpolate": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    "pn2cpu_three_interpolate_grad": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    "pn2_fp_fused_layers": (_I, [_P, _I, _I, _P]),
    "pn2_fp_fused": (_I, [_P, _P, _P, _I, _P, _I, _I, _I, _I, _P, _P]),
    "pn2_attn_reduce": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P]),
    "pn2_attn_reduce_layers": (_I, [_P, _I, _I, _P]),
    "pn2_attn_reduce_grad": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "pn2_group_pool": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "pn2_mlp_packed_size": (_S, [_I, _I]),
    "pn2_mlp_pack": (_I, [_P, _P, _P, _P, _I, _I, _P, _S, _P]),
    "pn2_group_mlp": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P, _P]),
    "pn2_group_mlp_attention": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P,
                                     _I, _P, _P]),
    "pn2_fp_mlp": (_I, [_P, _P, _P, _I, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "pn2_shared_mlp": (_I, [_P, _LL, _I, _I, _P, _P, _P]),
    "pn2_scene_workspace_size": (_S, [_I]),
    "pn2_scene_bbox": (_I, [_P, _I, _P, _P, _S, _P]),
    "pn2_crop_workspace_size": (_S, [_I, _I, _I]),
    "pn2_crop_sample": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _I, _P, _I, _P, _I, _P, _S, _P, _P,
                             _P, _P, _P, _P]),
    "pn2_subvolume_slices": (_I, [_I]),
    "pn2_subvolume_select": (_I, [_P, _I, _P, _I, ctypes.c_double, _P, _P, _P, _P]),
    "pn2_gather_rows": (_I, [_P, _LL, _I, _P, _LL, _P, _P]),
    # include/pn2plan.h: the native step executor
    "pn2_plan_create": (_P, []),
    "pn2_plan_destroy": (None, [_P]),
    "pn2_plan_graph": (_I, [_P, _P, _P]),
    "pn2_plan_record": (_I, [_P, _P, _P]),
    "pn2_plan_wait": (_I, [_P, _P, _P]),
    "pn2_plan_fps_chain": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P]),
    "pn2_plan_fps_chain_grid": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P, _S, _P]),
    "pn2_plan_mark_timed": (_I, [_P]),
    "pn2_plan_size": (_I, [_P]),
    "pn2_plan_launch": (_I, [_P]),
    "pn2_plan_launch_timed": (_I, [_P, _P, _P]),
    "pn2_plan_graph_direct": (_I, [_P, _P, _P]),
}

_lib = None


def lib():
    """The loaded libpn2hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (make -C pointcloud-segmentation-attention_amd/csrc). "
                "pn2hip has no CPU fallback.")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc, op):
    if rc == 0:
        return
    if rc == PN2_EINVAL:
        raise InvalidArgumentError(f"{op}: invalid argument")
    if rc == PN2_EFAULT:
        raise Pn2RuntimeError(f"{op}: an earlier sampler launch reported a device fault "
                              "(its indices are not trustworthy; see pn2_fault_status)")
    msg = lib().pn2_strerror(rc)
    raise Pn2RuntimeError(f"{op}: HIP error {rc}: {msg.decode() if msg else '?'}")


def check_device_faults(device=None):
    """Synchronise `device` and raise if a sampler launch stored a device fault code
    (include/pn2hip.h pn2_fault_status); clears the code."""
    torch.cuda.synchronize(device)
    code = lib().pn2_fault_status(1)
    if code:
        raise Pn2RuntimeError(f"device fault {code} reported by a sampler launch "
                              "(PN2_FAULT_FPS_POLL = 1: a cold wave's wait timed out)")


def stream_of(t):
    """hipStream_t handle of torch's current stream on t's device."""
    return torch.cuda.current_stream(t.device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def device_tensor(t, name, dtype):
    """Validate an op input: a GPU tensor of the reference dtype, made contiguous."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor, got {type(t).__name__}")
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{name} is on {t.device}: pn2hip ops run on the MI355X only (no CPU fallback)")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    return t.contiguous()
