"""pn2hip — importable name of the MI355X PointNet++ hot path.

The implementation lives in the directory `pointcloud-segmentation-attention_amd/` (the
name the build layout prescribes; its hyphens make it unimportable with a plain statement).
This package re-exports it so that model code imports by name, as the reference's models do
(pointnet2_tensorflow/utils/pointnet_util.py:10-12, attention_points/models/
pointnet2_sem_seg_attention.py:6-8):

    import pn2hip
    from pn2hip.tf_sampling import farthest_point_sample, gather_point
    from pn2hip.tf_grouping import query_ball_point, group_point, knn_point
    from pn2hip.tf_interpolate import three_nn, three_interpolate
    from pn2hip import ops            # torch.ops.pn2.* under the reference's op names

pn2hip.install_reference_names() additionally registers the reference's own top-level
module names (tf_sampling, tf_grouping, tf_interpolate, pointnet_util, tf_util,
attention_layer), so a model file that does `from tf_sampling import farthest_point_sample`
after its sys.path edits runs on these kernels unchanged.
"""
import importlib
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

_impl = importlib.import_module("pointcloud-segmentation-attention_amd")

MODULES = ("tf_sampling", "tf_grouping", "tf_interpolate", "pointnet_util", "tf_util",
           "attention_layer", "data_transformation", "complete_scene_loader", "grid", "stack",
           "shard", "synth")
for _name in MODULES:
    _mod = getattr(_impl, _name)
    globals()[_name] = _mod
    sys.modules[f"{__name__}.{_name}"] = _mod

lib = _impl.lib
LIB_PATH = _impl.LIB_PATH
InvalidArgumentError = _impl.InvalidArgumentError
Pn2RuntimeError = _impl.Pn2RuntimeError



def __getattr__(name):
    """`pn2hip.ops` loads lazily: importing pn2hip must not require libpn2torch.so (the C ABI
    and ctypes users do not need it); the first use of `ops` raises if it is missing."""
    if name == "ops":
        return importlib.import_module(f"{__name__}.ops")
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


REFERENCE_NAMES = ("tf_sampling", "tf_grouping", "tf_interpolate", "pointnet_util", "tf_util",
                   "attention_layer")


def install_reference_names():
    """Make `import tf_sampling` (and the other reference module names) resolve to these
    modules. Returns the names installed; an already-imported module of the same name is
    left alone and not returned."""
    done = []
    for name in REFERENCE_NAMES:
        if name not in sys.modules:
            sys.modules[name] = globals()[name]
            done.append(name)
    return done


__all__ = list(MODULES) + ["ops", "lib", "LIB_PATH", "InvalidArgumentError", "Pn2RuntimeError",
                           "install_reference_names"]
