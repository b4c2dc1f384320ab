"""Python owner of a native step plan (include/pn2plan.h, csrc/plan.hip).

A plan records a step's stream operations once -- hipGraph launches of the captured side-lane
tasks (or, when a task's graph is a plain chain of kernels, those kernels as direct launches),
the direct sampler launches, event records and cross-stream waits -- and enqueues all of them
with ONE call into libpn2hip.so per step (stack.GraphStep.replay_plan). The handles it
records are borrowed from torch (CUDAGraph.raw_cuda_graph(_exec)(), Event.cuda_event,
Stream.cuda_stream) and the sampler buffers from the step: the plan keeps references to those
objects so they outlive it.
"""
import ctypes

import torch

from . import tf_sampling
from ._lib import PN2_ENOTSUP, InvalidArgumentError, check, lib


def _event_handle(ev):
    """hipEvent_t of a torch event; torch creates the event at its first record, so an event
    that was never recorded is recorded once on the current stream first."""
    if ev.cuda_event == 0:
        ev.record()
    return ev.cuda_event


class Plan:
    def __init__(self):
        self._lib = lib()
        self.h = self._lib.pn2_plan_create()
        if not self.h:
            raise MemoryError("pn2_plan_create")
        self._keep = []  # graphs, events, streams, tensors and ctypes arrays the plan points at
        self.launches = {"direct": 0, "graph": 0}  # side segments by how they are enqueued

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            self._lib.pn2_plan_destroy(h)

    def __len__(self):
        return self._lib.pn2_plan_size(self.h)

    def graph(self, g, stream):
        """Launch the captured torch CUDAGraph `g` on `stream`."""
        self._keep += [g, stream]
        check(self._lib.pn2_plan_graph(self.h, g.raw_cuda_graph_exec(), stream.cuda_stream),
              "pn2_plan_graph")
        self.launches["graph"] += 1

    def graph_direct(self, g, stream):
        """The kernels of the captured torch CUDAGraph `g` (made with keep_graph=True) as direct
        launches on `stream` (pn2_plan_graph_direct); a graph that is not a plain chain of
        kernel / memset nodes is launched as a graph instead (pn2_plan_graph). Returns True
        when the kernels went in directly."""
        self._keep += [g, stream]
        rc = self._lib.pn2_plan_graph_direct(self.h, g.raw_cuda_graph(), stream.cuda_stream)
        if rc == PN2_ENOTSUP:
            self.graph(g, stream)
            return False
        check(rc, "pn2_plan_graph_direct")
        self.launches["direct"] += 1
        return True

    def record(self, ev, stream):
        self._keep += [ev, stream]
        check(self._lib.pn2_plan_record(self.h, _event_handle(ev), stream.cuda_stream),
              "pn2_plan_record")

    def wait(self, stream, ev):
        self._keep += [ev, stream]
        check(self._lib.pn2_plan_wait(self.h, stream.cuda_stream, _event_handle(ev)),
              "pn2_plan_wait")

    def fps_chain(self, npoints, xyz, outs, stream, grid0=None):
        """pn2_fps_chain(npoints) of `xyz` into the fixed buffers `outs` [(idx, new_xyz)];
        with grid0 (tf_sampling.farthest_point_sample_chain's) pn2_fps_chain_grid."""
        npoints = [int(m) for m in npoints]
        if (xyz.dim() != 3 or xyz.shape[2] != 3 or xyz.dtype != torch.float32
                or not xyz.is_contiguous() or len(outs) != len(npoints)):
            raise InvalidArgumentError("plan fps_chain: xyz must be contiguous float32 (B,N,3), "
                                       "one (idx, new_xyz) pair per stage")
        B, N = int(xyz.shape[0]), int(xyz.shape[1])
        for (i_, x_), m in zip(outs, npoints):
            if (i_.shape != (B, m) or i_.dtype != torch.int32 or x_.shape != (B, m, 3)
                    or x_.dtype != torch.float32 or not i_.is_contiguous()
                    or not x_.is_contiguous()):
                raise InvalidArgumentError("plan fps_chain: out tensors must be contiguous "
                                           "int32 (B,m) / float32 (B,m,3)")
        k = len(npoints)
        arr_i = (ctypes.c_int * k)(*npoints)
        arr_idx = (ctypes.c_void_p * k)(*[o[0].data_ptr() for o in outs])
        arr_nx = (ctypes.c_void_p * k)(*[o[1].data_ptr() for o in outs])
        self._keep += [xyz, outs, stream, arr_i, arr_idx, arr_nx, grid0]
        if grid0 is not None:
            tf_sampling.check_grid0(grid0, outs[0][1])
            check(self._lib.pn2_plan_fps_chain_grid(
                self.h, xyz.data_ptr(), B, N, k, ctypes.addressof(arr_i),
                ctypes.addressof(arr_idx), ctypes.addressof(arr_nx), grid0.buf.data_ptr(),
                grid0.nbytes, stream.cuda_stream), "pn2_plan_fps_chain_grid")
            return
        check(self._lib.pn2_plan_fps_chain(self.h, xyz.data_ptr(), B, N, k,
                                           ctypes.addressof(arr_i), ctypes.addressof(arr_idx),
                                           ctypes.addressof(arr_nx), stream.cuda_stream),
              "pn2_plan_fps_chain")

    def mark_timed(self):
        check(self._lib.pn2_plan_mark_timed(self.h), "pn2_plan_mark_timed")

    def launch(self, events=None):
        """Enqueue the plan; `events` = (start, end) torch events bracket the timed operation."""
        if events is None:
            check(self._lib.pn2_plan_launch(self.h), "pn2_plan_launch")
        else:
            check(self._lib.pn2_plan_launch_timed(self.h, _event_handle(events[0]),
                                                  _event_handle(events[1])),
                  "pn2_plan_launch")
