// The native step executor (include/pn2plan.h): a recorded list of stream operations that
// one host call enqueues. Host code only; no kernels of its own.
//
// Why: once consecutive steps' samplers run concurrently (stack.Pipeline, sampler_lanes > 1),
// the GPU finishes a cfg2 step in less time than the Python loop took to enqueue it (11 tasks:
// ctypes argument checks for each sampler launch, one torch call per event record, wait and
// graph replay -- 0.30 ms of host time per step, tools/host_overhead.py). A plan does the same
// hipGraphLaunch / hipEventRecord / hipStreamWaitEvent / kernel launches from C++, with the
// sampler arguments validated once when recorded.
#include <new>
#include <vector>

#include "common.h"
#include "../../include/pn2plan.h"

namespace {

enum OpKind { kGraph, kRecord, kWait, kFpsChain, kKernel, kMemset };

struct Op {
  OpKind kind;
  hipStream_t stream;
  void* handle;  // hipGraphExec_t or hipEvent_t
  // kFpsChain
  const float* xyz;
  int B, N, nstages;
  int npoint[4];
  int32_t* idx[4];
  float* nx[4];
  void* grid0;  // stage 0's picks' grid (pn2_fps_chain_grid) or NULL
  size_t grid0_bytes;
  // kKernel / kMemset: a node of a captured graph, launched directly (pn2_plan_graph_direct);
  // the argument arrays belong to the graph, which the caller keeps alive
  hipKernelNodeParams kp;
  hipMemsetParams mp;
};

}  // namespace

struct pn2_plan {
  std::vector<Op> ops;
  int timed = -1;
};

namespace {

int run_op(const Op& o) {
  switch (o.kind) {
    case kGraph:
      return (int)hipGraphLaunch((hipGraphExec_t)o.handle, o.stream);
    case kRecord:
      return (int)hipEventRecord((hipEvent_t)o.handle, o.stream);
    case kWait:
      return (int)hipStreamWaitEvent(o.stream, (hipEvent_t)o.handle, 0);
    case kFpsChain:
      return pn2::fps_chain_launch(o.xyz, o.B, o.N, o.nstages, o.npoint, o.idx, o.nx, o.stream,
                                   false, o.grid0, o.grid0_bytes);
    case kKernel:
      return (int)hipLaunchKernel(o.kp.func, o.kp.gridDim, o.kp.blockDim, o.kp.kernelParams,
                                  o.kp.sharedMemBytes, o.stream);
    case kMemset:  // one row (pn2_plan_graph_direct accepts nothing else)
      if (o.mp.elementSize == 4)
        return (int)hipMemsetD32Async((hipDeviceptr_t)o.mp.dst, (int)o.mp.value, o.mp.width,
                                      o.stream);
      if (o.mp.elementSize == 2)
        return (int)hipMemsetD16Async((hipDeviceptr_t)o.mp.dst, (unsigned short)o.mp.value,
                                      o.mp.width, o.stream);
      return (int)hipMemsetAsync(o.mp.dst, (int)o.mp.value, o.mp.width, o.stream);
  }
  return PN2_EINVAL;
}

int launch(pn2_plan* p, void* ev0, void* ev1) {
  if (!p) return PN2_EINVAL;
  // a sampler fault stored by an earlier launch is reported here, once, before anything of
  // this step is enqueued: the plan's own sampler launches do not look at the fault word, so
  // a step is enqueued whole or not at all (its events then still describe the previous step)
  if (pn2::fps_take_fault()) return PN2_EFAULT;
  const int n = (int)p->ops.size();
  for (int i = 0; i < n; ++i) {
    const Op& o = p->ops[i];
    const bool timed = i == p->timed;
    if (timed && ev0) {
      const int rc = (int)hipEventRecord((hipEvent_t)ev0, o.stream);
      if (rc) return rc;
    }
    const int rc = run_op(o);
    if (rc) return rc;
    if (timed && ev1) {
      const int rc1 = (int)hipEventRecord((hipEvent_t)ev1, o.stream);
      if (rc1) return rc1;
    }
  }
  return PN2_OK;
}

int append(pn2_plan* p, const Op& o) {
  if (!p) return PN2_EINVAL;
  try {
    p->ops.push_back(o);
  } catch (const std::bad_alloc&) {
    return (int)hipErrorOutOfMemory;
  }
  return PN2_OK;
}

Op blank(OpKind k, hipStream_t s, void* h) {
  Op o{};
  o.kind = k;
  o.stream = s;
  o.handle = h;
  return o;
}

}  // namespace

extern "C" {

pn2_plan* pn2_plan_create(void) { return new (std::nothrow) pn2_plan(); }

void pn2_plan_destroy(pn2_plan* plan) { delete plan; }

int pn2_plan_graph(pn2_plan* plan, void* graph_exec, pn2_stream_t stream) {
  if (!graph_exec) return PN2_EINVAL;
  return append(plan, blank(kGraph, (hipStream_t)stream, graph_exec));
}

int pn2_plan_record(pn2_plan* plan, void* event, pn2_stream_t stream) {
  if (!event) return PN2_EINVAL;
  return append(plan, blank(kRecord, (hipStream_t)stream, event));
}

int pn2_plan_wait(pn2_plan* plan, pn2_stream_t stream, void* event) {
  if (!event) return PN2_EINVAL;
  return append(plan, blank(kWait, (hipStream_t)stream, event));
}

int pn2_plan_fps_chain(pn2_plan* plan, const float* xyz, int B, int N, int nstages,
                       const int* npoint, int32_t* const* idx, float* const* new_xyz,
                       pn2_stream_t stream) {
  return pn2_plan_fps_chain_grid(plan, xyz, B, N, nstages, npoint, idx, new_xyz, nullptr, 0,
                                 stream);
}

int pn2_plan_fps_chain_grid(pn2_plan* plan, const float* xyz, int B, int N, int nstages,
                            const int* npoint, int32_t* const* idx, float* const* new_xyz,
                            void* grid0, size_t grid0_bytes, pn2_stream_t stream) {
  const int rc = pn2::fps_chain_check(xyz, B, N, nstages, npoint, idx, new_xyz);
  if (rc != PN2_OK) return rc;
  if (grid0 && (!new_xyz[0] || grid0_bytes < pn2_grid_size(B, npoint[0]) ||
                ((uintptr_t)grid0 & 15)))
    return PN2_EINVAL;
  Op o = blank(kFpsChain, (hipStream_t)stream, nullptr);
  o.xyz = xyz;
  o.B = B;
  o.N = N;
  o.nstages = nstages;
  for (int i = 0; i < nstages; ++i) {
    o.npoint[i] = npoint[i];
    o.idx[i] = idx[i];
    o.nx[i] = new_xyz[i];
  }
  o.grid0 = grid0;
  o.grid0_bytes = grid0_bytes;
  return append(plan, o);
}

int pn2_plan_mark_timed(pn2_plan* plan) {
  if (!plan || plan->ops.empty()) return PN2_EINVAL;
  plan->timed = (int)plan->ops.size() - 1;
  return PN2_OK;
}

int pn2_plan_size(const pn2_plan* plan) { return plan ? (int)plan->ops.size() : PN2_EINVAL; }

int pn2_plan_launch(pn2_plan* plan) { return launch(plan, nullptr, nullptr); }

int pn2_plan_launch_timed(pn2_plan* plan, void* ev_start, void* ev_end) {
  return launch(plan, ev_start, ev_end);
}

// The nodes of a captured graph as direct launches, in dependency order: a single-kernel graph
// launch cost the host ~24 us per call against ~5 us for the kernel launch it wraps (rocprofv3
// --hip-runtime-trace, profiles/r5/start), and the side lanes' segments are one or two
// kernels each. Only a plain chain of kernel and memset nodes qualifies; anything else (a
// fork, an event or copy node) returns PN2_ENOTSUP with nothing appended, and the caller
// keeps the graph launch.
int pn2_plan_graph_direct(pn2_plan* plan, void* graph, pn2_stream_t stream) {
  if (!plan || !graph) return PN2_EINVAL;
  hipGraph_t g = (hipGraph_t)graph;
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return PN2_ENOTSUP;
  if (n == 0) return PN2_OK;
  std::vector<hipGraphNode_t> nodes(n);
  if (hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return PN2_ENOTSUP;
  // the chain: each node has at most one dependency, and no two nodes share one
  std::vector<int> prev(n, -1);
  std::vector<int> nxt(n, -1);
  for (size_t i = 0; i < n; ++i) {
    size_t nd = 0;
    if (hipGraphNodeGetDependencies(nodes[i], nullptr, &nd) != hipSuccess || nd > 1)
      return PN2_ENOTSUP;
    if (nd == 1) {
      hipGraphNode_t d = nullptr;
      if (hipGraphNodeGetDependencies(nodes[i], &d, &nd) != hipSuccess) return PN2_ENOTSUP;
      int j = -1;
      for (size_t k = 0; k < n; ++k)
        if (nodes[k] == d) j = (int)k;
      if (j < 0 || nxt[j] >= 0) return PN2_ENOTSUP;
      nxt[j] = (int)i;
      prev[i] = j;
    }
  }
  int head = -1;
  for (size_t i = 0; i < n; ++i) {
    if (prev[i] < 0) {
      if (head >= 0) return PN2_ENOTSUP;  // two roots
      head = (int)i;
    }
  }
  std::vector<Op> ops;
  size_t seen = 0;
  for (int i = head; i >= 0; i = nxt[i]) {
    if (++seen > n) return PN2_ENOTSUP;
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess) return PN2_ENOTSUP;
    Op o = blank(kKernel, (hipStream_t)stream, nullptr);
    if (t == hipGraphNodeTypeKernel) {
      if (hipGraphKernelNodeGetParams(nodes[i], &o.kp) != hipSuccess || o.kp.extra ||
          !o.kp.func)
        return PN2_ENOTSUP;
      // hipLaunchKernel takes a registered host stub only; a node captured from
      // hipModuleLaunchKernel holds a hipFunction_t instead, and node attributes (cooperative
      // launch, ...) would be dropped: such nodes keep the graph launch
      hipFuncAttributes fa;
      if (hipFuncGetAttributes(&fa, o.kp.func) != hipSuccess) return PN2_ENOTSUP;
      hipKernelNodeAttrValue av{};
      if (hipGraphKernelNodeGetAttribute(nodes[i], hipKernelNodeAttributeCooperative, &av) ==
              hipSuccess && av.cooperative)
        return PN2_ENOTSUP;
    } else if (t == hipGraphNodeTypeMemset) {
      o.kind = kMemset;
      if (hipGraphMemsetNodeGetParams(nodes[i], &o.mp) != hipSuccess || o.mp.height > 1 ||
          (o.mp.elementSize != 1 && o.mp.elementSize != 2 && o.mp.elementSize != 4))
        return PN2_ENOTSUP;
    } else if (t != hipGraphNodeTypeEmpty) {
      return PN2_ENOTSUP;
    } else {
      continue;
    }
    ops.push_back(o);
  }
  if (seen != n) return PN2_ENOTSUP;  // (a cycle or an unreachable node)
  for (const Op& o : ops) {
    const int rc = append(plan, o);
    if (rc != PN2_OK) return rc;
  }
  return PN2_OK;
}

}  // extern "C"
