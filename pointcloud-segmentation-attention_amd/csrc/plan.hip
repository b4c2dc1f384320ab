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

enum OpKind { kGraph, kRecord, kWait, kFpsChain };

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
                                   false);
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
  const int rc = pn2::fps_chain_check(xyz, B, N, nstages, npoint, idx, new_xyz);
  if (rc != PN2_OK) return rc;
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

// CU-partitioned streams (hipExtStreamCreateWithCUMask): `mask` holds one bit per CU (bit i of
// word i / 32 = CU i). Returns 0 and the new stream, or the HIP error.
int pn2_stream_create_cu_mask(const uint32_t* mask, int words, pn2_stream_t* stream) {
  if (!mask || words <= 0 || !stream) return PN2_EINVAL;
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (e != hipSuccess) return (int)e;
  *stream = (pn2_stream_t)s;
  return PN2_OK;
}

int pn2_stream_destroy(pn2_stream_t stream) {
  const hipError_t e = hipStreamDestroy((hipStream_t)stream);
  return e == hipSuccess ? PN2_OK : (int)e;
}

}  // extern "C"
