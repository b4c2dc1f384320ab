/* pn2plan.h — the native step executor of libpn2hip.so.
 *
 * A plan is a fixed list of stream operations recorded once and enqueued by ONE host call per
 * step: hipGraph launches (the captured side-lane tasks), direct sampler launches
 * (pn2_fps_chain), event records and cross-stream waits. It replaces the per-task Python
 * enqueue loop of stack.Step.run(), whose host cost (~0.2-0.3 ms per geometric step: ctypes
 * argument checks, one torch call per event, wait and graph replay) set the pace once the
 * samplers of consecutive steps ran concurrently. There is no reference
 * counterpart: the reference enqueues one TF op at a time from its session.
 *
 * All handles are borrowed: the caller keeps the graph executables, events, streams and
 * device buffers alive (and unchanged) for as long as the plan is launched. Nothing here
 * allocates device memory or synchronises.
 */
#ifndef PN2PLAN_H
#define PN2PLAN_H

#include <stdint.h>

#include "pn2hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pn2_plan pn2_plan;

/* a new, empty plan (NULL if out of host memory) */
pn2_plan* pn2_plan_create(void);
void pn2_plan_destroy(pn2_plan* plan);

/* append: launch the instantiated graph `graph_exec` (hipGraphExec_t) on `stream` */
int pn2_plan_graph(pn2_plan* plan, void* graph_exec, pn2_stream_t stream);
/* append: record `event` (hipEvent_t) on `stream` */
int pn2_plan_record(pn2_plan* plan, void* event, pn2_stream_t stream);
/* append: make `stream` wait for the last record of `event` */
int pn2_plan_wait(pn2_plan* plan, pn2_stream_t stream, void* event);
/* append: pn2_fps_chain(xyz, B, N, nstages, npoint, idx, new_xyz, stream) with these
 * arguments (the arrays are copied; the buffers they point to are borrowed). The arguments
 * are validated now, exactly as pn2_fps_chain validates them: PN2_EINVAL and nothing appended
 * on error. */
int pn2_plan_fps_chain(pn2_plan* plan, const float* xyz, int B, int N, int nstages,
                       const int* npoint, int32_t* const* idx, float* const* new_xyz,
                       pn2_stream_t stream);
/* append: pn2_fps_chain_grid (the same, plus stage 0's picks' grid into grid0) */
int pn2_plan_fps_chain_grid(pn2_plan* plan, const float* xyz, int B, int N, int nstages,
                            const int* npoint, int32_t* const* idx, float* const* new_xyz,
                            void* grid0, size_t grid0_bytes, pn2_stream_t stream);
/* mark the operation appended last as the timed one: pn2_plan_launch_timed brackets it with
 * its two events (recorded on that operation's stream) */
int pn2_plan_mark_timed(pn2_plan* plan);
/* number of operations in the plan */
int pn2_plan_size(const pn2_plan* plan);

/* enqueue every operation in order; returns 0, or PN2_EFAULT (and enqueues nothing) when an
 * earlier sampler launch stored a fault (the fault word is read and cleared once, before the
 * first operation; the plan's own sampler launches do not read it, so a step is never left
 * half enqueued by a fault), or the first failing operation's status (a hipError_t or
 * PN2_EINVAL) and stops */
int pn2_plan_launch(pn2_plan* plan);
/* the same with the marked operation bracketed by records of ev_start / ev_end (either may
 * be NULL) */
int pn2_plan_launch_timed(pn2_plan* plan, void* ev_start, void* ev_end);

/* append: the nodes of the captured graph `graph` (hipGraph_t, not instantiated: torch
 * CUDAGraph(keep_graph=True).raw_cuda_graph()) as direct kernel launches / memsets on
 * `stream`, in dependency order -- what launching the graph would enqueue, without the graph
 * launch's host cost (~24 vs ~5 us for a one-kernel graph, profiles/r5/start). Only a plain chain
 * of kernel and memset nodes qualifies: anything else returns PN2_ENOTSUP and appends nothing
 * (then use pn2_plan_graph). The graph's argument storage is borrowed: keep the graph alive and
 * unchanged while the plan is launched. */
int pn2_plan_graph_direct(pn2_plan* plan, void* graph, pn2_stream_t stream);

/* PN2_ENOTSUP (pn2hip.h), from pn2_plan_graph_direct: not a plain chain of kernel / memset nodes */

#ifdef __cplusplus
}
#endif

#endif /* PN2PLAN_H */
