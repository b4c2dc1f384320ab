#!/usr/bin/env python3
"""Per-step critical path of a pipelined bench run, from a rocprofv3 --kernel-trace CSV.

    python tools/critical_path.py <kernel_trace.csv> [--config cfg2] [--sets 9] [--lanes 3]

Kernels are assigned to steps by their order: each step launches every kernel of its task
list once (stack.Step), on a fixed queue, and a queue runs its kernels in order, so the j-th
occurrence of a kernel name on a queue belongs to the j-th step that used that queue (the SA1
samplers rotate over `lanes` queues). For every kernel the report knows the edges that can
hold its start (stack.py's task dependencies for the SSG step, SURVEY §8 order SA -> FP,
pointnet_util.py:90-159,206-236):
  queue   the previous kernel on the same queue was still running
  dep     a producer on another lane (the sampler, the grid, the later-sampler chain)
  host    the host had not enqueued it: the SA1 sampler of step k can only be enqueued once
          step k - sets has finished (the buffer set is reused), so its start is bounded by
          that step's last end (plus the host's own enqueue time)
  slack   nothing visible held it (dispatch / launch latency)
and walks back from the step's last kernel along the binding edges. The summary counts which
edge ended each step and the median time on each edge, and the per-queue busy fractions."""
import argparse
import csv
import statistics
from collections import defaultdict

# kernel-name fragments -> task (SSG geometric step, stack.Step._tasks_ssg)
TASKS = [("fps_hotcull", "fps1"), ("fps_v9", "fps1"), ("fps_chain", "fps234"),
         ("ball_group_layers", "sa234"), ("fp_fused_layers", "fp123"),
         ("ball_query_grid", "sa1"), ("three_nn_grid", "nn4"), ("fp_fused_kernel", "fp4"),
         ("fp_grid_fused", "fp4"),
         ("grid_build", "grid"), ("group_concat", "grp"), ("attn", "att")]
# task -> producers on other lanes (grid builds are matched on their own queue)
DEPS = {"sa1": ["fps1"], "nn4": ["fps1"], "fp4": ["fps1"], "fps234": ["fps1"],
        "sa234": ["fps234"], "fp123": ["fps234"], "grp": ["fps1"]}


def task_of(name):
    for frag, t in TASKS:
        if frag in name:
            return t
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--sets", type=int, default=9)
    ap.add_argument("--lanes", type=int, default=3)
    ap.add_argument("--skip", type=int, default=20, help="steps skipped at the start (warm-up)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    ks = []
    for r in rows:
        t = task_of(r["Kernel_Name"])
        if t:
            ks.append({"task": t, "q": r.get("Queue_Id", "?"), "s": int(r["Start_Timestamp"]),
                       "e": int(r["End_Timestamp"]), "name": r["Kernel_Name"]})
    # step numbers: SA1 samplers in start order; every other (task, queue) stream in order,
    # aligned so that its first occurrence after the first sampler is that sampler's step
    samplers = [k for k in ks if k["task"] == "fps1"]
    for j, k in enumerate(samplers):
        k["step"] = j
    first = samplers[0]["s"]
    streams = defaultdict(list)
    for k in ks:
        if k["task"] != "fps1":
            streams[(k["task"], k["q"])].append(k)
    # a task that runs on one queue for every step: its j-th launch is step j; a task spread
    # over several queues (per-set streams) is matched by start order over all of them
    by_task = defaultdict(list)
    for (t, q), lst in streams.items():
        by_task[t].append(lst)
    for t, lsts in by_task.items():
        if t == "grid":
            continue
        allk = sorted([k for lst in lsts for k in lst], key=lambda k: k["s"])
        allk = [k for k in allk if k["e"] >= first]
        for j, k in enumerate(allk):
            k["step"] = j
    # a grid build belongs to the step of the next kernel on its queue (SA1's ball-query grid
    # before that step's SA1 grouping, FP4's known grid before its three_nn)
    byq0 = defaultdict(list)
    for k in ks:
        byq0[k["q"]].append(k)
    for q, lst in byq0.items():
        lst.sort(key=lambda k: k["s"])
        for a_, b_ in zip(lst, lst[1:]):
            if a_["task"] == "grid" and "step" in b_:
                a_["step"] = b_["step"]
    steps = defaultdict(dict)
    for k in ks:
        if "step" in k:
            steps[k["step"]].setdefault(k["task"] + ("@" + k["q"] if k["task"] == "grid" else ""), k)
    nsteps = len(samplers)
    qprev = {}
    for lst in streams.values():
        pass
    byq = defaultdict(list)
    for k in ks:
        byq[k["q"]].append(k)
    for q, lst in byq.items():
        lst.sort(key=lambda k: k["s"])
        for p, k in zip(lst, lst[1:]):
            qprev[id(k)] = p
    qprev_s = {}
    for q, lst in byq.items():
        for p, k in zip(lst, lst[1:]):
            qprev_s[id(k)] = p

    def last_end(j):
        st = steps.get(j)
        return max(k["e"] for k in st.values()) if st else None

    edge_count = defaultdict(int)
    edge_time = defaultdict(list)
    lat = []
    lines = []
    for j in range(a.skip, nsteps - a.sets - 1):
        st = steps[j]
        if "fps1" not in st:
            continue
        end_k = max(st.values(), key=lambda k: k["e"])
        L = (end_k["e"] - st["fps1"]["s"]) / 1e3
        lat.append(L)
        path, k, first_edge = [], end_k, None
        for _ in range(12):
            cands = []
            p = qprev_s.get(id(k))
            if p is not None:
                cands.append(("queue", p["e"], p))
            for d in DEPS.get(k["task"], []):
                dk = st.get(d) if k.get("step") == j else steps.get(k["step"], {}).get(d)
                if dk is not None:
                    cands.append(("dep", dk["e"], dk))
            if k["task"] == "fps1" and k["step"] - a.sets >= 0:
                le = last_end(k["step"] - a.sets)
                if le is not None:
                    cands.append(("host", le, None))
            if not cands:
                break
            kind, t, src = max(cands, key=lambda c: c[1])
            gap = (k["s"] - t) / 1e3
            if gap > 5.0 or t > k["s"]:
                # the binding producer ended well before this kernel started (or after it:
                # an edge that cannot hold it): dispatch / launch latency
                if t <= k["s"]:
                    kind = "slack" if gap > 5.0 else kind
            path.append((k["task"], kind, round((k["e"] - k["s"]) / 1e3, 1), round(gap, 1)))
            if first_edge is None:
                first_edge = kind
            edge_time[kind].append(max(gap, 0.0))
            if kind in ("slack", "host") or src is None:
                break
            k = src
        edge_count[path[-1][1] if path else "none"] += 1
        if len(lines) < 12:
            lines.append(f"step {j}: latency {L:.1f} us, ends with {end_k['task']} on q{end_k['q']}: "
                         + " <- ".join(f"{t}[{d}us, {kind} +{g}us]" for t, kind, d, g in path))
    out = []
    span = (samplers[-1]["s"] - samplers[a.skip]["s"]) / 1e3 / max(1, nsteps - 1 - a.skip)
    out.append(f"{nsteps} steps; SA1 start to SA1 start {span:.1f} us per step; step latency "
               f"(SA1 start -> last kernel end) median {statistics.median(lat):.1f} us, "
               f"min {min(lat):.1f}, max {max(lat):.1f}")
    out.append("where the walk back from each step's last kernel stopped (the edge that holds "
               "the chain's start): " + ", ".join(f"{k} {v}" for k, v in sorted(edge_count.items())))
    out.append("median wait on each edge kind (us): " + ", ".join(
        f"{k} {statistics.median(v):.1f} (n={len(v)})" for k, v in sorted(edge_time.items())))
    # per-task start delay after its producers / queue predecessor
    dly = defaultdict(list)
    for j in range(a.skip, nsteps - a.sets - 1):
        for t, k in steps[j].items():
            p = qprev_s.get(id(k))
            ready = [p["e"]] if p is not None else []
            for d in DEPS.get(k["task"], []):
                if d in steps[j]:
                    ready.append(steps[j][d]["e"])
            if ready:
                dly[t].append((k["s"] - max(ready)) / 1e3)
    out.append("start delay after the last of (queue predecessor, producers), median us: "
               + ", ".join(f"{t} {statistics.median(v):.1f}" for t, v in sorted(dly.items())))
    dur = defaultdict(list)
    for j in range(a.skip, nsteps - a.sets - 1):
        for t, k in steps[j].items():
            dur[t].append((k["e"] - k["s"]) / 1e3)
    out.append("kernel duration median us: " + ", ".join(
        f"{t} {statistics.median(v):.1f}" for t, v in sorted(dur.items())))
    out += lines
    txt = "\n".join(out)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
