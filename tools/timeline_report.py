#!/usr/bin/env python3
"""Summary of a bench.py --timeline file (a pipelined run traced with events, no profiler):
per step the host's wait for its buffer set and its enqueue, the SA1 sampler's GPU start and
end, and the end of each side lane, on one clock (GPU times relative to a base event recorded
at the host's time origin, so host and GPU times agree to within the event's latency).

    python tools/timeline_report.py <timeline.json> [--skip 10] [--lanes]"""
import argparse
import json
import statistics


def med(v):
    return statistics.median(v) if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--skip", type=int, default=10)
    ap.add_argument("--show", type=int, default=12)
    ap.add_argument("--lanes", action="store_true",
                    help="per side lane: median period between consecutive steps' ends and "
                         "median lag of its end after the SA1 sampler's end")
    a = ap.parse_args()
    d = json.load(open(a.path))
    st = [s for s in d["steps"] if "sampler_ms" in s and "lane_end_ms" in s]
    rows = []
    for s in st:
        h0, h1, h2 = s["host_ms"]
        g0, g1 = s["sampler_ms"]
        end = max(s["lane_end_ms"].values())
        rows.append({"k": s["k"], "wait": h1 - h0, "enq": h2 - h1, "queued": g0 - h2,
                     "sampler": g1 - g0, "side_after": end - g1, "latency": end - g0,
                     "enq_to_end": end - h1, "h1": h1, "g0": g0})
    body = rows[a.skip:]
    gaps = [b["g0"] - x["g0"] for x, b in zip(body, body[1:])]
    print(f"{len(rows)} steps; elapsed {d['elapsed_ms']:.2f} ms; medians (ms): host wait "
          f"{med([r['wait'] for r in body]):.3f}, enqueue {med([r['enq'] for r in body]):.3f}, "
          f"enqueue-end -> sampler start {med([r['queued'] for r in body]):.3f}, sampler "
          f"{med([r['sampler'] for r in body]):.3f}, sampler end -> last lane end "
          f"{med([r['side_after'] for r in body]):.3f}, sampler start -> last lane end "
          f"{med([r['latency'] for r in body]):.3f}, enqueue -> last lane end "
          f"{med([r['enq_to_end'] for r in body]):.3f}; sampler start to next sampler start "
          f"{med(gaps):.3f}")
    if a.lanes:
        sb = st[a.skip:]
        for L in sorted(sb[0]["lane_end_ms"], key=int):
            e = [s["lane_end_ms"][L] for s in sb]
            lag = [s["lane_end_ms"][L] - s["sampler_ms"][1] for s in sb]
            print(f"lane {L}: period {med([y - x for x, y in zip(e, e[1:])]):.3f} ms, end after "
                  f"the sampler's {med(lag):.3f} ms")
    print("first steps (ms from the start): k, host wait start, enqueue, sampler start, end, last lane end")
    for s, r in zip(st[:a.show], rows[:a.show]):
        print(f"  {r['k']:3d}  {s['host_ms'][0]:8.3f} {s['host_ms'][1]:8.3f}  "
              f"{s['sampler_ms'][0]:8.3f} {s['sampler_ms'][1]:8.3f}  "
              f"{max(s['lane_end_ms'].values()):8.3f}")


if __name__ == "__main__":
    main()
