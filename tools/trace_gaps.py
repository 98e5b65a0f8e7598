#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace (CSV) of bench.py: steps delimited by k_plan launches; for the
last --steps complete steps: span, union-busy, per-stream busy, and the largest idle gaps of the GPU (no kernel on
any stream) with the kernels on either side.

usage: python tools/trace_gaps.py gpurun_out/tr_plain/run_kernel_trace.csv [--steps 5] [--top 12]"""
import argparse
import csv
import statistics as st


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").replace("hgnn::", "").split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    k = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Stream_Id", ""))
               for r in rows)
    starts = [s for s, e, n, q in k if n.startswith("k_plan")]
    # the last `steps` complete steps before the final k_plan (the profiled tail after the timed loop differs)
    bounds = starts[-(a.steps + 2):-1]
    spans, busys, gaps_all = [], [], []
    per_stream = {}
    for i in range(len(bounds) - 1):
        t0, t1 = bounds[i], bounds[i + 1]
        win = [x for x in k if t0 <= x[0] < t1]
        busy = 0
        cs, ce = win[0][0], win[0][1]
        prev = win[0]
        gaps = []
        for x in win[1:]:
            if x[0] > ce:
                busy += ce - cs
                gaps.append((x[0] - ce, prev[2], x[2]))
                cs, ce = x[0], x[1]
            elif x[1] > ce:
                ce = x[1]
            if x[1] >= ce:
                prev = x
        busy += ce - cs
        spans.append((t1 - t0) / 1e3)
        busys.append(busy / 1e3)
        gaps_all += gaps
        for q in {x[3] for x in win}:
            iv = [(s, e) for s, e, n, qq in win if qq == q]
            per_stream.setdefault(q, []).append((len(iv), sum(e - s for s, e in iv) / 1e3))
    print(f"{len(spans)} steps: span {st.median(spans):.1f} us (median), union busy {st.median(busys):.1f} us, "
          f"idle {st.median(spans) - st.median(busys):.1f} us")
    for q, v in sorted(per_stream.items()):
        print(f"  stream {q}: {st.median(x[0] for x in v):.0f} launches, kernel time {st.median(x[1] for x in v):.1f} us")
    n = max(1, len(spans))
    tot = {}
    for g, p, nx in gaps_all:
        key = (p, nx)
        tot[key] = tot.get(key, [0.0, 0])
        tot[key][0] += g / 1e3
        tot[key][1] += 1
    print(f"idle gaps of the whole GPU, summed per (before, after) pair, per step:")
    for (p, nx), (t, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"  {t / n:7.1f} us  x{c / n:4.1f}  {p}  ->  {nx}")


if __name__ == "__main__":
    main()
