#!/usr/bin/env python3
"""Unperturbed in-step timeline of the headline step from in-kernel stamps (HGNN_TIMER_STAMPS): every
executor kernel of --steps steps stamps s_memrealtime per wave at entry and exit, nothing is added to the
streams.  Prints, for the last step, every launch in enqueue order (class, stream, start, end, duration,
idle gap on its stream before it), then per-class totals and per-stream busy / idle over all timed steps.
Work outside the executor (torch's MSE loss, memsets, event waits) shows up as gaps.

usage: python tools/timeline.py [--steps 10] [--d 64] [--json out.json]"""
import argparse
import json
import os
import statistics as st
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from hgnn_amd import roofline as RF
    from hgnn_amd.net import TIMER_STAMPS, KernelTimer
    from models.gnns.model_mnb import GNN_lg
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = GNN_lg(0, a.d, 5, 5, 1, 1, 2).to(dev)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.to(dev) for t in bench.make_batch(512, 1000, 1, 0)]
    X.requires_grad_(True)
    W.requires_grad_(True)
    crit = torch.nn.MSELoss()
    params = list(model.parameters())

    def step():
        for p in params:
            p.grad = None
        X.grad = None
        W.grad = None
        crit(model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg), T).backward()

    for _ in range(30):
        step()
    torch.cuda.synchronize()
    wave_bound = 2 * (X.shape[0] * (X.shape[2] + XL.shape[2])) + 16384
    n = 200 * a.steps
    # a step's launches fit 2 words per wave; bound the buffer by the largest launch times the launches
    tm = KernelTimer(n, range(RF.N_CLASSES), mode=TIMER_STAMPS, stamp_words=4 * 1024 * 1024 * a.steps)
    with tm:
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    L = tm.launches(n)
    tm.close()
    per_step = len(L) // a.steps
    steps = [L[i * per_step:(i + 1) * per_step] for i in range(a.steps)]
    last = steps[-1]
    t0 = min(x[1] for x in last)
    print(f"{per_step} timed launches per step")
    print(f"{'#':>3} {'class':10s} {'strm':>4} {'start':>8} {'end':>8} {'dur':>7} {'gap':>7}")
    prev_end = {}
    for i, (c, e0, e1, sq) in enumerate(last):
        gap = e0 - prev_end[sq] if sq in prev_end else float("nan")
        prev_end[sq] = e1
        print(f"{i:3d} {RF.NAMES[c]:10s} {sq:4d} {e0 - t0:8.1f} {e1 - t0:8.1f} {e1 - e0:7.1f} {gap:7.1f}")
    # per-class totals and per-stream busy / gaps over all timed steps (median per step)
    cls_tot = {}
    busy = {}
    gaps = {}
    span = []
    for s_ in steps:
        tot = {}
        b = {}
        g = {}
        pe = {}
        for c, e0, e1, sq in s_:
            tot[c] = tot.get(c, 0.0) + (e1 - e0)
            b[sq] = b.get(sq, 0.0) + (e1 - e0)
            if sq in pe:
                g[sq] = g.get(sq, 0.0) + max(0.0, e0 - pe[sq])
            pe[sq] = e1
        for c, v in tot.items():
            cls_tot.setdefault(c, []).append(v)
        for q, v in b.items():
            busy.setdefault(q, []).append(v)
        for q, v in g.items():
            gaps.setdefault(q, []).append(v)
        span.append(max(x[2] for x in s_) - min(x[1] for x in s_))
    print(f"\nstep span (first entry -> last exit of the step's timed kernels), median: {st.median(span):.1f} us")
    for q in sorted(busy):
        print(f"stream {q}: kernels {st.median(busy[q]):.1f} us, idle gaps between them {st.median(gaps.get(q, [0])):.1f} us")
    print("per class (us per step, median):")
    for c, v in sorted(cls_tot.items(), key=lambda kv: -st.median(kv[1])):
        print(f"  {RF.NAMES[c]:10s} {st.median(v):8.1f}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump({"launches": L, "per_step": per_step, "names": RF.NAMES}, fh)


if __name__ == "__main__":
    main()
