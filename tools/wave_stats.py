#!/usr/bin/env python3
"""Per-wave view of the headline step's launches from the in-kernel stamps (HGNN_TIMER_STAMPS): for every
timed launch of the last of --steps steps, its wave count, span, when its waves started (entry percentiles
from the launch's first entry: a late tail means waves waited for a free slot) and how long they ran
(duration percentiles), and the mean number of waves live over the span.  --split K also splits the waves
of the launches of class --split-class into K equal consecutive groups (e.g. the two operator families of
the extraction grid (bs, 2), whose waves are numbered block-major).

usage: python tools/wave_stats.py [--steps 3] [--split 2 --split-class struct]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def describe(tag, w):
    w = np.asarray([x for x in w if x[0] >= 0 and x[1] >= 0])
    if len(w) == 0:
        return f"{tag:28s} no stamps"
    e, x = w[:, 0], w[:, 1]
    t0 = e.min()
    d = x - e
    span = x.max() - t0
    pe = np.percentile(e - t0, [50, 90, 100])
    pd = np.percentile(d, [10, 50, 90, 100])
    return (f"{tag:28s} waves {len(w):6d} span {span:7.1f} | entry p50 {pe[0]:6.1f} p90 {pe[1]:6.1f} max {pe[2]:6.1f}"
            f" | dur p10 {pd[0]:6.1f} p50 {pd[1]:6.1f} p90 {pd[2]:6.1f} max {pd[3]:6.1f} | live {d.sum() / max(span, 1e-9):7.1f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--split", type=int, default=2)
    ap.add_argument("--split-class", default="struct")
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
    n = 200 * a.steps
    tm = KernelTimer(n, range(RF.N_CLASSES), mode=TIMER_STAMPS, stamp_words=4 * 1024 * 1024 * a.steps)
    with tm:
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    L = tm.launches(n)
    per_step = len(L) // a.steps
    first = per_step * (a.steps - 1)
    print(f"{per_step} timed launches per step; last step's launches (times in us)")
    for i in range(first, first + per_step):
        c = L[i][0]
        w = tm.waves(i)
        print(f"{i - first:3d} " + describe(f"{RF.NAMES[c]} s{L[i][3]}", w), flush=True)
        if RF.NAMES[c] == a.split_class and a.split > 1 and len(w) >= a.split:
            g = len(w) // a.split
            for k in range(a.split):
                print("    " + describe(f"  group {k}", w[k * g:(k + 1) * g]))
    tm.close()


if __name__ == "__main__":
    main()
