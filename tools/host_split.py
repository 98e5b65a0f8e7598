#!/usr/bin/env python3
"""Host time of the headline step split into the executor's C++ enqueue (the ctypes calls of
hgnn_net_forward / hgnn_net_backward_ex, timed by wrapping them) and everything else (Python autograd,
argument marshalling, torch's loss kernels).  GPU-bound steps leave the host idle part of the time, so
only the per-call times are meaningful, not their sum against the step.

usage: python tools/host_split.py [--steps 40]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    from hgnn_amd import _lib as L
    from models.gnns.model_mnb import GNN_lg
    lib = L.lib()
    acc = {}

    def wrap(name):
        f = getattr(lib, name)

        def timed(*args):
            t0 = time.perf_counter()
            r = f(*args)
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
            return r
        setattr(lib, name, timed)

    for n in ("hgnn_net_forward", "hgnn_net_backward_ex", "hgnn_net_backward", "hgnn_net_workspace_size"):
        if hasattr(lib, n):
            wrap(n)
    import hgnn_amd.net as N
    fb = N._NetFn.backward

    def timed_backward(ctx, dout):
        t0 = time.perf_counter()
        r = fb(ctx, dout)
        acc["_NetFn.backward (Python incl. the C++ call)"] = acc.get("_NetFn.backward (Python incl. the C++ call)", 0.0) + time.perf_counter() - t0
        return r
    N._NetFn.backward = staticmethod(timed_backward)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).to(dev)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.to(dev) for t in bench.make_batch(512, 1000, 1, 0)]
    X.requires_grad_(True)
    W.requires_grad_(True)
    crit = torch.nn.MSELoss()
    params = list(model.parameters())
    tb = [0.0, 0.0]

    def step():
        for p in params:
            p.grad = None
        X.grad = W.grad = None
        t0 = time.perf_counter()
        loss = crit(model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg), T)
        t1 = time.perf_counter()
        loss.backward()
        tb[0] += t1 - t0
        tb[1] += time.perf_counter() - t1

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    acc.clear()
    tb[0] = tb[1] = 0.0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    n = a.steps
    print(f"per step: wall {wall / n * 1e3:.3f} ms, host loop {host / n * 1e3:.3f} ms "
          f"(forward+loss {tb[0] / n * 1e3:.3f}, backward {tb[1] / n * 1e3:.3f})")
    for k, v in sorted(acc.items()):
        print(f"  {k}: {v / n * 1e3:.3f} ms per step (C++ enqueue inside the ctypes call)")


if __name__ == "__main__":
    main()
