"""Is the headline step host-bound?  Times the host's enqueue of K eager steps (until the loop
returns, before any synchronisation) against the GPU-complete time, the forward / backward
host time per step, and a HIP-graph replay of the same step.

usage: python tools/host_bound.py [--steps 20]
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
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from models.gnns.model_mnb import GNN_lg
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).to(dev)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.to(dev) for t in bench.make_batch(512, 1000, 1, 0)]
    X.requires_grad_(True)
    W.requires_grad_(True)
    crit = torch.nn.MSELoss()
    params = list(model.parameters())
    tf = [0.0]
    tb = [0.0]

    def step():
        for p in params:
            p.grad = None
        X.grad = None
        W.grad = None
        t0 = time.perf_counter()
        out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        loss = crit(out, T)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        tf[0] += t1 - t0
        tb[0] += t2 - t1

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    tf[0] = tb[0] = 0.0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    n = a.steps
    print(f"eager: host enqueue {t_enq / n * 1e3:.3f} ms/step (forward {tf[0] / n * 1e3:.3f}, backward "
          f"{tb[0] / n * 1e3:.3f}), GPU-complete {t_all / n * 1e3:.3f} ms/step")
    # graph replay of the same step
    keep = {}

    def gstep():
        for p in params:
            p.grad = None
        X.grad = None
        W.grad = None
        out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        crit(out, T).backward()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            gstep()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        gstep()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"graph: host enqueue {t_enq / n * 1e3:.3f} ms/step, GPU-complete {t_all / n * 1e3:.3f} ms/step")
    del keep


if __name__ == "__main__":
    main()
