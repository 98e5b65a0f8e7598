"""Host enqueue time of ONE headline step issued into an idle GPU (synchronised before), against the GPU
time of that step -- unlike a back-to-back loop, whose enqueue blocks once the launch queue is full and so
reads as the GPU's time.  Median over --steps steps; forward / backward split of the enqueue.

usage: python tools/host_step.py [--steps 30]"""
import argparse
import os
import statistics as st
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
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
    rec = []
    for i in range(a.steps + 5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for p in params:
            p.grad = None
        X.grad = None
        W.grad = None
        out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        loss = crit(out, T)
        t1 = time.perf_counter()
        loss.backward()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if i >= 5:
            rec.append((t1 - t0, t2 - t1, t2 - t0, t3 - t0))
    m = [st.median(x[k] for x in rec) * 1e3 for k in range(4)]
    print(f"one step into an idle GPU (median of {len(rec)}): host enqueue {m[2]:.3f} ms (forward {m[0]:.3f}, "
          f"backward {m[1]:.3f}); enqueue start -> GPU complete {m[3]:.3f} ms", flush=True)
    # the same, back to back (steady state): wall per step
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        for p in params:
            p.grad = None
        X.grad = None
        W.grad = None
        crit(model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg), T).backward()
    torch.cuda.synchronize()
    print(f"back to back: {(time.perf_counter() - t0) / a.steps * 1e3:.3f} ms per step", flush=True)


if __name__ == "__main__":
    main()
