#!/usr/bin/env python3
"""Host-side cost of the bench step with and without the forced RCCL world-1 bucketed all-reduce: perf_counter of
each phase (forward enqueue, loss, backward enqueue, all-reduce enqueue) over --steps steps without synchronising,
then a cProfile of the DP steps (top functions by own time).

usage: python tools/dp_host_prof.py [--steps 200] [--buckets layer|one]"""
import argparse
import cProfile
import os
import pstats
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--single", type=int, default=0)
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    from hgnn_amd.dp import LayerBucketAllReduce
    from models.gnns.model_mnb import GNN_lg
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).to(dev)
    params = list(model.parameters())
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.to(dev) for t in bench.make_batch(512, 1000)]
    X.requires_grad_(True)
    W.requires_grad_(True)
    crit = torch.nn.MSELoss()
    dp = LayerBucketAllReduce(model, force=True, single=bool(a.single))
    ph = {"zero": 0.0, "fwd": 0.0, "loss": 0.0, "bwd": 0.0, "dp": 0.0}

    def step(use_dp, t):
        t0 = time.perf_counter()
        for p in params:
            p.grad = None
        X.grad = None
        W.grad = None
        t1 = time.perf_counter()
        out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        t2 = time.perf_counter()
        loss = crit(out, T)
        t3 = time.perf_counter()
        loss.backward()
        t4 = time.perf_counter()
        if use_dp:
            dp()
        t5 = time.perf_counter()
        if t:
            for k, v in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4)):
                ph[k] += v

    for use_dp in (False, True):
        for _ in range(30):
            step(use_dp, False)
        torch.cuda.synchronize()
        for k in ph:
            ph[k] = 0.0
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step(use_dp, True)
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tw = time.perf_counter() - t0
        print(f"dp={use_dp}: host {th * 1e3 / a.steps:.3f} ms/step, wall {tw * 1e3 / a.steps:.3f} ms/step; phases (us/step): "
              + ", ".join(f"{k} {v * 1e6 / a.steps:.1f}" for k, v in ph.items()), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        step(True, False)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
