#!/usr/bin/env python3
"""What the gradient all-reduce costs a step, piece by piece, in an RCCL ("nccl") group of world size 1 on one GPU:
the bench step (GNN_lg config 2) without DP, with the per-layer buckets, with one bucket, one bucket without the
running statistics, a bare all_reduce of the flat buffer after the step, and a bare all_reduce of 4 bytes.  Wall and
host (enqueue) ms per step over --steps steps each, variants interleaved over --reps rounds.

usage: python tools/dp_ab.py [--steps 100] [--reps 3]"""
import argparse
import os
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
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    from hgnn_amd import dp as DP
    from models.gnns.model_mnb import GNN_lg
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).to(dev)
    params = list(model.parameters())
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.to(dev) for t in bench.make_batch(512, 1000)]
    X.requires_grad_(True)
    W.requires_grad_(True)
    crit = torch.nn.MSELoss()
    flat = torch.zeros(sum(p.numel() for p in params), device=dev)
    tiny = torch.zeros(1, device=dev)

    def compute():
        for p in params:
            p.grad = None
        X.grad = None
        W.grad = None
        crit(model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg), T).backward()

    variants = {
        "no_dp": lambda: None,
        "layer_buckets": ("dp", dict(force=True)),
        "one_bucket": ("dp", dict(force=True, single=True)),
        "one_bucket_no_running": ("dp", dict(force=True, single=True, sync_running=False)),
        "bare_allreduce_flat": lambda: dist.all_reduce(flat, op=dist.ReduceOp.AVG),
        "bare_allreduce_4B": lambda: dist.all_reduce(tiny, op=dist.ReduceOp.AVG),
    }
    res = {k: [] for k in variants}
    for rep in range(a.reps):
        for name, v in variants.items():
            obj = None
            if isinstance(v, tuple):
                obj = DP.LayerBucketAllReduce(model, **v[1])
                fn = obj
            else:
                fn = v
            for _ in range(20):
                compute()
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                compute()
                fn()
            th = time.perf_counter() - t0
            torch.cuda.synchronize()
            tw = time.perf_counter() - t0
            res[name].append((tw * 1e3 / a.steps, th * 1e3 / a.steps))
            if obj is not None:
                obj.detach()
                for p in params:
                    p.grad = None
    for name, r in res.items():
        print(f"{name:24s} wall " + " ".join(f"{w:.3f}" for w, _ in r) + "  host " + " ".join(f"{h:.3f}" for _, h in r),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
