#!/usr/bin/env python3
"""Throughput of the other BASELINE.json configurations on one GPU (not the bench line).

bench.py measures the headline metric (config 2).  This script times the
remaining configurations of BASELINE.json on the same executor, each as
graphs/s of a training pass (forward + loss + backward) with inputs resident
in HBM, and the LG-GNN forward alone (the north star's "batched LG-GNN
forward" roofline):

  cfg1   GNN_simple(0, 2, 20, 5, 1, 1), 32 SBM N=50 graphs per step
  cfg2f  GNN_lg d=64 order 2 L=5, 512 QM9-shape graphs, forward only (train-mode BN)
  cfg2o1 / cfg2o3  the same step with orders 1 / 3
  cfg2csr the config-2 step on a CsrBatch from the native batcher (no dense W -> no dense dW)
  cfg2train / cfg2train_csr  the whole train_with_mnb step on the device (TrainStep: + MSE + Adamax)
  cfg3   CCN_1D(5, 1, 2, 2), 256 QM9-shape graphs (A + I), per-graph MSE summed
  cfg3_pergraph  the same 256 graphs one at a time as scripts/train_ccn.py runs them (forward,
         MSE, backward, Adamax step per graph)
  cfg4   GNN_lg d=128 order 2 L=5, 512 QM9-shape graphs (one GPU's share of 4096)
  cfg5   CCN_2D(5, 1, 2, 2), 64 SBM N=200 graphs (A + I)
  cfg5_pergraph  the same 64 graphs one at a time (forward, MSE, backward, Adamax step per graph)
  cfg5q / cfg5qg  CCN_2D(5, 1, 2, 2), 256 QM9-shape graphs batched (eager / replayed from a HIP graph)
  cfg5q_pergraph  the same 256 graphs one at a time (the reference driver's CCN_2D call pattern)
  (HGNN_CCN_SMALL=0 puts the QM9-size CCN batches on the general path for an A/B)

Prints one JSON line per configuration.  Usage:
  python tools/bench_configs.py [--only cfg3,cfg5] [--steps 20] [--warmup 5]
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "hgnn-2_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def lg_batch(bs, seed, sbm_n=None):
    import hgnn_amd.datagen as dg
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    graphs = dg.sbm_dataset(bs, n=sbm_n, seed=seed) if sbm_n else dg.qm9_shape_dataset(bs, seed=seed)
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    return [t.cuda() for t in prepare_batch(data, 0, 1)]


def ccn_batch(graphs):
    bs = len(graphs)
    nmax = max(X.shape[0] for X, _, _ in graphs)
    f = graphs[0][0].shape[1]
    X = torch.zeros(bs, nmax, f)
    A = torch.zeros(bs, nmax, nmax)
    T = torch.zeros(bs, 1)
    nb = torch.zeros(bs, dtype=torch.int64)
    for b, (x, a, t) in enumerate(graphs):
        n = x.shape[0]
        X[b, :n] = x
        A[b, :n, :n] = a + torch.eye(n)  # scripts/train_ccn.py:36
        T[b, 0] = t[0]
        nb[b] = n
    return X.cuda(), A.cuda(), T.cuda(), nb.cuda()


def graphed(step, warmup=3):
    """Capture one call of step() (forward + loss + backward: every executor launch, the side
    stream's fork/join included) in a HIP graph; returns its replay."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(warmup):
            step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    return g.replay


def timeit(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def run_lg(name, desc, d, order, bs, steps, warmup, backward=True):
    from models.gnns.model_mnb import GNN_lg
    torch.manual_seed(0)
    model = GNN_lg(0, d, 5, 5, 1, 1, order).cuda()
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = lg_batch(bs, 1000)
    crit = torch.nn.MSELoss()
    if backward:
        X.requires_grad_(True)
        W.requires_grad_(True)

    def step():
        if backward:
            model.zero_grad(set_to_none=True)
            X.grad = W.grad = None
            crit(model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg), T).backward()
        else:
            with torch.no_grad():
                model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)

    sec = timeit(step, steps, warmup)
    return dict(config=name, workload=desc, graphs_per_step=bs, ms_per_step=round(sec * 1e3, 4),
                value=round(bs / sec, 2), unit="graphs/s", dtype="fp32",
                nodes=int(Nb.sum()), edge_slots=int(Eb.sum()))


def run_lg_csr(steps, warmup, bs=512):
    """Config 2 on the native batcher's CsrBatch: no dense operators, no extraction pass, and
    (as there is no dense W) no dense dW -- the SURVEY §8 b default input-gradient policy."""
    import hgnn_amd.datagen as dg
    from hgnn_amd.csr import CsrBatch
    from models.gnns.model_mnb import GNN_lg
    torch.manual_seed(0)
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).cuda()
    graphs = dg.qm9_shape_dataset(bs, seed=1000)
    t0 = time.perf_counter()
    b = CsrBatch([(X, A) for X, A, _ in graphs], targets=torch.stack([t[0] for _, _, t in graphs]))
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    b.x.requires_grad_(True)
    crit = torch.nn.MSELoss()

    def step():
        model.zero_grad(set_to_none=True)
        b.x.grad = None
        crit(model.forward_csr(b), b.T).backward()

    sec = timeit(step, steps, warmup)
    return dict(config="cfg2csr", workload="GNN_lg d=64 order 2 L=5 fwd+bwd on a CsrBatch (no dense dW), 512 QM9-shape",
                graphs_per_step=bs, ms_per_step=round(sec * 1e3, 4), value=round(bs / sec, 2), unit="graphs/s",
                dtype="fp32", batch_build_ms=round(build_s * 1e3, 2), image_bytes=int(b.layout.bytes))


def run_train(steps, warmup, bs=512, csr=False):
    """Full train_with_mnb step on the device: forward, MSE, backward, Adamax (hgnn_amd.train.TrainStep)."""
    import hgnn_amd.datagen as dg
    from hgnn_amd.csr import CsrBatch
    from hgnn_amd.train import TrainStep
    from models.gnns.model_mnb import GNN_lg
    torch.manual_seed(0)
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).cuda()
    if csr:
        graphs = dg.qm9_shape_dataset(bs, seed=1000)
        batch = CsrBatch([(X, A) for X, A, _ in graphs], targets=torch.stack([t[0] for _, _, t in graphs]))
    else:
        batch = lg_batch(bs, 1000)
        batch[0].requires_grad_(True)   # X, W require grad as in scripts/train_mnb.py:56-57
        batch[1].requires_grad_(True)
    step = TrainStep(model, lr=3e-4, t_mean=0.5, t_std=2.0)
    sec = timeit(lambda: step(batch), steps, warmup)
    name = "cfg2train_csr" if csr else "cfg2train"
    return dict(config=name, workload="GNN_lg d=64 order 2 L=5 train step (fwd, MSE, bwd, Adamax) on "
                + ("a CsrBatch" if csr else "dense inputs (X, W require grad)") + ", 512 QM9-shape",
                graphs_per_step=bs, ms_per_step=round(sec * 1e3, 4), value=round(bs / sec, 2), unit="graphs/s",
                dtype="fp32", loss=float(step.stats[0].item()))


def run_simple(steps, warmup, graph=False):
    from models.gnns.model_mnb import GNN_simple
    torch.manual_seed(0)
    model = GNN_simple(0, 2, 20, 5, 1, 1).cuda()
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = lg_batch(32, 1000, sbm_n=50)
    X.requires_grad_(True)
    W.requires_grad_(True)
    crit = torch.nn.MSELoss()

    def step():
        for p in model.parameters():
            p.grad = None
        X.grad = W.grad = None
        crit(model([X, W], Nb, mask), T).backward()

    sec = timeit(graphed(step) if graph else step, steps, warmup)
    return dict(config="cfg1g" if graph else "cfg1",
                workload="GNN_simple(0,2,20,5,1,1) fwd+bwd, 32 SBM N=50 graphs"
                + (", step replayed from a HIP graph" if graph else ", eager"),
                graphs_per_step=32, ms_per_step=round(sec * 1e3, 4), value=round(32 / sec, 2), unit="graphs/s",
                dtype="fp32")


def run_ccn(name, order, graphs, desc, steps, warmup, graph=False):
    from models.compnets.model_ccn import CCN_1D, CCN_2D
    torch.manual_seed(0)
    net = (CCN_1D if order == 1 else CCN_2D)(5, 1, 2, 2).cuda()
    X, A, T, nb = ccn_batch(graphs)
    X.requires_grad_(True)
    # graph mode: the batch is planned once, outside the capture -- unless the small-graph CCN-1D
    # kernels take it (QM9-size graphs), which need no plan
    import hgnn_amd.ccn as HC
    small = HC.SMALL and net._spec().small(X.shape[0], X.shape[1]) is not None
    plan = net.plan(A, nb) if graph and not small else None

    def step():
        for p in net.parameters():
            p.grad = None
        X.grad = None
        out = net.forward_batch(X, A, nb, plan)
        ((out - T) ** 2).sum().backward()  # sum of the per-graph MSE losses (scripts/train_ccn.py:52-60)

    sec = timeit(graphed(step) if graph else step, steps, warmup)
    if graph:
        name += "g"
        desc += (", step replayed from a HIP graph (small-graph kernels)" if small else
                 ", plan built once, step replayed from a HIP graph")
    deg = (A > 0).sum(-1).double()
    sd, sd2, sd3 = float(deg.sum()), float((deg ** 2).sum()), float((deg ** 3).sum())
    return dict(config=name, workload=desc, graphs_per_step=len(graphs), ms_per_step=round(sec * 1e3, 4),
                value=round(len(graphs) / sec, 2), unit="graphs/s", dtype="fp32",
                sum_d=int(sd), sum_d2=int(sd2), sum_d3=int(sd3), d_max=int(deg.max()),
                roofline=ccn_roofline(order, net, sd, sd2, sd3, sec))


def run_ccn_pergraph(name, order, graphs, desc, steps, warmup):
    """The reference driver's CCN step as it is written (scripts/train_ccn.py:31-73): per graph,
    A + I, net(X, A) (the drop-in per-graph forward), MSE against t[task], backward and an
    Adamax step (scripts/main_ccn_qm9.py:178) -- one optimizer step per graph.  A "step" here is a
    pass over all the graphs; inputs already resident on the device."""
    from models.compnets.model_ccn import CCN_1D, CCN_2D
    torch.manual_seed(0)
    net = (CCN_1D if order == 1 else CCN_2D)(5, 1, 2, 2).cuda()
    opt = torch.optim.Adamax(net.parameters(), lr=1e-3)
    crit = torch.nn.MSELoss()
    data = [(x.cuda(), (a + torch.eye(a.shape[0])).cuda(), t[0].view(1).cuda()) for x, a, t in graphs]

    def epoch():
        for x, a, t in data:
            opt.zero_grad()
            loss = crit(net(x, a), t)
            loss.backward()
            opt.step()

    sec = timeit(epoch, steps, warmup)
    return dict(config=name, workload=desc, graphs_per_step=len(graphs), ms_per_step=round(sec * 1e3, 4),
                ms_per_graph=round(sec * 1e3 / len(graphs), 4), value=round(len(graphs) / sec, 2),
                unit="graphs/s", dtype="fp32")


def ccn_roofline(order, net, sd, sd2, sd3, sec, bw=8.0e12, peak=157.3e12):
    """SURVEY.md §8 d CCN formulas over the step's batch (Σd, Σd², Σd³ with the self loop):
    per layer, CCN-1D bytes 4(Σd·C_in + Σd·h + Σd²), FLOPs 2Σd²·C + 4Σd·C·h; CCN-2D bytes
    4(Σd²·C_in + Σd²·h + Σd²), FLOPs 2Σd³·C + 36Σd²·C·h (gathered bytes 4Σd³·C reported apart);
    fwd+bwd = 3x the forward."""
    c_in, h, layers = net.input_feats, net.hidden_size, net.layers
    cs = [c_in] + [h] * (layers - 1)
    byt = flo = gath = 0.0
    for c in cs:
        if order == 1:
            byt += 4 * (sd * c + sd * h + sd2)
            flo += 2 * sd2 * c + 4 * sd * c * h
        else:
            byt += 4 * (sd2 * c + sd2 * h + sd2)
            flo += 2 * sd3 * c + 36 * sd2 * c * h
            gath += 4 * sd3 * c
    byt, flo, gath = 3 * byt, 3 * flo, 3 * gath
    t_hbm, t_mfma = byt / bw, flo / peak
    out = dict(bound="hbm" if t_hbm >= t_mfma else "mfma", bytes_per_step=byt, flops_per_step=flo,
               achieved_gbs=round(byt / sec / 1e9, 3), frac_hbm=round(byt / sec / bw, 5),
               achieved_tflops=round(flo / sec / 1e12, 4), frac_mfma=round(flo / sec / peak, 5),
               frac_roofline=round(max(t_hbm, t_mfma) / sec, 5),
               formula="SURVEY.md §8 d, fwd+bwd = 3x forward")
    if order == 2:
        out["gathered_bytes_per_step"] = gath
        out["gathered_gbs"] = round(gath / sec / 1e9, 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    only = set(x for x in a.only.split(",") if x)
    import hgnn_amd.datagen as dg
    jobs = {
        "cfg1": lambda: run_simple(a.steps, a.warmup),
        "cfg1g": lambda: run_simple(a.steps, a.warmup, graph=True),
        "cfg2f": lambda: run_lg("cfg2f", "GNN_lg d=64 order 2 L=5, forward only, 512 QM9-shape", 64, 2, 512,
                                a.steps, a.warmup, backward=False),
        "cfg2o1": lambda: run_lg("cfg2o1", "GNN_lg d=64 order 1 L=5 fwd+bwd, 512 QM9-shape", 64, 1, 512, a.steps,
                                 a.warmup),
        "cfg2o3": lambda: run_lg("cfg2o3", "GNN_lg d=64 order 3 L=5 fwd+bwd, 512 QM9-shape", 64, 3, 512, a.steps,
                                 a.warmup),
        "cfg2csr": lambda: run_lg_csr(a.steps, a.warmup),
        "cfg2train": lambda: run_train(a.steps, a.warmup),
        "cfg2train_csr": lambda: run_train(a.steps, a.warmup, csr=True),
        "cfg3": lambda: run_ccn("cfg3", 1, dg.qm9_shape_dataset(256, seed=0),
                                "CCN_1D(5,1,2,2) fwd+bwd, 256 QM9-shape graphs", a.steps, a.warmup),
        "cfg3g": lambda: run_ccn("cfg3", 1, dg.qm9_shape_dataset(256, seed=0),
                                 "CCN_1D(5,1,2,2) fwd+bwd, 256 QM9-shape graphs", a.steps, a.warmup, graph=True),
        "cfg3_pergraph": lambda: run_ccn_pergraph(
            "cfg3_pergraph", 1, dg.qm9_shape_dataset(256, seed=0),
            "CCN_1D(5,1,2,2) per graph as scripts/train_ccn.py: net(X, A+I), MSE, backward, Adamax step; "
            "256 QM9-shape graphs", max(2, a.steps // 5), 1),
        "cfg4": lambda: run_lg("cfg4", "GNN_lg d=128 order 2 L=5 fwd+bwd, 512 QM9-shape (1 GPU of 4096)", 128, 2,
                               512, a.steps, a.warmup),
        "cfg5_pergraph": lambda: run_ccn_pergraph(
            "cfg5_pergraph", 2, dg.sbm_dataset(64, n=200, seed=0),
            "CCN_2D(5,1,2,2) per graph as scripts/train_ccn.py: net(X, A+I), MSE, backward, Adamax step; "
            "64 SBM N=200 graphs", 2, 1),
        "cfg5q_pergraph": lambda: run_ccn_pergraph(
            "cfg5q_pergraph", 2, dg.qm9_shape_dataset(256, seed=0),
            "CCN_2D(5,1,2,2) per graph as scripts/train_ccn.py: net(X, A+I), MSE, backward, Adamax step; "
            "256 QM9-shape graphs", max(2, a.steps // 5), 1),
        "cfg5q": lambda: run_ccn("cfg5q", 2, dg.qm9_shape_dataset(256, seed=0),
                                 "CCN_2D(5,1,2,2) fwd+bwd, 256 QM9-shape graphs", a.steps, a.warmup),
        "cfg5qg": lambda: run_ccn("cfg5q", 2, dg.qm9_shape_dataset(256, seed=0),
                                  "CCN_2D(5,1,2,2) fwd+bwd, 256 QM9-shape graphs", a.steps, a.warmup, graph=True),
        "cfg5": lambda: run_ccn("cfg5", 2, dg.sbm_dataset(64, n=200, seed=0),
                                "CCN_2D(5,1,2,2) fwd+bwd, 64 SBM N=200 graphs", max(3, a.steps // 4),
                                max(1, a.warmup // 2)),
    }
    for k, fn in jobs.items():
        if only and k not in only:
            continue
        print(json.dumps(fn()), flush=True)


if __name__ == "__main__":
    main()
