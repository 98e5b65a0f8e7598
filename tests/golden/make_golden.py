#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REAL reference.

Run once, in the survey container, where /root/reference is mounted:

    python tests/golden/make_golden.py

It imports the reference's own modules (functions/operators.py,
functions/batching.py, models/..., functions/utils_ccn.py,
functions/contraction.py) and records their outputs on seeded synthetic
inputs.  Only the resulting .npz data files are committed; nothing of the
reference travels to the GPU box.

Harness-side shims (the reference files are never edited):
* CCN `_get_chi` (functions/utils_ccn.py:80-82) guards an empty nonzero() with
  `shape == torch.Size([0])`, which torch>=1.0 broke (SURVEY.md §8 c, Q12);
  the shim restores the 2018 semantics with a numel()==0 guard.
* fp64 runs re-bind the module-level `dtype` globals to DoubleTensor
  (models/layers/layers_mnb.py:20-23, models/layers/batch_normalization.py:16-21)
  and call .double() on the model.
"""

import importlib.util
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, HERE)

import fixture_util as fu  # noqa: E402

spec = importlib.util.spec_from_file_location("datagen", os.path.join(REPO, "hgnn-2_amd", "hgnn_amd", "datagen.py"))
dg = importlib.util.module_from_spec(spec)
spec.loader.exec_module(dg)

from functions import operators as r_ops  # noqa: E402
from functions import batching as r_batch  # noqa: E402
from functions import contraction as r_contr  # noqa: E402
from functions import utils_ccn as r_ccn  # noqa: E402
from models.layers import layers_mnb as r_layers  # noqa: E402
from models.layers import batch_normalization as r_bn  # noqa: E402
from models.gnns import model_mnb as r_model  # noqa: E402
from models.compnets import model_ccn as r_mccn  # noqa: E402

torch.set_num_threads(8)


def _get_chi_shim(self, i, j):
    di = self.deg[i].item()
    dj = self.deg[j].item()
    chi = torch.zeros(di, dj).type(r_ccn.dtype)
    for k in range(di):
        ind_i = self.neighbors[i][k].item()
        ind_j = (self.neighbors[j] == ind_i).nonzero()
        if ind_j.numel() != 0:
            chi[k, ind_j.item()] = 1
    return chi


r_ccn.CompnetUtils._get_chi = _get_chi_shim


def set_dtype(dt):
    r_layers.dtype = dt
    r_bn.dtype = dt


def edge_case_graphs():
    g = []

    def mk(n, edges, selfloops=()):
        A = torch.zeros(n, n)
        for i, j, w in edges:
            A[i, j] = w
            A[j, i] = w
        for i in selfloops:
            A[i, i] = 1.0
        X = torch.eye(5)[torch.arange(n) % 5]
        return X, A, torch.zeros(13)

    g.append(mk(5, [(0, 1, 1), (1, 2, 1), (2, 3, 1), (3, 4, 1)]))                 # path
    g.append(mk(4, [(0, 1, 1), (1, 2, 1.5), (0, 2, 2), (2, 3, 1)]))               # triangle + pendant
    g.append(mk(5, [(0, 1, 1), (0, 2, 1.5), (0, 3, 2), (0, 4, 3)]))               # star, bond orders
    g.append(mk(7, [(0, 1, 1), (0, 2, 1), (1, 3, 2), (1, 4, 1), (2, 5, 3), (2, 6, 1.5)]))  # tree
    g.append(mk(6, [(0, 1, 1), (1, 2, 1), (3, 4, 2)]))                            # isolated node 5
    g.append(mk(5, [(0, 1, 1), (1, 2, 2), (2, 3, 1)], selfloops=(1, 4)))          # self loops (M counts diag)
    g.append(mk(2, [(0, 1, 1.5)]))                                                # single bond
    g.append(mk(4, [(1, 2, 1), (2, 3, 1)]))                                       # node 0 has no bond
    g.append(mk(6, [(0, 1, 1), (1, 2, 1), (2, 0, 1), (3, 4, 1), (4, 5, 1), (5, 3, 1), (0, 3, 2)]))  # two triangles
    return g


def gen_operators(out):
    t0 = time.time()
    rec = {}
    graphs = edge_case_graphs() + dg.qm9_shape_dataset(48, seed=11) + dg.sbm_dataset(4, n=50, seed=12)
    js = [1] * len(graphs)
    # J=2 on a few graphs (A^2 slice, AL^2 slice)
    extra = edge_case_graphs()[:4] + dg.qm9_shape_dataset(4, seed=13)
    graphs = graphs + extra
    js = js + [2] * len(extra)
    rec.update(fu.pack_graphs(graphs))
    rec["J"] = np.array(js, dtype=np.int64)
    for k, ((X, A, _t), J) in enumerate(zip(graphs, js)):
        W, WL, Pm, Pd = r_ops.graph_operators([X, A], J, True)
        Wo = r_ops.graph_operators([X, A], J, False)
        assert torch.equal(W, Wo)
        rec[f"W_{k}"] = W.numpy()
        rec[f"WL_{k}"] = WL.numpy()
        rec[f"Pm_{k}"] = Pm.numpy()
        rec[f"Pd_{k}"] = Pd.numpy()
    np.savez_compressed(os.path.join(out, "operators.npz"), **rec)
    print(f"operators: {len(graphs)} graphs, {time.time() - t0:.1f}s")


def gen_operators_hij(out):
    """J = 3, 4, 5 operators (slices up to A^16 / AL^16) of the QM9-shape graphs the large-J GPU tests use
    (tests/test_gpu_net.py::test_large_J_vs_oracle_fp64: qm9_shape_dataset(32, seed=40 + J)), as the reference's
    graph_operators (functions/operators.py:25-29, fp32 torch.matmul powers) computes them on this CPU: pins the
    operator bits the network tests feed to the GPU (J >= 4 powers leave fp32's exact range, so their rounding
    depends on the matmul's summation order)."""
    t0 = time.time()
    rec = {}
    for J in (3, 4, 5):
        graphs = dg.qm9_shape_dataset(32, seed=40 + J)
        rec.update({f"J{J}.{k}": v for k, v in fu.pack_graphs(graphs).items()})
        for k, (X, A, _t) in enumerate(graphs):
            W, WL, Pm, Pd = r_ops.graph_operators([X, A], J, True)
            rec[f"J{J}.W_{k}"] = W.numpy()
            rec[f"J{J}.WL_{k}"] = WL.numpy()
    np.savez_compressed(os.path.join(out, "operators_hij.npz"), **rec)
    print(f"operators_hij: {time.time() - t0:.1f}s")


def instances(graphs, J=1):
    data = []
    for X, A, t in graphs:
        W, WL, Pm, Pd = r_ops.graph_operators([X, A], J, True)
        data.append([X, A, t, W, WL, Pm, Pd])
    return data


def gen_batch(out):
    graphs = dg.qm9_shape_dataset(8, seed=21) + edge_case_graphs()[:4]
    data = instances(graphs)
    names = ["X", "W", "T", "XL", "WL", "Pm", "Pd", "mask", "mask_lg", "N_batch", "E_batch"]
    rec = fu.pack_graphs(graphs)
    b = r_batch.prepare_batch(data, 0, 1)
    for nm, v in zip(names, b):
        rec[nm] = v.numpy()
    # get_batches / _divide_batch index lists (functions/batching.py:26-74), unshuffled
    idx = r_batch.get_batches(23, 5, None, False, False)
    rec["batches_23_5"] = np.array([i for blk in idx for i in blk] + [-1] + [len(blk) for blk in idx])
    np.savez_compressed(os.path.join(out, "batch.npz"), **rec)
    print("batch: ok")


def run_lg(graphs, d, L, order, wseed, dtype64=False, J=1, train_then_eval=False):
    set_dtype(torch.DoubleTensor if dtype64 else torch.FloatTensor)
    data = instances(graphs, J)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, N_batch, E_batch = r_batch.prepare_batch(data, 0, J)
    model = r_model.GNN_lg(0, d, L, 5, 1, J, order)
    fu.det_init(model, wseed)
    if dtype64:
        model = model.double()
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg = [v.double() for v in (X, W, T, XL, WL, Pm, Pd, mask, mask_lg)]
    X.requires_grad = True
    W.requires_grad = True
    model.train()
    outp = model([X, XL, W, WL, Pm, Pd], N_batch, mask, E_batch, mask_lg)
    loss = torch.nn.MSELoss()(outp, T)
    loss.backward()
    res = {"out": outp.detach().numpy().copy(), "loss": np.array(loss.item())}
    res["dX"] = X.grad.numpy().copy()
    res["dW"] = W.grad.numpy().copy()
    for name, p in model.named_parameters():
        res["grad." + name] = p.grad.numpy().copy()
    for name, m in model.named_modules():
        if isinstance(m, r_bn.BN):
            res["rmean." + name] = m.running_mean.detach().numpy().copy()
            res["rstd." + name] = m.running_std.detach().numpy().copy()
    if train_then_eval:
        model.eval()
        with torch.no_grad():
            res["out_eval"] = model([X, XL, W, WL, Pm, Pd], N_batch, mask, E_batch, mask_lg).numpy().copy()
    set_dtype(torch.FloatTensor)
    return res


def gen_lggnn(out):
    cases = [
        # name, d, L, order, bs, graph seed, weight seed
        ("lg_d16_o1", 16, 5, 1, 32, 31, 101),
        ("lg_d16_o2", 16, 5, 2, 32, 32, 102),
        ("lg_d16_o3", 16, 5, 3, 32, 33, 103),
        ("lg_d64_o2", 64, 5, 2, 32, 34, 104),
        ("lg_d16_o2_L3", 16, 3, 2, 16, 35, 105),
        ("lg_d8_o2_L2", 8, 2, 2, 8, 36, 106),
    ]
    for name, d, L, order, bs, gseed, wseed in cases:
        t0 = time.time()
        graphs = dg.qm9_shape_dataset(bs, seed=gseed)
        if name == "lg_d16_o2":
            graphs = graphs[:-4] + edge_case_graphs()[:4]
        r32 = run_lg(graphs, d, L, order, wseed, train_then_eval=True)
        r64 = run_lg(graphs, d, L, order, wseed, dtype64=True)
        rec = fu.pack_graphs(graphs)
        rec["cfg"] = np.array([d, L, order, bs, wseed])
        for k, v in r32.items():
            rec[k] = v
        rec["out64"] = r64["out"]
        rec["loss64"] = r64["loss"]
        for k, v in r64.items():
            if k.startswith("grad.") or k in ("dX",):
                rec["g64." + k] = v
        np.savez_compressed(os.path.join(out, name + ".npz"), **rec)
        print(f"{name}: loss {float(r32['loss']):.6f}  |out32-out64| {np.abs(r32['out'] - r64['out']).max():.3e}  {time.time() - t0:.1f}s")


def gen_gnn_simple(out):
    graphs = dg.sbm_dataset(32, n=50, seed=41)
    data = instances(graphs)
    res = {}
    for dt in ("32", "64"):
        set_dtype(torch.DoubleTensor if dt == "64" else torch.FloatTensor)
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, N_batch, E_batch = r_batch.prepare_batch(data, 0, 1)
        model = r_model.GNN_simple(0, 2, 20, 5, 1, 1)
        fu.det_init(model, 201)
        if dt == "64":
            model = model.double()
            X, W, T, mask = X.double(), W.double(), T.double(), mask.double()
        X.requires_grad = True
        W.requires_grad = True
        model.train()
        o = model([X, W], N_batch, mask)
        loss = torch.nn.MSELoss()(o, T)
        loss.backward()
        res["out" + dt] = o.detach().numpy().copy()
        res["loss" + dt] = np.array(loss.item())
        res["dX" + dt] = X.grad.numpy().copy()
        for name, p in model.named_parameters():
            res[f"grad{dt}.{name}"] = p.grad.numpy().copy()
        if dt == "32":
            model.eval()
            with torch.no_grad():
                res["out_eval"] = model([X, W], N_batch, mask).numpy().copy()
    set_dtype(torch.FloatTensor)
    rec = fu.pack_graphs(graphs)
    rec.update(res)
    np.savez_compressed(os.path.join(out, "gnn_simple.npz"), **rec)
    print(f"gnn_simple: loss {float(res['loss32']):.6f} |d| {np.abs(res['out32'] - res['out64']).max():.3e}")


def gen_layers(out):
    """Layer-level I/O: graph_oper, P_multi, BN train/eval (fixed inputs)."""
    g = torch.Generator().manual_seed(51)
    graphs = dg.qm9_shape_dataset(6, seed=52)
    data = instances(graphs)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, N_batch, E_batch = r_batch.prepare_batch(data, 0, 1)
    F = 7
    Xf = torch.randn(X.shape[0], F, X.shape[2], generator=g)
    XLf = torch.randn(X.shape[0], F, XL.shape[2], generator=g)
    rec = fu.pack_graphs(graphs)
    rec["Xf"] = Xf.numpy()
    rec["XLf"] = XLf.numpy()
    rec["gop_W"] = r_layers.graph_oper()(W, Xf).numpy()
    rec["gop_WL"] = r_layers.graph_oper()(WL, XLf).numpy()
    rec["pm_XL"] = r_layers.P_multi()(Pm, XLf).numpy()
    rec["pdT_X"] = r_layers.P_multi()(Pd.transpose(2, 1), Xf).numpy()
    bn = r_bn.BN(F)
    with torch.no_grad():
        bn.weight.fill_(0.7)
        bn.bias.fill_(-0.2)
    bn.train()
    rec["bn_train"] = bn(Xf, N_batch, mask).detach().numpy()
    rec["bn_rmean"] = bn.running_mean.detach().numpy()
    rec["bn_rstd"] = bn.running_std.detach().numpy()
    bn.eval()
    rec["bn_eval"] = bn(Xf * 0.5 + 0.1, N_batch, mask).detach().numpy()
    np.savez_compressed(os.path.join(out, "layers.npz"), **rec)
    print("layers: ok")


def gen_ccn(out):
    t0 = time.time()
    rec = {}
    # collapse6to3 via python_contract(T, I) on random T (functions/utils_ccn.py:37-45)
    g = torch.Generator().manual_seed(61)
    cu = r_ccn.CompnetUtils(False)
    for d in range(1, 7):
        T = torch.randn(d, d, d, 3, generator=g)
        rec[f"c6_T_{d}"] = T.numpy()
        rec[f"c6_out_{d}"] = cu.outer_contract(T, torch.eye(d)).numpy()
    qm = dg.qm9_shape_dataset(12, seed=62)
    sb = dg.sbm_dataset(2, n=24, seed=63)
    graphs = qm + sb
    rec.update(fu.pack_graphs(graphs))
    for k, (X, A, t) in enumerate(graphs):
        adj = A + torch.eye(A.shape[0])
        deg, nbr, pos = fu.chi_position_maps(adj.numpy())
        rec[f"deg_{k}"] = deg
        rec[f"nbr_{k}"] = nbr
        rec[f"pos_{k}"] = pos
        # reference chi matrices -> position maps (cross-check of the helper)
        u = r_ccn.CompnetUtils(False)
        u.get_F0_1D(X, adj)
        rp = []
        for i in range(adj.shape[0]):
            for j in range(adj.shape[0]):
                if adj[i, j] > 0:
                    chi = u.chis[i][j]
                    for x in range(chi.shape[0]):
                        nz = torch.nonzero(chi[x]).flatten()
                        rp.append(int(nz[0]) if nz.numel() else -1)
        assert np.array_equal(np.array(rp), pos), "chi helper mismatch"
    for kind, cls in (("1d", r_mccn.CCN_1D), ("2d", r_mccn.CCN_2D)):
        for k, (X, A, t) in enumerate(graphs):
            if kind == "2d" and k >= len(qm) + 1:
                continue
            net = cls(5, 1, 2, 2, False)
            fu.det_init(net, 300 + k)
            adj = A + torch.eye(A.shape[0])
            Xr = X.clone().requires_grad_(True)
            o = net(Xr, adj)
            y = t[0].view(1)
            loss = torch.nn.MSELoss()(o, y)
            loss.backward()
            rec[f"{kind}_out_{k}"] = o.detach().numpy()
            rec[f"{kind}_loss_{k}"] = np.array(loss.item())
            rec[f"{kind}_dX_{k}"] = Xr.grad.numpy()
            for name, p in net.named_parameters():
                rec[f"{kind}_grad_{k}.{name}"] = p.grad.numpy()
    np.savez_compressed(os.path.join(out, "ccn.npz"), **rec)
    print(f"ccn: {time.time() - t0:.1f}s")


if __name__ == "__main__":
    out = HERE
    which = sys.argv[1:] or ["operators", "batch", "layers", "lggnn", "gnn_simple", "ccn"]
    for w in which:
        globals()["gen_" + w](out)
