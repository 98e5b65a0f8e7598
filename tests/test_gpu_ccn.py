"""CCN-1D / CCN-2D on the GPU vs the reference's fixtures and the oracle (oracle/ref_ccn.py).

Tolerances (north_star: fp32 within 1e-5 of the reference's CPU forward):
outputs |gpu - ref| <= 1e-5 max(1, |ref|); gradients within
1e-4 max|g| + 1e-5 |g| (summation order differs from the reference's
per-node autograd); index construction bit-exact.
"""

import numpy as np
import pytest
import torch

import fixture_util as fu
from test_oracle import ccn_graphs, ccn_params

pytestmark = pytest.mark.gpu


def _close(got, ref, what, rel=1e-5):
    got = got.detach().double().cpu()
    ref = torch.as_tensor(ref).double()
    err = (got - ref).abs().max().item() if got.numel() else 0.0
    tol = rel * max(1.0, ref.abs().max().item() if ref.numel() else 0.0)
    assert err <= tol, f"{what}: max err {err:.3g} > {tol:.3g}"


def _grad_close(got, ref, what):
    got = got.detach().double().cpu()
    ref = torch.as_tensor(ref).double()
    tol = 1e-4 * ref.abs().max().item() + 1e-5 * ref.abs() + 1e-7
    bad = (got - ref).abs() > tol
    assert not bad.any(), f"{what}: max err {(got - ref).abs().max().item():.3g}"


def _pad(graphs, dev):
    bs = len(graphs)
    nmax = max(X.shape[0] for X, _, _ in graphs)
    f = graphs[0][0].shape[1]
    X = torch.zeros(bs, nmax, f)
    A = torch.zeros(bs, nmax, nmax)
    for b, (x, a, _) in enumerate(graphs):
        n = x.shape[0]
        X[b, :n] = x
        A[b, :n, :n] = a
    nb = torch.tensor([g[0].shape[0] for g in graphs], dtype=torch.int64)
    return X.to(dev), A.to(dev), nb.to(dev)


def test_ccn_plan_maps_bit_exact(golden):
    from hgnn_amd.ccn import plan_maps
    z = golden("ccn")
    graphs = ccn_graphs(z)
    X, A, nb = _pad(graphs, "cuda")
    for order in (1, 2):
        maps = plan_maps(order, X, A, nb)
        for k, (deg, nbr, pos) in enumerate(maps):
            assert np.array_equal(deg, z[f"deg_{k}"]), k
            assert np.array_equal(nbr, z[f"nbr_{k}"]), k
            assert np.array_equal(pos, z[f"pos_{k}"]), k


def test_collapse6to3_matches_reference(golden):
    from functions.contraction import collapse6to3
    z = golden("ccn")
    for d in range(1, 7):
        T = torch.from_numpy(z[f"c6_T_{d}"])
        H = (T.permute(3, 0, 1, 2).unsqueeze(4).unsqueeze(5) * torch.eye(d)).contiguous().cuda()
        _close(collapse6to3(H), z[f"c6_out_{d}"], f"collapse d={d}")


def test_collapse6to3_general_and_adjoint():
    """General F (not T (x) I) vs the oracle's einsum restatement; backward = exact adjoint."""
    from functions.contraction import collapse6to3
    from oracle import ref_ccn as RC
    g = torch.Generator().manual_seed(5)
    for c, n in ((1, 2), (3, 4), (2, 5)):
        F = torch.randn(c, n, n, n, n, n, generator=g)
        Fg = F.cuda().requires_grad_(True)
        out = collapse6to3(Fg)
        _close(out, RC.collapse6to3(F.double()), f"general collapse c={c} n={n}")
        G = torch.randn(out.shape, generator=g)
        out.backward(G.cuda())
        lhs = (RC.collapse6to3(F.double()) * G.double()).sum().item()
        rhs = (F.double() * Fg.grad.double().cpu()).sum().item()
        assert abs(lhs - rhs) <= 1e-4 * max(1.0, abs(lhs)), (c, n, lhs, rhs)


@pytest.mark.parametrize("kind", ["1d", "2d"])
def test_ccn_per_graph_matches_reference(golden, kind):
    """The drop-in forward(X, adj) + MSE backward, graph by graph, as scripts/train_ccn.py runs it."""
    z = golden("ccn")
    for k, (X, adj, t) in enumerate(ccn_graphs(z)):
        if f"{kind}_out_{k}" not in z:
            continue
        net, _ = ccn_params(kind, k)
        net = net.cuda()
        Xr = X.cuda().requires_grad_(True)
        out = net(Xr, adj.cuda())
        assert out.shape == (1,)
        loss = torch.nn.MSELoss()(out, t[0].view(1).cuda())
        loss.backward()
        _close(out, z[f"{kind}_out_{k}"], f"{kind} out {k}")
        _close(loss.view(1), np.array([z[f"{kind}_loss_{k}"]]), f"{kind} loss {k}")
        _grad_close(Xr.grad, z[f"{kind}_dX_{k}"], f"{kind} dX {k}")
        for n, p in net.named_parameters():
            _grad_close(p.grad, z[f"{kind}_grad_{k}.{n}"], f"{kind} grad {k} {n}")


@pytest.mark.parametrize("order", [1, 2])
def test_ccn_batched_matches_oracle(order):
    """A padded batch of QM9-shape + SBM graphs in one call vs the fp64 oracle per graph."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D, CCN_2D
    from oracle import ref_ccn as RC
    graphs = dg.qm9_shape_dataset(24, seed=71) + dg.sbm_dataset(3, n=20, seed=72)
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in graphs]
    f = graphs[0][0].shape[1]
    sbm_f = graphs[-1][0].shape[1]
    if sbm_f != f:
        graphs = graphs[:24]
    net = (CCN_1D if order == 1 else CCN_2D)(f, 2, 3, 3)
    fu.det_init(net, 77)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    Xr = X.clone().requires_grad_(True)
    out = net.forward_batch(Xr, A, nb)
    w = torch.randn(out.shape, generator=torch.Generator().manual_seed(3))
    (out * w.cuda()).sum().backward()
    for b, (x, a, _) in enumerate(graphs):
        xr = x.double().requires_grad_(True)
        ref = RC.ccn_forward(p64, xr, a.double(), order, 3)
        _close(out[b], ref, f"order {order} graph {b}")
        (ref * w[b].double()).sum().backward()
        n = x.shape[0]
        _grad_close(Xr.grad[b, :n], xr.grad, f"dX graph {b}")
        assert Xr.grad[b, n:].abs().max().item() == 0.0 if n < X.shape[1] else True
    for n, p in net.named_parameters():
        _grad_close(p.grad, p64[n].grad, f"grad {n}")


def test_ccn_batched_equals_per_graph():
    """Packing is invisible: forward_batch rows equal the single-graph forward."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_2D
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in dg.qm9_shape_dataset(10, seed=81)]
    net = CCN_2D(5, 1, 2, 2).cuda()
    X, A, nb = _pad(graphs, "cuda")
    with torch.no_grad():
        ob = net.forward_batch(X, A, nb)
        for b, (x, a, _) in enumerate(graphs):
            o = net(x.cuda(), a.cuda())
            _close(o, ob[b].cpu(), f"graph {b}", rel=1e-6)


def test_ccn_missing_self_loop_raises():
    from models.compnets.model_ccn import CCN_1D
    net = CCN_1D(5, 1, 2, 2).cuda()
    A = torch.zeros(4, 4)
    A[0, 1] = A[1, 0] = 1.0
    with pytest.raises(RuntimeError, match="self loop"):
        net(torch.randn(4, 5).cuda(), A.cuda())


def test_ccn2_sbm200_config5_matches_closed_form_oracle():
    """Config 5 size (SBM N = 200, degrees up to ~57): the reference cannot run it (d^5 intermediates,
    SURVEY.md §6), so the batched HIP CCN-2D is checked against the fp64 closed-form oracle
    (oracle/ref_ccn.py ccn2_forward_closed, itself pinned to the literal restatement on the CPU):
    outputs, parameter gradients and dX for a batch of 3 SBM-200 graphs."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_2D
    from oracle import ref_ccn as RC
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in dg.sbm_dataset(3, n=200, seed=0)]
    net = CCN_2D(5, 1, 2, 2)
    fu.det_init(net, 55)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    Xr = X.clone().requires_grad_(True)
    out = net.forward_batch(Xr, A, nb)
    w = torch.tensor([[1.0], [-0.5], [0.25]])
    (out * w.cuda()).sum().backward()
    for b, (x, a, _) in enumerate(graphs):
        xr = x.double().requires_grad_(True)
        ref = RC.ccn2_forward_closed(p64, xr, a.double(), 2)
        _close(out[b], ref, f"sbm200 graph {b}")
        (ref * w[b].double()).sum().backward()
        _grad_close(Xr.grad[b, :x.shape[0]], xr.grad, f"sbm200 dX graph {b}")
    for n, p in net.named_parameters():
        _grad_close(p.grad, p64[n].grad, f"sbm200 grad {n}")


def test_ccn1_sbm_large_degree_vs_oracle():
    """CCN-1D beyond one wave of receptive field: SBM N = 400 (degrees ~70-90) and N = 1000 (~175-210,
    the north star's largest SBM) in one padded batch vs the fp64 vectorised oracle
    (oracle/ref_ccn.py ccn1_forward_vec, pinned to the literal restatement): outputs, dX, grads."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D
    from oracle import ref_ccn as RC
    graphs = dg.sbm_dataset(2, n=400, seed=41) + dg.sbm_dataset(1, n=1000, seed=42)
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in graphs]
    assert max(int((a > 0).sum(1).max()) for _, a, _ in graphs) > 128
    net = CCN_1D(5, 1, 2, 2)
    fu.det_init(net, 43)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    Xr = X.clone().requires_grad_(True)
    out = net.forward_batch(Xr, A, nb)
    w = torch.tensor([[1.0], [-0.5], [0.25]])
    (out * w.cuda()).sum().backward()
    for b, (x, a, _) in enumerate(graphs):
        xr = x.double().requires_grad_(True)
        ref = RC.ccn1_forward_vec(p64, xr, a.double(), 2)
        _close(out[b], ref, f"sbm graph {b}")
        (ref * w[b].double()).sum().backward()
        _grad_close(Xr.grad[b, :x.shape[0]], xr.grad, f"sbm dX graph {b}")
    for n, p in net.named_parameters():
        _grad_close(p.grad, p64[n].grad, f"sbm grad {n}")


@pytest.mark.parametrize("hidden", [16, 12])
def test_ccn2_wide_channels_vs_closed_form_oracle(hidden):
    """CCN-2D with hidden > 8 (the wide kernel instantiations, channels <= 16) vs the fp64 closed-form
    oracle on QM9-shape graphs and one SBM-30 graph: outputs, dX and parameter gradients."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_2D
    from oracle import ref_ccn as RC
    graphs = dg.qm9_shape_dataset(6, seed=91) + dg.sbm_dataset(1, n=30, seed=92)
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in graphs]
    net = CCN_2D(5, 1, hidden, 2)
    fu.det_init(net, 93)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    Xr = X.clone().requires_grad_(True)
    out = net.forward_batch(Xr, A, nb)
    w = torch.randn(out.shape, generator=torch.Generator().manual_seed(94))
    (out * w.cuda()).sum().backward()
    for b, (x, a, _) in enumerate(graphs):
        xr = x.double().requires_grad_(True)
        ref = RC.ccn2_forward_closed(p64, xr, a.double(), 2)
        _close(out[b], ref, f"hidden {hidden} graph {b}")
        (ref * w[b].double()).sum().backward()
        _grad_close(Xr.grad[b, :x.shape[0]], xr.grad, f"hidden {hidden} dX graph {b}")
    for n, p in net.named_parameters():
        _grad_close(p.grad, p64[n].grad, f"hidden {hidden} grad {n}")


def test_ccn1_config3_full_batch_256_vs_oracle():
    """Config 3 at its size: CCN_1D(5, 1, 2, 2) (scripts/main_ccn_qm9.py:69-74 defaults) on 256
    QM9-shape graphs in one forward_batch call, loss = sum of the per-graph MSE (the reference's
    per-graph train_ccn step, scripts/train_ccn.py:52-60, summed), against the fp64 oracle per graph
    (oracle/ref_ccn.py ccn1_forward_vec, pinned to the literal restatement): every output, every
    graph's dX and the parameter gradients."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D
    from oracle import ref_ccn as RC
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in dg.qm9_shape_dataset(256, seed=303)]
    net = CCN_1D(5, 1, 2, 2)
    fu.det_init(net, 303)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    T = torch.stack([t[0] for _, _, t in graphs]).view(-1, 1)
    Xr = X.clone().requires_grad_(True)
    out = net.forward_batch(Xr, A, nb)
    ((out - T.cuda()) ** 2).sum().backward()
    loss64 = 0.0
    for b, (x, a, _) in enumerate(graphs):
        xr = x.double().requires_grad_(True)
        ref = RC.ccn1_forward_vec(p64, xr, a.double(), 2)
        _close(out[b], ref, f"cfg3 graph {b}")
        lb = ((ref - T[b].double()) ** 2).sum()
        lb.backward()
        loss64 += lb.item()
        _grad_close(Xr.grad[b, :x.shape[0]], xr.grad, f"cfg3 dX graph {b}")
    for n, p in net.named_parameters():
        _grad_close(p.grad, p64[n].grad, f"cfg3 grad {n}")


def test_ccn2_config5_full_batch_64_sbm200():
    """Config 5 at its size: CCN_2D(5, 1, 2, 2) on 64 SBM-200 graphs (degrees up to ~57).
    (1) Full-size property: one forward_batch call equals the drop-in per-graph forward(X, adj)
    that scripts/train_ccn.py:52 calls, on all 64 graphs -- outputs, each graph's dX and the
    parameter gradients (the per-graph backward passes summed).  (2) The reference cannot run
    SBM-200 (d^5 intermediates): 8 of the 64 graphs against the fp64 closed-form
    oracle (oracle/ref_ccn.py ccn2_forward_closed, pinned to the literal restatement) -- outputs,
    dX, and the parameter gradients of those 8 graphs' terms."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_2D
    from oracle import ref_ccn as RC
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in dg.sbm_dataset(64, n=200, seed=505)]
    net = CCN_2D(5, 1, 2, 2)
    fu.det_init(net, 505)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    w = torch.randn(64, 1, generator=torch.Generator().manual_seed(506))
    Xr = X.clone().requires_grad_(True)
    out = net.forward_batch(Xr, A, nb)
    params = [p for _, p in net.named_parameters()]
    gb = torch.autograd.grad((out * w.cuda()).sum(), [Xr] + params, retain_graph=True)
    # (1) per-graph drop-in path on all 64 graphs
    gsum = [torch.zeros_like(p) for p in params]
    for b, (x, a, _) in enumerate(graphs):
        xr = x.cuda().requires_grad_(True)
        o = net(xr, a.cuda())
        _close(o, out[b].detach().cpu(), f"cfg5 per-graph out {b}", rel=1e-6)
        gs = torch.autograd.grad((o * w[b].cuda()).sum(), [xr] + params)
        _close(gs[0], gb[0][b, :x.shape[0]].cpu(), f"cfg5 per-graph dX {b}", rel=1e-5)
        for acc, g in zip(gsum, gs[1:]):
            acc += g
    for (n, _), g1, g2 in zip(net.named_parameters(), gb[1:], gsum):
        _grad_close(g1, g2.cpu(), f"cfg5 per-graph sum grad {n}")
    # (2) the closed-form fp64 oracle on 8 of the graphs
    sel = list(range(0, 64, 8))
    wsel = torch.zeros(64, 1)
    wsel[sel] = w[sel]
    g8 = torch.autograd.grad((out * wsel.cuda()).sum(), params)
    for b in sel:
        x, a, _ = graphs[b]
        xr = x.double().requires_grad_(True)
        ref = RC.ccn2_forward_closed(p64, xr, a.double(), 2)
        _close(out[b], ref, f"cfg5 graph {b}")
        (ref * w[b].double()).sum().backward()
        _grad_close(gb[0][b, :x.shape[0]], xr.grad, f"cfg5 dX graph {b}")
    for (n, _), g in zip(net.named_parameters(), g8):
        _grad_close(g, p64[n].grad, f"cfg5 grad {n}")


@pytest.mark.parametrize("hidden", [2, 12])
def test_ccn2_degree_above_64_vs_closed_form_oracle(hidden):
    """CCN-2D receptive fields beyond one wave: SBM N = 300 (degrees ~40-75, so one graph mixes the
    fast d <= 64 kernels and the large-degree ones) and N = 400 (~60-100) in one padded batch vs the
    fp64 closed-form oracle (oracle/ref_ccn.py ccn2_forward_closed): outputs, dX, parameter grads;
    and the per-graph drop-in forward equals the batched one."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_2D
    from oracle import ref_ccn as RC
    graphs = dg.sbm_dataset(1, n=300, seed=41) + dg.sbm_dataset(1, n=400, seed=42)
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in graphs]
    degs = [int((a > 0).sum(1).max()) for _, a, _ in graphs]
    assert max(degs) > 64 and min(int((a > 0).sum(1).min()) for _, a, _ in graphs) <= 64, degs
    net = CCN_2D(5, 1, hidden, 2)
    fu.det_init(net, 64 + hidden)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    Xr = X.clone().requires_grad_(True)
    out = net.forward_batch(Xr, A, nb)
    w = torch.tensor([[1.0], [-0.75]])
    (out * w.cuda()).sum().backward()
    for b, (x, a, _) in enumerate(graphs):
        with torch.no_grad():
            _close(net(x.cuda(), a.cuda()), out[b].detach().cpu(), f"per-graph {b}", rel=1e-6)
        xr = x.double().requires_grad_(True)
        ref = RC.ccn2_forward_closed(p64, xr, a.double(), 2)
        _close(out[b], ref, f"deg>64 graph {b}")
        (ref * w[b].double()).sum().backward()
        _grad_close(Xr.grad[b, :x.shape[0]], xr.grad, f"deg>64 dX graph {b}")
    for n, p in net.named_parameters():
        _grad_close(p.grad, p64[n].grad, f"deg>64 grad {n}")


@pytest.mark.parametrize("layers", [1, 4])
def test_ccn2_layer_counts_vs_closed_form_oracle(layers):
    """CCN-2D with one level (the top level is level 0: its backward reads the readout slice directly and
    runs the closed-form level-0 pass) and with four (three gather levels) on QM9-shape graphs and one
    SBM-40 graph, against the fp64 closed-form oracle: outputs, dX, parameter gradients."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_2D
    from oracle import ref_ccn as RC
    graphs = dg.qm9_shape_dataset(5, seed=120 + layers) + dg.sbm_dataset(1, n=40, seed=130 + layers)
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in graphs]
    net = CCN_2D(5, 1, 2, layers)
    fu.det_init(net, 140 + layers)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    Xr = X.clone().requires_grad_(True)
    out = net.forward_batch(Xr, A, nb)
    w = torch.randn(out.shape, generator=torch.Generator().manual_seed(150 + layers))
    (out * w.cuda()).sum().backward()
    for b, (x, a, _) in enumerate(graphs):
        xr = x.double().requires_grad_(True)
        ref = RC.ccn2_forward_closed(p64, xr, a.double(), layers)
        _close(out[b], ref, f"L={layers} graph {b}")
        (ref * w[b].double()).sum().backward()
        _grad_close(Xr.grad[b, :x.shape[0]], xr.grad, f"L={layers} dX graph {b}")
    for n, p in net.named_parameters():
        _grad_close(p.grad, p64[n].grad, f"L={layers} grad {n}")


def _run_path(small, net, X, A, nb, w):
    """forward_batch + weighted-sum backward on one path (hgnn_amd.ccn.SMALL)"""
    import hgnn_amd.ccn as HC
    old = HC.SMALL
    HC.SMALL = small
    try:
        net.zero_grad(set_to_none=True)
        Xr = X.clone().requires_grad_(True)
        out = net.forward_batch(Xr, A, nb)
        (out * w).sum().backward()
        torch.cuda.synchronize()
        return out.detach().cpu(), Xr.grad.cpu(), {n: p.grad.detach().cpu().clone() for n, p in net.named_parameters()}
    finally:
        HC.SMALL = old


@pytest.mark.parametrize("f,h,layers,bs", [(5, 2, 2, 1), (5, 2, 2, 64), (7, 5, 4, 16), (3, 8, 1, 5)])
def test_ccn1_small_graph_path_equals_general_path(f, h, layers, bs):
    """The one-workgroup-per-graph CCN-1D kernels (csrc/ccn_small.hip) against the general path on
    the same batch: outputs and dX bit-identical (same fp32 order per level, same fp64 readout), weight
    gradients on the gradient bound (different summation order), and against the fp64 oracle."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D
    from oracle import ref_ccn as RC
    graphs = [(X[:, :f] if X.shape[1] >= f else torch.cat([X, torch.rand(X.shape[0], f - X.shape[1])], 1),
               A + torch.eye(A.shape[0]), t) for X, A, t in dg.qm9_shape_dataset(bs, seed=500 + bs)]
    net = CCN_1D(f, 2, h, layers)
    fu.det_init(net, 91 + layers)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    assert net._spec().small(X.shape[0], X.shape[1]) is not None
    w = torch.randn(bs, 2, generator=torch.Generator().manual_seed(bs)).cuda()
    os_, dxs, gs = _run_path(True, net, X, A, nb, w)
    og, dxg, gg = _run_path(False, net, X, A, nb, w)
    assert torch.equal(os_, og), f"outputs differ: {(os_ - og).abs().max().item():.3g}"
    assert torch.equal(dxs, dxg), f"dX differs: {(dxs - dxg).abs().max().item():.3g}"
    for n in gg:
        _grad_close(gs[n], gg[n], f"small vs general grad {n}")
    for b, (x, a, _) in enumerate(graphs[:8]):
        xr = x.double().requires_grad_(True)
        ref = RC.ccn_forward(p64, xr, a.double(), 1, layers)
        _close(os_[b], ref, f"small path graph {b}")
        (ref * w[b].double().cpu()).sum().backward()
        _grad_close(dxs[b, :x.shape[0]], xr.grad, f"small path dX graph {b}")
        assert dxs[b, x.shape[0]:].abs().max().item() == 0.0 if x.shape[0] < X.shape[1] else True


def test_ccn1_small_graph_path_per_graph_drop_in():
    """net(X, A + I) per graph (n_batch None: the small path without any index tensor) equals the
    batched general path row by row; the input gradient of the per-graph call as well."""
    import hgnn_amd.ccn as HC
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D
    graphs = [(X, A + torch.eye(A.shape[0]), t) for X, A, t in dg.qm9_shape_dataset(12, seed=515)]
    net = CCN_1D(5, 1, 2, 2)
    fu.det_init(net, 515)
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    old = HC.SMALL
    HC.SMALL = False
    try:
        ob = net.forward_batch(X, A, nb).detach().cpu()
    finally:
        HC.SMALL = old
    for b, (x, a, _) in enumerate(graphs):
        xr = x.cuda().requires_grad_(True)
        o = net(xr, a.cuda())
        assert torch.equal(o.detach().cpu(), ob[b]), f"graph {b}"
        o.sum().backward()
        assert torch.isfinite(xr.grad).all()


def test_ccn1_small_graph_path_validation():
    """The small path reports the general plan's validation bits: missing self loop, asymmetric
    pattern, n_b > nmax -- raised by the next check (HGNN_STRICT semantics unchanged)."""
    from hgnn_amd.net import check_errors
    from models.compnets.model_ccn import CCN_1D
    net = CCN_1D(5, 1, 2, 2).cuda()
    A = torch.eye(4)
    A[0, 1] = 1.0  # 1 does not list 0
    with pytest.raises(RuntimeError, match="not symmetric"):
        net(torch.randn(4, 5).cuda(), A.cuda())
        check_errors()
    A = torch.eye(4).unsqueeze(0)
    with pytest.raises(RuntimeError, match="negative count"):
        net.forward_batch(torch.randn(1, 4, 5).cuda(), A.cuda(), torch.tensor([5]).cuda())
        check_errors()
    # a clean call after the failures raises nothing (tags: older words do not count)
    net(torch.randn(4, 5).cuda(), torch.eye(4).cuda())
    check_errors()


def test_ccn1_small_graph_path_ragged_edge_cases():
    """Ragged batch with a single-node graph, an empty slot (n_b = 0) and a QM9-shape graph: the small-graph
    kernels equal the general path (outputs, dX, zeroed padding rows) and the empty slot reads fc.bias."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D
    (xq, aq, _), = dg.qm9_shape_dataset(1, seed=9)
    n = xq.shape[0]
    X = torch.zeros(3, n, 5)
    A = torch.zeros(3, n, n)
    X[0, :1] = torch.randn(1, 5)
    A[0, 0, 0] = 1.0
    X[2, :n] = xq
    A[2, :n, :n] = aq + torch.eye(n)
    nb = torch.tensor([1, 0, n], dtype=torch.int64)
    net = CCN_1D(5, 1, 2, 2)
    fu.det_init(net, 909)
    net = net.cuda()
    X, A, nb = X.cuda(), A.cuda(), nb.cuda()
    w = torch.ones(3, 1).cuda()
    os_, dxs, gs = _run_path(True, net, X, A, nb, w)
    og, dxg, gg = _run_path(False, net, X, A, nb, w)
    assert torch.equal(os_, og)
    assert torch.equal(dxs, dxg)
    for k in gg:
        _grad_close(gs[k], gg[k], f"ragged grad {k}")
    assert torch.equal(os_[1], net.fc.bias.detach().cpu())
    assert dxs[1].abs().max().item() == 0.0 and dxs[0, 1:].abs().max().item() == 0.0


def test_ccn1_small_graph_path_inplace_input_change_raises():
    """The small path's backward rebuilds every level from X, adj and the weights (ccn_small.hip), so
    they are saved through autograd: changing X in place between forward and backward raises the
    version error instead of returning gradients of a different input."""
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D
    (x, a, _), = dg.qm9_shape_dataset(1, seed=21)
    net = CCN_1D(5, 1, 2, 2).cuda()
    X = x.cuda().requires_grad_(True)
    Xi = X * 1.0  # a non-leaf the caller may reuse as a staging buffer
    out = net(Xi, (a + torch.eye(a.shape[0])).cuda())
    assert net._spec().small(1, x.shape[0]) is not None
    with torch.no_grad():
        Xi.add_(1.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        out.sum().backward()


def _qm9_2d(bs, seed, f=5):
    import hgnn_amd.datagen as dg
    return [(X[:, :f] if X.shape[1] >= f else torch.cat([X, torch.rand(X.shape[0], f - X.shape[1])], 1),
             A + torch.eye(A.shape[0]), t) for X, A, t in dg.qm9_shape_dataset(bs, seed=seed)]


@pytest.mark.parametrize("f,h,layers,bs", [(5, 2, 2, 1), (5, 2, 2, 64), (7, 1, 3, 16), (3, 2, 1, 5)])
def test_ccn2_small_graph_path_equals_general_path(f, h, layers, bs):
    """The one-workgroup-per-graph CCN-2D kernels (csrc/ccn2_small.hip) against the general path on the
    same batch: outputs, dX and the weight gradients bit-identical (the general kernels' arithmetic in the
    same order, the batch's parameter partials reduced in k_ccn_param_reduce's order), and against the
    closed-form fp64 oracle (oracle/ref_ccn.py ccn2_forward_closed)."""
    from models.compnets.model_ccn import CCN_2D
    from oracle import ref_ccn as RC
    graphs = _qm9_2d(bs, 700 + bs, f)
    net = CCN_2D(f, 2, h, layers)
    fu.det_init(net, 93 + layers)
    p64 = {n: v.detach().double().clone().requires_grad_(True) for n, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = _pad(graphs, "cuda")
    assert net._spec().small(X.shape[0], X.shape[1]) is not None
    w = torch.randn(bs, 2, generator=torch.Generator().manual_seed(bs)).cuda()
    os_, dxs, gs = _run_path(True, net, X, A, nb, w)
    og, dxg, gg = _run_path(False, net, X, A, nb, w)
    assert torch.equal(os_, og), f"outputs differ: {(os_ - og).abs().max().item():.3g}"
    assert torch.equal(dxs, dxg), f"dX differs: {(dxs - dxg).abs().max().item():.3g}"
    for n in gg:
        assert torch.equal(gs[n], gg[n]), f"grad {n} differs: {(gs[n] - gg[n]).abs().max().item():.3g}"
    for b, (x, a, _) in enumerate(graphs[:6]):
        xr = x.double().requires_grad_(True)
        ref = RC.ccn2_forward_closed(p64, xr, a.double(), layers)
        _close(os_[b], ref, f"small path graph {b}")
        (ref * w[b].double().cpu()).sum().backward()
        _grad_close(dxs[b, :x.shape[0]], xr.grad, f"small path dX graph {b}")
        assert dxs[b, x.shape[0]:].abs().max().item() == 0.0 if x.shape[0] < X.shape[1] else True


def test_ccn2_small_graph_path_fixtures(golden):
    """The reference's CCN_2D fixtures (tests/golden/ccn.npz, generated from the reference) through the
    small path, per graph as scripts/train_ccn.py calls it, and bit-identical to the general path."""
    import hgnn_amd.ccn as HC
    z = golden("ccn")
    seen = 0
    for k, (X, adj, t) in enumerate(ccn_graphs(z)):
        if f"2d_out_{k}" not in z:
            continue
        net, _ = ccn_params("2d", k)
        net = net.cuda()
        assert net._spec().small(1, X.shape[0]) is not None
        res = {}
        for small in (True, False):
            old = HC.SMALL
            HC.SMALL = small
            try:
                net.zero_grad(set_to_none=True)
                Xr = X.cuda().requires_grad_(True)
                out = net(Xr, adj.cuda())
                torch.nn.MSELoss()(out, t[0].view(1).cuda()).backward()
                res[small] = (out.detach().cpu(), Xr.grad.cpu(),
                              {n: p.grad.detach().cpu().clone() for n, p in net.named_parameters()})
            finally:
                HC.SMALL = old
        out, dx, gr = res[True]
        _close(out, z[f"2d_out_{k}"], f"2d out {k}")
        _grad_close(dx, z[f"2d_dX_{k}"], f"2d dX {k}")
        for n, g in gr.items():
            _grad_close(g, z[f"2d_grad_{k}.{n}"], f"2d grad {k} {n}")
        assert torch.equal(out, res[False][0]) and torch.equal(dx, res[False][1]), k
        for n in gr:
            assert torch.equal(gr[n], res[False][2][n]), (k, n)
        seen += 1
    assert seen > 0


def test_ccn2_small_graph_path_complete_graph_nmax32():
    """The size bound of the small path: a complete 32-node graph (every receptive field of degree 32, the
    position maps and P at their largest) equals the general path and the closed-form oracle."""
    from models.compnets.model_ccn import CCN_2D
    from oracle import ref_ccn as RC
    n = 32
    g = torch.Generator().manual_seed(32)
    x = torch.rand(n, 5, generator=g)
    a = torch.ones(n, n)
    net = CCN_2D(5, 1, 2, 2)
    fu.det_init(net, 32)
    p64 = {k: v.detach().double().clone().requires_grad_(True) for k, v in net.named_parameters()}
    net = net.cuda()
    X, A, nb = x.view(1, n, 5).cuda(), a.view(1, n, n).cuda(), torch.tensor([n]).cuda()
    assert net._spec().small(1, n) is not None
    w = torch.ones(1, 1).cuda()
    os_, dxs, gs = _run_path(True, net, X, A, nb, w)
    og, dxg, gg = _run_path(False, net, X, A, nb, w)
    assert torch.equal(os_, og) and torch.equal(dxs, dxg)
    for k in gg:
        assert torch.equal(gs[k], gg[k]), k
    xr = x.double().requires_grad_(True)
    ref = RC.ccn2_forward_closed(p64, xr, a.double(), 2)
    _close(os_[0], ref, "complete graph")
    ref.sum().backward()
    _grad_close(dxs[0], xr.grad, "complete graph dX")


def test_ccn2_small_graph_path_ragged_and_validation():
    """Ragged batch (single node, empty slot, QM9 graph) equals the general path, the empty slot reads
    fc.bias; the small path reports missing self loops / asymmetric patterns / n_b > nmax."""
    from hgnn_amd.net import check_errors
    from models.compnets.model_ccn import CCN_2D
    (xq, aq, _), = _qm9_2d(1, 19)
    n = xq.shape[0]
    X = torch.zeros(3, n, 5)
    A = torch.zeros(3, n, n)
    X[0, :1] = torch.randn(1, 5)
    A[0, 0, 0] = 1.0
    X[2, :n] = xq
    A[2, :n, :n] = aq
    nb = torch.tensor([1, 0, n], dtype=torch.int64)
    net = CCN_2D(5, 1, 2, 2)
    fu.det_init(net, 919)
    net = net.cuda()
    X, A, nb = X.cuda(), A.cuda(), nb.cuda()
    w = torch.ones(3, 1).cuda()
    os_, dxs, gs = _run_path(True, net, X, A, nb, w)
    og, dxg, gg = _run_path(False, net, X, A, nb, w)
    assert torch.equal(os_, og) and torch.equal(dxs, dxg)
    for k in gg:
        assert torch.equal(gs[k], gg[k]), k
    assert torch.equal(os_[1], net.fc.bias.detach().cpu())
    assert dxs[1].abs().max().item() == 0.0 and dxs[0, 1:].abs().max().item() == 0.0
    A1 = torch.eye(4)
    A1[0, 1] = 1.0  # 1 does not list 0
    with pytest.raises(RuntimeError, match="not symmetric"):
        net(torch.randn(4, 5).cuda(), A1.cuda())
        check_errors()
    A2 = torch.ones(4, 4)
    A2[2, 2] = 0.0
    with pytest.raises(RuntimeError, match="self loop"):
        net(torch.randn(4, 5).cuda(), A2.cuda())
        check_errors()
    with pytest.raises(RuntimeError, match="negative count"):
        net.forward_batch(torch.randn(1, 4, 5).cuda(), torch.eye(4).unsqueeze(0).cuda(), torch.tensor([5]).cuda())
        check_errors()
    net(torch.randn(4, 5).cuda(), torch.eye(4).cuda())
    check_errors()


def test_ccn2_small_graph_path_inplace_input_change_raises():
    """The small path's backward re-plans from adj and reads X: both saved through autograd, so an in-place
    change between forward and backward raises the version error."""
    from models.compnets.model_ccn import CCN_2D
    (x, a, _), = _qm9_2d(1, 23)
    net = CCN_2D(5, 1, 2, 2).cuda()
    X = x.cuda().requires_grad_(True)
    Xi = X * 1.0
    out = net(Xi, a.cuda())
    assert net._spec().small(1, x.shape[0]) is not None
    with torch.no_grad():
        Xi.add_(1.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        out.sum().backward()
