"""GPU parity of the network executor (GNN_lg / GNN_simple) against the reference.

Checks against (a) the golden fixtures recorded from /root/reference and (b)
the oracle (oracle/ref_mnb.py, fp64) at larger batches, plus size-independent
properties at the benchmark size.  Tolerances (SURVEY.md §8 c):
  outputs   |d| <= 1e-5 * max(1, max|ref32|)  and  |gpu - ref64| <= 2 |ref32 - ref64| + 1e-6
  gradients |d| <= 1e-4 * max_global|g| + 1e-5 |g|   (global floor: cv2/cv4 bias grads are 0)
"""

import os

import numpy as np
import pytest
import torch

import fixture_util as fu
from oracle import parity as PP
from oracle import ref_mnb as R

pytestmark = pytest.mark.gpu

LG_CASES = ["lg_d16_o1", "lg_d16_o2", "lg_d16_o3", "lg_d8_o2_L2", "lg_d16_o2_L3", "lg_d64_o2"]


def _batch(graphs, J=1):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    data = [[X, A, t, *graph_operators([X, A], J, True)] for X, A, t in graphs]
    return list(prepare_batch(data, 0, J))


def _cuda(b):
    return [t.cuda() for t in b]


def _check_grads(named_grads, ref, prefix="grad."):
    gmax = max(np.abs(ref[k]).max() for k in ref.files if k.startswith(prefix))
    n = 0
    for k in ref.files:
        if not k.startswith(prefix):
            continue
        g = named_grads[k[len(prefix):]]
        assert g is not None, k
        g = g.detach().cpu().numpy()
        err = np.abs(g - ref[k])
        bound = 1e-4 * gmax + 1e-5 * np.abs(ref[k])
        assert np.all(err <= bound), (k, float(err.max()), float(gmax))
        n += 1
    assert n > 0


@pytest.mark.parametrize("name", LG_CASES)
def test_gnn_lg_matches_reference_fixture(golden, name):
    from models.gnns.model_mnb import GNN_lg
    z = golden(name)
    d, L, order, bs, wseed = [int(v) for v in z["cfg"]]
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(_batch(fu.unpack_graphs(z)))
    model = GNN_lg(0, d, L, 5, 1, 1, order).cuda()
    fu.det_init(model, wseed)
    model.train()
    X.requires_grad_(True)
    W.requires_grad_(True)  # as scripts/train_mnb.py:56-57: the reference materialises W.grad
    out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    loss = torch.nn.MSELoss()(out, T)
    loss.backward()
    torch.cuda.synchronize()
    dw = W.grad.cpu().numpy()
    assert np.max(np.abs(dw - z["dW"])) <= 1e-4 * max(1.0, np.abs(z["dW"]).max()) + 1e-6
    o = out.detach().cpu().numpy()
    ref, ref64 = z["out"], z["out64"]
    assert np.max(np.abs(o - ref)) <= 1e-5 * max(1.0, np.abs(ref).max())
    assert np.max(np.abs(o - ref64)) <= 2 * np.max(np.abs(ref - ref64)) + 1e-6
    assert abs(loss.item() - float(z["loss"])) <= 1e-5 * max(1.0, abs(float(z["loss"])))
    _check_grads({k: p.grad for k, p in model.named_parameters()}, z)
    dx = X.grad.cpu().numpy()
    assert np.max(np.abs(dx - z["dX"])) <= 1e-4 * max(1.0, np.abs(z["dX"]).max()) + 1e-6
    for l in range(L - 1):
        layer = model.layer0 if l == 0 else getattr(model, f"layer{l}")
        for nm in ("bn1", "bn2"):
            bn = getattr(layer, nm)
            np.testing.assert_allclose(bn.running_mean.cpu().numpy(), z[f"rmean.layer{l}.{nm}"], rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(bn.running_std.cpu().numpy(), z[f"rstd.layer{l}.{nm}"], rtol=1e-5, atol=1e-5)
    model.eval()
    with torch.no_grad():
        oe = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg).cpu().numpy()
    assert np.max(np.abs(oe - z["out_eval"])) <= 1e-5 * max(1.0, np.abs(z["out_eval"]).max())


def test_gnn_simple_matches_reference_fixture(golden):
    from models.gnns.model_mnb import GNN_simple
    z = golden("gnn_simple")
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(_batch(fu.unpack_graphs(z)))
    model = GNN_simple(0, 2, 20, 5, 1, 1).cuda()
    fu.det_init(model, 201)
    X.requires_grad_(True)
    out = model([X, W], Nb, mask)
    loss = torch.nn.MSELoss()(out, T)
    loss.backward()
    o = out.detach().cpu().numpy()
    assert np.max(np.abs(o - z["out32"])) <= 1e-5 * max(1.0, np.abs(z["out32"]).max())
    assert np.max(np.abs(o - z["out64"])) <= 2 * np.max(np.abs(z["out32"] - z["out64"])) + 1e-6
    _check_grads({k: p.grad for k, p in model.named_parameters()}, z, prefix="grad32.")
    assert np.max(np.abs(X.grad.cpu().numpy() - z["dX32"])) <= 1e-4 * max(1.0, np.abs(z["dX32"]).max()) + 1e-6
    model.eval()
    with torch.no_grad():
        oe = model([X, W], Nb, mask).cpu().numpy()
    assert np.max(np.abs(oe - z["out_eval"])) <= 1e-5 * max(1.0, np.abs(z["out_eval"]).max())


def _oracle_lg(model, b, L, order, dtype=torch.float64, grads=True):
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cpu() for t in b]
    p = {k: v.detach().cpu().to(dtype).requires_grad_(grads) for k, v in model.state_dict().items()}
    st = R.bn_states(L, 2 * model.n_features, dtype=dtype)
    Xo = X.to(dtype).requires_grad_(grads)
    out = R.gnn_lg(p, [Xo, XL.to(dtype), W.to(dtype), WL.to(dtype), Pm.to(dtype), Pd.to(dtype)], Nb,
                   mask.to(dtype), Eb, mask_lg.to(dtype), L, order, st, True)
    loss = torch.nn.MSELoss()(out, T.to(dtype))
    if not grads:
        return out.detach(), loss.item(), None, None
    loss.backward()
    return out.detach(), loss.item(), {k: v.grad for k, v in p.items()}, Xo.grad


@pytest.mark.parametrize("order", [1, 2, 3])
def test_gnn_lg_vs_oracle_fp64_bs128(order):
    """bs=128, d=64, L=5 (config-2 model at a quarter batch) against the fp64 oracle."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    graphs = dg.qm9_shape_dataset(128, seed=1)
    b = _batch(graphs)
    model = GNN_lg(0, 64, 5, 5, 1, 1, order).cuda()
    fu.det_init(model, 77 + order)
    ref_out, ref_loss, ref_g, ref_dx = _oracle_lg(model, b, 5, order)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(b)
    X.requires_grad_(True)
    out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    loss = torch.nn.MSELoss()(out, T)
    loss.backward()
    # SURVEY §8 c two-leg output bound: the reference-order fp32 forward and the fp64 anchor
    with torch.no_grad():
        ref32 = _oracle_lg(model, b, 5, order, dtype=torch.float32, grads=False)[0]
    o = PP.outputs_two_leg(out, ref32, ref_out)
    assert o["pass"], o
    gmax = max(g.abs().max().item() for g in ref_g.values())
    for k, p in model.named_parameters():
        err = (p.grad.cpu().double() - ref_g[k]).abs()
        assert torch.all(err <= 1e-4 * gmax + 1e-5 * ref_g[k].abs()), (k, err.max().item(), gmax)
    err = (X.grad.cpu().double() - ref_dx).abs().max().item()
    assert err <= 1e-4 * max(1.0, ref_dx.abs().max().item())


@pytest.mark.parametrize("d", [2, 4, 8])
def test_gnn_simple_narrow_widths_vs_oracle_fp64(d):
    """GNN_simple at 2d = 4 / 8 / 16 channels on 24 SBM-50 graphs (1 200 node rows: several 256-row
    BN tiles), X and W requiring grad: the narrow-channel BN backward (k_bn_bwd_part2s /
    apply2s, c = 4L), the direct dense dW for F <= 16 (k_dw_dense_narrow) and the readout
    backward from R_b (k_readout_agg_bwd, k_dw_readout) against the fp64 oracle
    (model_mnb.py:58-66); outputs on the two-leg policy, every gradient incl. W.grad."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_simple
    L = 4
    b = _batch(dg.sbm_dataset(24, n=50, seed=7 + d))
    model = GNN_simple(0, d, L, 5, 1, 1).cuda()
    fu.det_init(model, 300 + d)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cpu() for t in b]

    def oracle(dtype, grads):
        p = {k: v.detach().cpu().to(dtype).requires_grad_(grads) for k, v in model.state_dict().items()}
        Xo = X.to(dtype).requires_grad_(grads)
        Wo = W.to(dtype).requires_grad_(grads)
        out = R.gnn_simple(p, [Xo, Wo], Nb, mask.to(dtype), L, R.bn_states(L, 2 * d, "simple", dtype), True)
        if grads:
            torch.nn.MSELoss()(out, T.to(dtype)).backward()
        return out.detach(), p, Xo, Wo

    ref64, p64, X64, W64 = oracle(torch.float64, True)
    with torch.no_grad():
        ref32 = oracle(torch.float32, False)[0]
    Xg, Wg, Tg, maskg, Nbg = X.cuda().requires_grad_(True), W.cuda().requires_grad_(True), T.cuda(), mask.cuda(), Nb.cuda()
    out = model([Xg, Wg], Nbg, maskg)
    torch.nn.MSELoss()(out, Tg).backward()
    o = PP.outputs_two_leg(out, ref32, ref64)
    assert o["pass"], o
    gmax = max(v.grad.abs().max().item() for v in p64.values())
    for k, prm in model.named_parameters():
        err = (prm.grad.cpu().double() - p64[k].grad).abs()
        assert torch.all(err <= 1e-4 * gmax + 1e-5 * p64[k].grad.abs()), (k, err.max().item(), gmax)
    for g, r in ((Xg.grad, X64.grad), (Wg.grad, W64.grad)):
        err = (g.cpu().double() - r).abs().max().item()
        assert err <= 1e-4 * max(1.0, r.abs().max().item()), err


def test_config2_batch_permutation_equivariance():
    """bs=512 QM9-shape (the benchmark batch): permuting the graphs permutes the outputs."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    graphs = dg.qm9_shape_dataset(512, seed=0)
    perm = torch.randperm(512, generator=torch.Generator().manual_seed(3)).tolist()
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).cuda()
    fu.det_init(model, 9)
    outs = []
    for gs in (graphs, [graphs[i] for i in perm]):
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(_batch(gs))
        with torch.no_grad():
            outs.append(model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg).cpu())
    a, b = outs
    assert torch.allclose(a[perm], b, rtol=1e-5, atol=1e-5 * max(1.0, a.abs().max().item()))
    # determinism: a second identical call is bitwise identical (no atomics in the path)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(_batch(graphs))
    with torch.no_grad():
        a2 = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg).cpu()
    assert torch.equal(a, a2)


def test_invalid_padding_and_mask_raise():
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    graphs = dg.qm9_shape_dataset(8, seed=4)
    model = GNN_lg(0, 8, 3, 5, 1, 1, 2).cuda()
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(_batch(graphs))
    i = int(torch.argmin(Nb))
    n = int(Nb[i])
    Wbad = W.clone()
    Wbad[i, n, 0, 2] = 1.0  # an entry in a padded row
    with pytest.raises(RuntimeError, match="padding"):
        model([X, XL, Wbad, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    mbad = mask.clone()
    mbad[i, n, 0] = 1.0
    with pytest.raises(RuntimeError, match="mask"):
        model([X, XL, W, WL, Pm, Pd], Nb, mbad, Eb, mask_lg)
    # the line-graph block: a padded column of a live row, the last padded element; Pm / Pd padding;
    # the line-graph mask
    e = int(Eb[i])
    for r, c, j in ((0, e, 1), (WL.shape[1] - 1, WL.shape[2] - 1, WL.shape[3] - 1)):
        WLbad = WL.clone()
        WLbad[i, r, c, j] = 0.5
        with pytest.raises(RuntimeError, match="padding"):
            model([X, XL, W, WLbad, Pm, Pd], Nb, mask, Eb, mask_lg)
    for k in range(2):
        P = (Pm, Pd)[k].clone()
        P[i, 0, e] = 1.0  # a live node row, a padded edge column
        args = [X, XL, W, WL, P, Pd] if k == 0 else [X, XL, W, WL, Pm, P]
        with pytest.raises(RuntimeError, match="padding"):
            model(args, Nb, mask, Eb, mask_lg)
    mlbad = mask_lg.clone()
    mlbad[i, e - 1, 0] = 0.0  # a live edge marked padded
    with pytest.raises(RuntimeError, match="mask"):
        model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mlbad)
    # a valid call still works afterwards
    model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)


def test_empty_line_graph_and_single_node_graphs():
    """Graphs with no bonds (M = 0) and tiny graphs mixed into one batch."""
    from models.gnns.model_mnb import GNN_lg
    g = [(torch.eye(5)[[0, 1, 2]], torch.zeros(3, 3), torch.zeros(13)),
         (torch.eye(5)[[3, 4]], torch.tensor([[0.0, 2.0], [2.0, 0.0]]), torch.ones(13))]
    import hgnn_amd.datagen as dg
    g += dg.qm9_shape_dataset(6, seed=8)
    b = _batch(g)
    model = GNN_lg(0, 16, 4, 5, 1, 1, 2).cuda()
    fu.det_init(model, 5)
    ref_out, _, ref_g, _ = _oracle_lg(model, b, 4, 2)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(b)
    out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    torch.nn.MSELoss()(out, T).backward()
    with torch.no_grad():
        ref32 = _oracle_lg(model, b, 4, 2, dtype=torch.float32, grads=False)[0]
    o = PP.outputs_two_leg(out, ref32, ref_out)
    assert o["pass"], o
    gmax = max(v.abs().max().item() for v in ref_g.values())
    for k, p in model.named_parameters():
        assert torch.all((p.grad.cpu().double() - ref_g[k]).abs() <= 1e-4 * gmax + 1e-5 * ref_g[k].abs()), k


@pytest.mark.parametrize("kind,order", [("lg", 1), ("lg", 2), ("lg", 3), ("simple", 0)])
def test_csr_batch_path_equals_dense_path(kind, order):
    """The native batcher's CSR batch (no dense operators, no extraction pass) runs the
    same kernels on the same lists: outputs, parameter grads and dX are bitwise equal."""
    import copy

    import hgnn_amd.datagen as dg
    from hgnn_amd.csr import CsrBatch
    from models.gnns.model_mnb import GNN_lg, GNN_simple
    graphs = dg.qm9_shape_dataset(96, seed=404)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(_batch(graphs))
    torch.manual_seed(5)
    model = (GNN_lg(0, 16, 4, 5, 1, 1, order) if kind == "lg" else GNN_simple(0, 8, 4, 5, 1, 1)).cuda()
    twin = copy.deepcopy(model)
    X.requires_grad_(True)
    out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg) if kind == "lg" else model([X, W], Nb, mask)
    (out * torch.linspace(-1, 1, out.numel(), device="cuda").view_as(out)).sum().backward()
    b = CsrBatch([(x, a) for x, a, _ in graphs], dual=kind == "lg")
    b.x.requires_grad_(True)
    out2 = twin.forward_csr(b)
    (out2 * torch.linspace(-1, 1, out2.numel(), device="cuda").view_as(out2)).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
    for (n, p), (_, q) in zip(model.named_parameters(), twin.named_parameters()):
        assert torch.equal(p.grad, q.grad), n
    n0 = 0
    nb = Nb.cpu().tolist()
    for g, n in enumerate(nb):
        assert torch.equal(X.grad[g, :, :n].t(), b.x.grad[n0:n0 + n]), g
        n0 += n
    # running statistics advanced identically
    for (n, m1), (_, m2) in zip(model.named_modules(), twin.named_modules()):
        if hasattr(m1, "running_mean") and torch.is_tensor(getattr(m1, "running_mean")):
            assert torch.equal(m1.running_mean.cpu(), m2.running_mean.cpu()), n


def test_gnn_lg_d128_config4_model_vs_oracle_fp64():
    """Config-4 model width (d = 128: 2d = 256 output channels, two 128-column GEMM tiles, 4-channel
    lanes in the aggregation) on a 48-graph batch against the fp64 oracle."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    graphs = dg.qm9_shape_dataset(48, seed=12)
    b = _batch(graphs)
    model = GNN_lg(0, 128, 4, 5, 1, 1, 2).cuda()
    fu.det_init(model, 128)
    ref_out, ref_loss, ref_g, ref_dx = _oracle_lg(model, b, 4, 2)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(b)
    X.requires_grad_(True)
    out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    torch.nn.MSELoss()(out, T).backward()
    with torch.no_grad():
        ref32 = _oracle_lg(model, b, 4, 2, dtype=torch.float32, grads=False)[0]
    o = PP.outputs_two_leg(out, ref32, ref_out)
    assert o["pass"], o
    gmax = max(g.abs().max().item() for g in ref_g.values())
    for k, p in model.named_parameters():
        err = (p.grad.cpu().double() - ref_g[k]).abs()
        assert torch.all(err <= 1e-4 * gmax + 1e-5 * ref_g[k].abs()), (k, err.max().item(), gmax)
    err = (X.grad.cpu().double() - ref_dx).abs().max().item()
    # the plain §8(c) bound: measured round 5 (tools/parity_margins.py, profiles/r05_parity_margins.jsonl) at
    # 0.018 of it -- the reference's own fp32 evaluation is 2.5x over it here (dX at this width is
    # ill-conditioned), the split-bf16 GEMMs are not; the round-2..4 relaxation (2x the reference's fp32
    # error) is gone
    assert err <= 1e-4 * max(1.0, ref_dx.abs().max().item()), err


@pytest.mark.parametrize("name", LG_CASES + ["gnn_simple"])
def test_csr_path_matches_reference_fixture(golden, name):
    """The CSR executor path (native batcher -> hgnn_net_forward_csr / hgnn_net_backward_csr, no
    dense operators) on the reference's fixture graphs against the reference's own recorded
    outputs, loss, parameter grads, dX, running statistics and eval outputs
    (functions/batching.py:77-185 semantics, models/gnns/model_mnb.py:58-66, 124-129)."""
    from hgnn_amd.csr import CsrBatch
    from models.gnns.model_mnb import GNN_lg, GNN_simple
    z = golden(name)
    graphs = fu.unpack_graphs(z)
    lg = name != "gnn_simple"
    if lg:
        d, L, order, bs, wseed = [int(v) for v in z["cfg"]]
        model = GNN_lg(0, d, L, 5, 1, 1, order).cuda()
        out_key, out64_key, gpref, dx_key = "out", "out64", "grad.", "dX"
    else:
        L, wseed = 20, 201
        model = GNN_simple(0, 2, L, 5, 1, 1).cuda()
        out_key, out64_key, gpref, dx_key = "out32", "out64", "grad32.", "dX32"
    fu.det_init(model, wseed)
    model.train()
    b = CsrBatch([(x, a) for x, a, _ in graphs], dual=lg, targets=torch.stack([t[0] for _, _, t in graphs]))
    b.x.requires_grad_(True)
    out = model.forward_csr(b)
    loss = torch.nn.MSELoss()(out, b.T)
    loss.backward()
    torch.cuda.synchronize()
    o = out.detach().cpu().numpy()
    ref, ref64 = z[out_key], z[out64_key]
    assert np.max(np.abs(o - ref)) <= 1e-5 * max(1.0, np.abs(ref).max())
    assert np.max(np.abs(o - ref64)) <= 2 * np.max(np.abs(ref - ref64)) + 1e-6
    lref = float(z["loss" if lg else "loss32"])
    assert abs(loss.item() - lref) <= 1e-5 * max(1.0, abs(lref))
    _check_grads({k: p.grad for k, p in model.named_parameters()}, z, prefix=gpref)
    # dX: the fixture's dense (bs, f, Nmax) gradient, packed like the CSR batch's rows
    dxr = z[dx_key]
    packed = np.concatenate([dxr[g, :, :x.shape[0]].T for g, (x, _, _) in enumerate(graphs)])
    dx = b.x.grad.cpu().numpy()
    assert dx.shape == packed.shape
    assert np.max(np.abs(dx - packed)) <= 1e-4 * max(1.0, np.abs(packed).max()) + 1e-6
    if lg:
        for l in range(L - 1):
            layer = model.layer0 if l == 0 else getattr(model, f"layer{l}")
            for nm in ("bn1", "bn2"):
                bn = getattr(layer, nm)
                np.testing.assert_allclose(bn.running_mean.cpu().numpy(), z[f"rmean.layer{l}.{nm}"], rtol=1e-5, atol=1e-5)
                np.testing.assert_allclose(bn.running_std.cpu().numpy(), z[f"rstd.layer{l}.{nm}"], rtol=1e-5, atol=1e-5)
    model.eval()
    with torch.no_grad():
        oe = model.forward_csr(b).cpu().numpy()
    assert np.max(np.abs(oe - z["out_eval"])) <= 1e-5 * max(1.0, np.abs(z["out_eval"]).max())


@pytest.mark.parametrize("J", [4, 5])
def test_large_J_vs_oracle_fp64(J):
    """J + 2 = 6 / 7 operator slices (I, D, A, A^2, .., A^(2^(J-1)); the reference takes any J,
    functions/operators.py:19-29, models/layers/layers_mnb.py:391-411): GNN_lg order 2 (d = 16,
    L = 4, 32 QM9-shape graphs, X requiring grad) and GNN_simple (d = 8, L = 3, X and
    W requiring grad, 16 sparse SBM-24 graphs) against the fp64 oracle: every gradient; outputs on the
    1e-5 relative bound (GNN_lg, whose outputs reach ~4e6) and the two-leg policy (GNN_simple)."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg, GNN_simple
    b = _batch(dg.qm9_shape_dataset(32, seed=40 + J), J)
    model = GNN_lg(0, 16, 4, 5, 1, J, 2).cuda()
    fu.det_init(model, 500 + J)
    ref_out, _, ref_g, ref_dx = _oracle_lg(model, b, 4, 2)
    with torch.no_grad():
        ref32 = _oracle_lg(model, b, 4, 2, dtype=torch.float32, grads=False)[0]
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(b)
    assert W.shape[3] == J + 2
    X.requires_grad_(True)
    out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    torch.nn.MSELoss()(out, T).backward()
    if J == 5:
        # the plain two-leg policy (measured round 5 at 0.20 of its fp64 leg, profiles/r05_parity_margins.jsonl)
        o = PP.outputs_two_leg(out.detach(), ref32, ref_out)
        assert o["pass"], o
    else:
        # J = 4: A^8 of the weighted QM9-shape adjacencies reaches ~1e8 and the outputs ~4e6; the fp64 leg
        # measured round 5 at 2.5x the strict two-leg bound.  Where it enters (round 6,
        # tools/parity_order_spread.py -> profiles/r06_parity_order_spread.txt): the reference's OWN fp32 error on
        # these 32 graphs moves 0.23x-5.52x (median 1.89x) with a mere relabelling of the nodes -- the same
        # function, only the order of the graph_oper / P_multi / BN sums changed, 5 of 12 relabellings above the
        # policy's 2x -- so the cancellation in the aggregation sums sets it, not a kernel.  The operator bits
        # are not the cause either: the builder's J = 4 operators equal the reference's own (its BLAS powers,
        # tests/golden/operators_hij.npz) in all but 27 of 407 220 entries, by 1-2 ulp
        # (test_builder.py::test_high_j_operators_vs_reference_fixture), and the fp64 and fp32 oracles here read
        # the same operator bits as the GPU.  This case keeps the north star's 1e-5 relative bound on both legs
        for ref in (ref32, ref_out):
            err = (out.detach().cpu().double() - ref.double()).abs().max().item()
            assert err <= 1e-5 * max(1.0, ref.abs().max().item()), (err, ref.abs().max().item())
    gmax = max(g.abs().max().item() for g in ref_g.values())
    for k, p in model.named_parameters():
        err = (p.grad.cpu().double() - ref_g[k]).abs()
        assert torch.all(err <= 1e-4 * gmax + 1e-5 * ref_g[k].abs()), (k, err.max().item(), gmax)
    err = (X.grad.cpu().double() - ref_dx).abs().max().item()
    assert err <= 1e-4 * max(1.0, ref_dx.abs().max().item()), err

    # sparse SBM graphs (mean degree ~2): A^16 stays ~1e5 (dense SBM-50 reaches 1e15 and W.grad 1e15,
    # where fp32 itself has no digits left to compare)
    L, d = 3, 8
    b = _batch(dg.sbm_dataset(16, n=24, seed=60 + J, p_in=0.15, p_out=0.02), J)
    model = GNN_simple(0, d, L, 5, 1, J).cuda()
    fu.det_init(model, 600 + J)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cpu() for t in b]

    def oracle(dtype, grads):
        p = {k: v.detach().cpu().to(dtype).requires_grad_(grads) for k, v in model.state_dict().items()}
        Xo = X.to(dtype).requires_grad_(grads)
        Wo = W.to(dtype).requires_grad_(grads)
        o = R.gnn_simple(p, [Xo, Wo], Nb, mask.to(dtype), L, R.bn_states(L, 2 * d, "simple", dtype), True)
        if grads:
            torch.nn.MSELoss()(o, T.to(dtype)).backward()
        return o.detach(), p, Xo, Wo

    ref64, p64, X64, W64 = oracle(torch.float64, True)
    with torch.no_grad():
        ref32 = oracle(torch.float32, False)[0]
    Xg, Wg = X.cuda().requires_grad_(True), W.cuda().requires_grad_(True)
    out = model([Xg, Wg], Nb.cuda(), mask.cuda())
    torch.nn.MSELoss()(out, T.cuda()).backward()
    o = PP.outputs_two_leg(out, ref32, ref64)
    assert o["pass"], o
    gmax = max(v.grad.abs().max().item() for v in p64.values())
    for k, prm in model.named_parameters():
        err = (prm.grad.cpu().double() - p64[k].grad).abs()
        assert torch.all(err <= 1e-4 * gmax + 1e-5 * p64[k].grad.abs()), (k, err.max().item(), gmax)
    for g, r in ((Xg.grad, X64.grad), (Wg.grad, W64.grad)):
        err = (g.cpu().double() - r).abs().max().item()
        assert err <= 1e-4 * max(1.0, r.abs().max().item()), err


@pytest.mark.gpu
@pytest.mark.parametrize("J,n", [(3, 20), (4, 18), (5, 16)])
def test_gnn_simple_small_graphs_jtot_beyond_4(J, n):
    """J_tot = J + 2 = 5..7 on graphs small enough for the register-staged extraction's size bounds
    (nmax * J_tot <= 128: ADVICE r05 -- k_extract_reg has J_tot 3 / 4 instances only, the other J_tot must
    take the LDS / global extraction): GNN_simple (d = 8, L = 3, X and W requiring grad) on 16 sparse
    SBM-n graphs against the fp64 oracle, outputs on the two-leg policy, every gradient, dX and dW."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_simple
    L, d = 3, 8
    b = _batch(dg.sbm_dataset(16, n=n, seed=70 + J, p_in=0.2, p_out=0.03), J)
    model = GNN_simple(0, d, L, 5, 1, J).cuda()
    fu.det_init(model, 700 + J)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cpu() for t in b]
    assert W.shape[3] == J + 2 and W.shape[1] * (J + 2) <= 128

    def oracle(dtype, grads):
        p = {k: v.detach().cpu().to(dtype).requires_grad_(grads) for k, v in model.state_dict().items()}
        Xo = X.to(dtype).requires_grad_(grads)
        Wo = W.to(dtype).requires_grad_(grads)
        o = R.gnn_simple(p, [Xo, Wo], Nb, mask.to(dtype), L, R.bn_states(L, 2 * d, "simple", dtype), True)
        if grads:
            torch.nn.MSELoss()(o, T.to(dtype)).backward()
        return o.detach(), p, Xo, Wo

    ref64, p64, X64, W64 = oracle(torch.float64, True)
    with torch.no_grad():
        ref32 = oracle(torch.float32, False)[0]
    Xg, Wg = X.cuda().requires_grad_(True), W.cuda().requires_grad_(True)
    out = model([Xg, Wg], Nb.cuda(), mask.cuda())
    torch.nn.MSELoss()(out, T.cuda()).backward()
    o = PP.outputs_two_leg(out, ref32, ref64)
    assert o["pass"], o
    gmax = max(v.grad.abs().max().item() for v in p64.values())
    for k, prm in model.named_parameters():
        err = (prm.grad.cpu().double() - p64[k].grad).abs()
        assert torch.all(err <= 1e-4 * gmax + 1e-5 * p64[k].grad.abs()), (k, err.max().item(), gmax)
    for g, r in ((Xg.grad, X64.grad), (Wg.grad, W64.grad)):
        err = (g.cpu().double() - r).abs().max().item()
        assert err <= 1e-4 * max(1.0, r.abs().max().item()), err


def test_offdiagonal_identity_or_degree_slice_raises():
    """The diagonal I / D columns (HGNN_DIAG_ID=1; d = 32: 2d = 64, the split-bf16 GEMMs) take operator slices 0
    and 1 as graph_operators' I and diag(D) (functions/operators.py:19-23); an off-diagonal entry in either slice
    of W or WL is reported (HGNN_DEVERR_DIAG_ID) instead of being dropped, and a valid call works afterwards.  The
    switch is read once per process: a child process runs the case."""
    import subprocess
    import sys
    env = dict(os.environ, HGNN_DIAG_ID="1", HGNN_STRICT="1")
    r = subprocess.run([sys.executable, "-c", "import conftest, test_gpu_net as T; T._offdiag_case()"], env=env,
                       cwd=os.path.dirname(os.path.abspath(__file__)), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "offdiag ok" in r.stdout


def _offdiag_case():
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    graphs = dg.qm9_shape_dataset(8, seed=5)
    model = GNN_lg(0, 32, 3, 5, 1, 1, 2).cuda()
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _cuda(_batch(graphs))
    for j in (0, 1):
        Wbad = W.clone()
        Wbad[0, 0, 1, j] = 0.25  # inside graph 0's real block, off the diagonal
        with pytest.raises(RuntimeError, match="off-diagonal"):
            model([X, XL, Wbad, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        e = int(Eb[0])
        WLbad = WL.clone()
        WLbad[0, 0, e - 1, j] = 0.25
        with pytest.raises(RuntimeError, match="off-diagonal"):
            model([X, XL, W, WLbad, Pm, Pd], Nb, mask, Eb, mask_lg)
    out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    assert torch.isfinite(out).all()
    print("offdiag ok")
