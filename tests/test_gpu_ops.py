"""GPU parity of the layer-level drop-ins: graph_oper, P_multi, BN, Conv1d and the layer modules."""

import numpy as np
import pytest
import torch

import fixture_util as fu
from oracle import parity as PP
from oracle import ref_mnb as R

pytestmark = pytest.mark.gpu


def _layers_batch(golden):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    z = golden("layers")
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in fu.unpack_graphs(z)]
    return z, list(prepare_batch(data, 0, 1))


def test_graph_oper_and_p_multi_match_reference(golden):
    from models.layers.layers_mnb import graph_oper, P_multi
    from functions.utils import graph_op, Pmul
    z, b = _layers_batch(golden)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cuda() for t in b]
    Xf = torch.from_numpy(z["Xf"]).cuda()
    XLf = torch.from_numpy(z["XLf"]).cuda()
    for fn in (graph_oper(), graph_op):
        np.testing.assert_allclose(fn(W, Xf).cpu().numpy(), z["gop_W"], rtol=1e-6, atol=1e-5)
        np.testing.assert_allclose(fn(WL, XLf).cpu().numpy(), z["gop_WL"], rtol=1e-6, atol=1e-5)
    for fn in (P_multi(), Pmul):
        np.testing.assert_allclose(fn(Pm, XLf).cpu().numpy(), z["pm_XL"], rtol=1e-6, atol=1e-5)
        np.testing.assert_allclose(fn(Pd.transpose(2, 1), Xf).cpu().numpy(), z["pdT_X"], rtol=1e-6, atol=1e-5)


def test_graph_oper_p_multi_backward_vs_oracle(golden):
    from models.layers.layers_mnb import graph_oper, P_multi
    z, b = _layers_batch(golden)
    W, Pm = b[1], b[5]
    Xf = torch.from_numpy(z["Xf"]).double()
    XLf = torch.from_numpy(z["XLf"]).double()
    g = torch.Generator().manual_seed(3)
    for kind in ("gop", "pmT"):
        A = (W if kind == "gop" else Pm).double().requires_grad_(True)
        x = (Xf if kind == "gop" else Xf).clone().requires_grad_(True)
        if kind == "gop":
            ref = R.graph_oper(A, x)
        else:
            ref = R.p_multi(A.transpose(2, 1), x)
        up = torch.randn(ref.shape, generator=g, dtype=torch.float64)
        (ref * up).sum().backward()
        Ag = A.detach().float().cuda().requires_grad_(True)
        xg = x.detach().float().cuda().requires_grad_(True)
        out = graph_oper()(Ag, xg) if kind == "gop" else P_multi()(Ag.transpose(2, 1), xg)
        (out * up.float().cuda()).sum().backward()
        np.testing.assert_allclose(out.detach().cpu().double().numpy(), ref.detach().numpy(), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(xg.grad.cpu().double().numpy(), x.grad.numpy(), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(Ag.grad.cpu().double().numpy(), A.grad.numpy(), rtol=1e-4, atol=1e-4)
    del XLf


def test_bn_train_eval_match_reference(golden):
    from models.layers.batch_normalization import BN
    z, b = _layers_batch(golden)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cuda() for t in b]
    Xf = torch.from_numpy(z["Xf"]).cuda()
    bn = BN(Xf.shape[1]).cuda()
    with torch.no_grad():
        bn.weight.fill_(0.7)
        bn.bias.fill_(-0.2)
    bn.train()
    out = bn(Xf, Nb, mask)
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["bn_train"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(bn.running_mean.cpu().numpy(), z["bn_rmean"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(bn.running_std.cpu().numpy(), z["bn_rstd"], rtol=1e-5, atol=1e-6)
    bn.eval()
    out = bn(Xf * 0.5 + 0.1, Nb, mask)
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["bn_eval"], rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("training", [True, False])
def test_bn_backward_vs_oracle(golden, training):
    from models.layers.batch_normalization import BN
    z, b = _layers_batch(golden)
    Nb, mask = b[9], b[7]
    Xf = torch.from_numpy(z["Xf"]).double().requires_grad_(True)
    st = {"running_mean": torch.linspace(-0.3, 0.3, Xf.shape[1]).double(),
          "running_std": torch.linspace(0.5, 1.5, Xf.shape[1]).double()}
    w = torch.tensor(0.8, dtype=torch.float64, requires_grad=True)
    bb = torch.tensor(0.1, dtype=torch.float64, requires_grad=True)
    ref = R.bn(Xf, Nb, mask.double(), w, bb, dict(st), training)
    up = torch.randn(ref.shape, generator=torch.Generator().manual_seed(5), dtype=torch.float64)
    (ref * up).sum().backward()
    bn = BN(Xf.shape[1]).cuda()
    with torch.no_grad():
        bn.weight.fill_(0.8)
        bn.bias.fill_(0.1)
    bn.running_mean = st["running_mean"].float().cuda()
    bn.running_std = st["running_std"].float().cuda()
    bn.train(training)
    xg = Xf.detach().float().cuda().requires_grad_(True)
    out = bn(xg, Nb.cuda(), mask.cuda())
    (out * up.float().cuda()).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().double().numpy(), ref.detach().numpy(), rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(xg.grad.cpu().double().numpy(), Xf.grad.numpy(), rtol=1e-4, atol=1e-4)
    assert abs(bn.weight.grad.item() - w.grad.item()) <= 1e-4 * max(1.0, abs(w.grad.item()))
    assert abs(bn.bias.grad.item() - bb.grad.item()) <= 1e-4 * max(1.0, abs(bb.grad.item()))


@pytest.mark.parametrize("cin,cout,n", [(640, 64, 70), (13, 64, 29), (271, 64, 29), (12, 2, 50)])
def test_conv1x1_vs_torch_fp32(cin, cout, n):
    """The Conv1d GEMM against a plain PyTorch fp32 reference of the same op."""
    from hgnn_amd import ops
    g = torch.Generator().manual_seed(cin)
    x = torch.randn(7, cin, n, generator=g).cuda().requires_grad_(True)
    w = (0.1 * torch.randn(cout, cin, 1, generator=g)).cuda().requires_grad_(True)
    bias = (0.1 * torch.randn(cout, generator=g)).cuda().requires_grad_(True)
    for relu in (False, True):
        y = ops.conv1x1(x, w, bias, relu=relu)
        x2 = x.detach().double().requires_grad_(True)
        w2 = w.detach().double().requires_grad_(True)
        b2 = bias.detach().double().requires_grad_(True)
        ref = torch.nn.functional.conv1d(x2, w2, b2)
        if relu:
            ref = torch.relu(ref)
        up = torch.randn(ref.shape, generator=g, dtype=torch.float64)
        (y * up.float().cuda()).sum().backward()
        (ref * up.cuda()).sum().backward()
        tol = 1e-5 * max(1.0, ref.abs().max().item())
        assert (y.double() - ref).abs().max().item() <= 2 * tol
        assert (x.grad.double() - x2.grad).abs().max().item() <= 1e-4 * max(1.0, x2.grad.abs().max().item())
        assert (w.grad.double() - w2.grad).abs().max().item() <= 1e-4 * max(1.0, w2.grad.abs().max().item())
        assert (bias.grad.double() - b2.grad).abs().max().item() <= 1e-4 * max(1.0, b2.grad.abs().max().item())
        x.grad = w.grad = bias.grad = None


@pytest.mark.parametrize("order", [1, 2, 3])
def test_layer_with_lg_modules_vs_oracle(order):
    """layer_with_lg_{1,2,3} used one at a time (layer-level API) against the oracle."""
    import hgnn_amd.datagen as dg
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    from models.layers import layers_mnb as Lm
    graphs = dg.qm9_shape_dataset(12, seed=17)
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    b = list(prepare_batch(data, 0, 1))
    cls = {1: Lm.layer_with_lg_1, 2: Lm.layer_with_lg_2, 3: Lm.layer_with_lg_3}[order]
    layer = cls([5, 1, 8], 3).cuda()
    fu.det_init(layer, 31 + order)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = b

    def oracle(dtype, grads):
        p = {"layer0." + k: v.detach().cpu().to(dtype).requires_grad_(grads) for k, v in layer.state_dict().items()}
        st = R.bn_states(2, 16, dtype=dtype)
        Xd = X.to(dtype).requires_grad_(grads)
        args = (p, "layer0.")
        c = lambda t: t.to(dtype)  # noqa: E731
        with torch.set_grad_enabled(grads):
            if order == 1:
                Z = R._lg_node(*args, Xd, c(XL), c(W), c(Pm), c(Pd), Nb, c(mask), st, True)
                ZL = R._lg_edge(*args, c(XL), Z, c(WL), c(Pm), c(Pd), Eb, c(mask_lg), st, True)
            elif order == 2:
                ZL = R._lg_edge(*args, c(XL), Xd, c(WL), c(Pm), c(Pd), Eb, c(mask_lg), st, True)
                Z = R._lg_node(*args, Xd, ZL, c(W), c(Pm), c(Pd), Nb, c(mask), st, True)
            else:
                Z = R._lg_node(*args, Xd, c(XL), c(W), c(Pm), c(Pd), Nb, c(mask), st, True)
                ZL = R._lg_edge(*args, c(XL), Xd, c(WL), c(Pm), c(Pd), Eb, c(mask_lg), st, True)
        return p, Xd, Z, ZL

    p, Xd, Z, ZL = oracle(torch.float64, True)
    _, _, Z32, ZL32 = oracle(torch.float32, False)
    g = torch.Generator().manual_seed(order)
    u1 = torch.randn(Z.shape, generator=g, dtype=torch.float64)
    u2 = torch.randn(ZL.shape, generator=g, dtype=torch.float64)
    ((Z * u1).sum() + (ZL * u2).sum()).backward()
    Xg = X.cuda().requires_grad_(True)
    z, zl, *_ = layer([Xg, XL.cuda(), W.cuda(), WL.cuda(), Pm.cuda(), Pd.cuda()], Nb.cuda(), mask.cuda(),
                      Eb.cuda(), mask_lg.cuda())
    ((z * u1.float().cuda()).sum() + (zl * u2.float().cuda()).sum()).backward()
    # SURVEY §8 c two-leg output bound on both halves' BN outputs (padded slots included)
    for got, r32, r64 in ((z, Z32, Z), (zl, ZL32, ZL)):
        o = PP.outputs_two_leg(got, r32, r64.detach())
        assert o["pass"], o
    gmax = max(v.grad.abs().max().item() for v in p.values())
    for k, v in layer.named_parameters():
        ref = p["layer0." + k].grad
        assert (v.grad.cpu().double() - ref).abs().max().item() <= 1e-4 * gmax + 1e-5 * ref.abs().max().item(), k
    assert (Xg.grad.cpu().double() - Xd.grad).abs().max().item() <= 1e-4 * max(1.0, Xd.grad.abs().max().item())
