"""torch.library operators of the executor (hgnn_amd.library): the registered
hgnn_amd::net_forward / net_backward compute exactly what the autograd.Function path
computes (same kernels, same order), and torch.compile traces the drop-in modules
through them (aot_eager backend: AOTAutograd builds the joint forward/backward graph
around the opaque operators; no code generation)."""

import copy

import pytest
import torch

import fixture_util as fu
from hgnn_amd.dp import running_stats

pytestmark = pytest.mark.gpu


def _batch(graphs):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    return [t.cuda() for t in prepare_batch(data, 0, 1)]


def _model(kind):
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg, GNN_simple
    if kind == "simple":
        b = _batch(dg.sbm_dataset(8, n=30, seed=21))
        model = GNN_simple(0, 4, 5, 5, 1, 1).cuda()
    else:
        b = _batch(dg.qm9_shape_dataset(48, seed=22))
        model = GNN_lg(0, 16, 4, 5, 1, 1, 2).cuda()
    fu.det_init(model, 23)
    return model, b


def _step(model, b, kind, fn=None):
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.clone() for t in b]
    X.requires_grad_(True)
    W.requires_grad_(True)
    fn = model if fn is None else fn
    out = fn([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg) if kind == "lg" else fn([X, W], Nb, mask)
    loss = torch.nn.MSELoss()(out, T)
    loss.backward()
    torch.cuda.synchronize()
    return (out.detach(), [p.grad.clone() for p in model.parameters()], X.grad, W.grad,
            [t.clone() for t in running_stats(model)])


def _equal(a, b):
    out_a, g_a, dx_a, dw_a, r_a = a
    out_b, g_b, dx_b, dw_b, r_b = b
    assert torch.equal(out_a, out_b)
    assert all(torch.equal(x, y) for x, y in zip(g_a, g_b))
    assert torch.equal(dx_a, dx_b) and torch.equal(dw_a, dw_b)
    assert all(torch.equal(x, y) for x, y in zip(r_a, r_b))


@pytest.mark.parametrize("kind", ["simple", "lg"])
def test_torch_ops_path_equals_function_path(monkeypatch, kind):
    model, b = _model(kind)
    twin = copy.deepcopy(model)
    monkeypatch.setenv("HGNN_TORCH_OPS", "0")
    ref = _step(model, b, kind)
    monkeypatch.setenv("HGNN_TORCH_OPS", "1")
    got = _step(twin, b, kind)
    _equal(ref, got)
    # eval mode: running statistics read, not written
    model.eval()
    twin.eval()
    monkeypatch.setenv("HGNN_TORCH_OPS", "0")
    ref = _step(model, b, kind)
    monkeypatch.setenv("HGNN_TORCH_OPS", "1")
    got = _step(twin, b, kind)
    _equal(ref, got)


@pytest.mark.parametrize("kind", ["simple", "lg"])
def test_torch_compile_traces_the_operators(monkeypatch, kind):
    from torch._dynamo.backends.registry import lookup_backend
    monkeypatch.setenv("HGNN_TORCH_OPS", "0")
    torch._dynamo.reset()
    model, b = _model(kind)
    twin = copy.deepcopy(model)
    ref = _step(model, b, kind)
    graphs = []

    def recording(gm, example_inputs):
        graphs.append(str(gm.graph))
        return lookup_backend("aot_eager")(gm, example_inputs)

    compiled = torch.compile(twin, backend=recording)
    got = _step(twin, b, kind, fn=compiled)
    _equal(ref, got)
    assert any("hgnn_amd.net_forward" in g for g in graphs), graphs
