"""The torch.library registrations (hgnn_amd.library) on CPU: schemas exist and the fake
(meta) implementations propagate shapes -- including the workspace size, from the C ABI's
host-only query -- so FakeTensor tracing needs no GPU."""

import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import hgnn_amd.library  # noqa: F401  (registers the operators)
from hgnn_amd import _lib as L


def _fake_inputs(bs=8, n=12, e=20, jt=3):
    X = torch.empty(bs, 1, n)
    W = torch.empty(bs, n, n, jt)
    XL = torch.empty(bs, 1, e)
    WL = torch.empty(bs, e, e, jt)
    Pm = torch.empty(bs, n, e)
    Pd = torch.empty(bs, n, e)
    Nb = torch.empty(bs, dtype=torch.int64)
    mask = torch.empty(bs, n)
    Eb = torch.empty(bs, dtype=torch.int64)
    mask_lg = torch.empty(bs, e)
    return X, W, Nb, mask, XL, WL, Pm, Pd, Eb, mask_lg


def test_schemas_registered():
    assert "running" in str(torch.ops.hgnn_amd.net_forward.default._schema)
    assert "need_dw" in str(torch.ops.hgnn_amd.net_backward.default._schema)


def test_fake_shapes_match_workspace_query():
    with FakeTensorMode():
        X, W, Nb, mask, XL, WL, Pm, Pd, Eb, mask_lg = _fake_inputs()
        params = [torch.empty(3), torch.empty(7)]
        running = [torch.empty(5)]
        out, ws, run2 = torch.ops.hgnn_amd.net_forward(X, W, Nb, mask, XL, WL, Pm, Pd, Eb, mask_lg, params,
                                                       running, 1, 2, 16, 3, 2, True)
        dX, dW, grads = torch.ops.hgnn_amd.net_backward(out, ws, X, W, Nb, mask, XL, WL, Pm, Pd, Eb, mask_lg,
                                                        params, 1, 2, 16, 3, 2, True, True, False)
    assert tuple(out.shape) == (8, 2) and ws.dtype == torch.uint8
    assert [tuple(t.shape) for t in run2] == [(5,)]
    assert tuple(dX.shape) == (8, 1, 12) and dW.numel() == 0
    assert [tuple(g.shape) for g in grads] == [(3,), (7,)]
    cfg = L.NetConfig()
    cfg.kind, cfg.order, cfg.bs, cfg.nmax, cfg.emax, cfg.f_in = 1, 2, 8, 12, 20, 1
    cfg.d, cfg.n_layers, cfg.j_tot, cfg.dim_out, cfg.training = 16, 3, 3, 2, 1
    import ctypes
    assert ws.numel() == L.lib().hgnn_net_workspace_bytes(ctypes.byref(cfg))
