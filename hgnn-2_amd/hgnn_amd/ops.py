"""Autograd wrappers of the layer-level dense ops (graph_oper, P_multi, BN, 1x1 conv).

These serve the reference's layer-level API (layers used one at a time on the
dense padded tensors).  GNN_lg / GNN_simple do not go through here: they use
the fused network executor (hgnn_amd.net).  Every op requires CUDA tensors and
raises otherwise; there is no CPU path.
"""

import ctypes

import torch

from . import _lib as L


def _cuda(*ts, what):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError(f"hgnn_amd: {what} runs on the GPU only (got a CPU tensor)")


def _c(t):
    return t.contiguous().to(torch.float32)


def _stream(t):
    return L.stream_handle(t.device)


class _GraphOper(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A, X):
        A, X = _c(A), _c(X)
        bs, n, _, j = A.shape
        f = X.shape[1]
        out = torch.empty(bs, j * f, n, device=X.device, dtype=torch.float32)
        L.check(L.lib().hgnn_graph_oper_forward(L.ptr(A), L.ptr(X), L.ptr(out), bs, n, j, f, _stream(X)),
                "graph_oper forward")
        ctx.save_for_backward(A, X)
        return out

    @staticmethod
    def backward(ctx, dout):
        A, X = ctx.saved_tensors
        dout = _c(dout)
        bs, n, _, j = A.shape
        f = X.shape[1]
        dX = torch.empty_like(X) if ctx.needs_input_grad[1] else None
        dA = torch.empty_like(A) if ctx.needs_input_grad[0] else None
        if dX is None and dA is None:
            return None, None
        dXp = dX if dX is not None else torch.empty_like(X)
        L.check(L.lib().hgnn_graph_oper_backward(L.ptr(A), L.ptr(X), L.ptr(dout), L.ptr(dXp), L.ptr(dA), bs, n, j,
                                                 f, _stream(X)), "graph_oper backward")
        return dA, dX


def graph_oper(A, X):
    """out[b, j*F + f, n] = sum_m A[b, n, m, j] X[b, f, m]  (layers_mnb.py:395-411)."""
    _cuda(A, X, what="graph_oper")
    if A.dim() != 4 or X.dim() != 3 or A.shape[0] != X.shape[0] or A.shape[1] != A.shape[2] or A.shape[1] != X.shape[2]:
        raise RuntimeError(f"graph_oper: shapes A {tuple(A.shape)} and X {tuple(X.shape)} do not match")
    return _GraphOper.apply(A, X)


class _PMulti(torch.autograd.Function):
    @staticmethod
    def forward(ctx, P, X):
        X = _c(X)
        if P.dtype != torch.float32:
            P = P.to(torch.float32)
        bs, n, m = P.shape
        f = X.shape[1]
        sb, sn, sm = P.stride()
        out = torch.empty(bs, f, n, device=X.device, dtype=torch.float32)
        L.check(L.lib().hgnn_p_multi_forward(L.ptr(P), sb, sn, sm, L.ptr(X), L.ptr(out), bs, n, m, f, _stream(X)),
                "P_multi forward")
        ctx.save_for_backward(P, X)
        return out

    @staticmethod
    def backward(ctx, dout):
        P, X = ctx.saved_tensors
        dout = _c(dout)
        bs, n, m = P.shape
        f = X.shape[1]
        sb, sn, sm = P.stride()
        dX = torch.empty_like(X)
        dP = torch.empty(bs, n, m, device=X.device, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        L.check(L.lib().hgnn_p_multi_backward(L.ptr(P), sb, sn, sm, L.ptr(X), L.ptr(dout), L.ptr(dX), L.ptr(dP), bs,
                                              n, m, f, _stream(X)), "P_multi backward")
        return dP, (dX if ctx.needs_input_grad[1] else None)


def p_multi(P, X):
    """out[b, f, n] = sum_m P[b, n, m] X[b, f, m]  (layers_mnb.py:418-434); P may be a transposed view."""
    _cuda(P, X, what="P_multi")
    if P.dim() != 3 or X.dim() != 3 or P.shape[0] != X.shape[0] or P.shape[2] != X.shape[2]:
        raise RuntimeError(f"P_multi: shapes P {tuple(P.shape)} and X {tuple(X.shape)} do not match")
    return _PMulti.apply(P, X)


class _BN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, w, b, Nb, mask, mean, std):
        X = _c(X)
        mask = _c(mask)
        Nb = Nb.to(torch.int64).contiguous()
        bs, c, n = X.shape
        training = mean is None
        if training:
            mean = torch.empty(c, device=X.device, dtype=torch.float32)
            std = torch.empty(c, device=X.device, dtype=torch.float32)
        else:
            mean, std = _c(mean), _c(std)
        w32, b32 = _c(w), _c(b)
        out = torch.empty_like(X)
        L.check(L.lib().hgnn_bn_forward(L.ptr(X), L.ptr(Nb), L.ptr(mask), L.ptr(w32), L.ptr(b32), L.ptr(mean),
                                        L.ptr(std), L.ptr(out), bs, c, n, 1 if training else 0, _stream(X)),
                "BN forward")
        ctx.save_for_backward(X, Nb, mask, w32, mean, std)
        ctx.training = training
        ctx.mark_non_differentiable(mean, std)
        return out, mean, std

    @staticmethod
    def backward(ctx, dout, _dm, _ds):
        X, Nb, mask, w32, mean, std = ctx.saved_tensors
        bs, c, n = X.shape
        dout = _c(dout)
        dX = torch.empty_like(X)
        dw = torch.empty((), device=X.device, dtype=torch.float32)
        db = torch.empty((), device=X.device, dtype=torch.float32)
        scratch = torch.empty(2 * c, device=X.device, dtype=torch.float32)
        L.check(L.lib().hgnn_bn_backward(L.ptr(X), L.ptr(Nb), L.ptr(mask), L.ptr(w32), L.ptr(mean), L.ptr(std),
                                         L.ptr(dout), L.ptr(dX), L.ptr(dw), L.ptr(db), L.ptr(scratch), bs, c, n,
                                         1 if ctx.training else 0, _stream(X)), "BN backward")
        return dX, dw, db, None, None, None, None


def bn(X, N_batch, mask, w, b, mean=None, std=None):
    """BN of batch_normalization.py:34-43 -> (out, mean, std); batch statistics when mean is None."""
    _cuda(X, mask, w, b, what="BN")
    if not N_batch.is_cuda:
        N_batch = N_batch.to(X.device)
    if X.dim() != 3 or mask.shape != (X.shape[0], X.shape[2], X.shape[2]):
        raise RuntimeError(f"BN: X {tuple(X.shape)} and mask {tuple(mask.shape)} do not match")
    return _BN.apply(X, w, b, N_batch, mask, mean, std)


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu):
        x = _c(x)
        cout, cin = w.shape[0], w.shape[1]
        w2 = _c(w.reshape(cout, cin))
        b2 = _c(b)
        bs, _, n = x.shape
        nbytes = L.lib().hgnn_conv1x1_workspace_bytes(bs, cin, cout, n)
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=x.device)
        y = torch.empty(bs, cout, n, device=x.device, dtype=torch.float32)
        L.check(L.lib().hgnn_conv1x1_forward(L.ptr(x), L.ptr(w2), L.ptr(b2), L.ptr(y), bs, cin, cout, n,
                                             1 if relu else 0, ctypes.c_void_p(ws.data_ptr()), _stream(x)),
                "conv1x1 forward")
        ctx.save_for_backward(x, w2, y)
        ctx.relu = relu
        ctx.wshape = w.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w2, y = ctx.saved_tensors
        dy = _c(dy)
        if ctx.relu:
            dy = dy * (y > 0)
        bs, cin, n = x.shape
        cout = w2.shape[0]
        nbytes = L.lib().hgnn_conv1x1_workspace_bytes(bs, cin, cout, n)
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=x.device)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty(cout, cin, device=x.device, dtype=torch.float32)
        db = torch.empty(cout, device=x.device, dtype=torch.float32)
        L.check(L.lib().hgnn_conv1x1_backward(L.ptr(x), L.ptr(w2), L.ptr(dy), L.ptr(dx), L.ptr(dw), L.ptr(db), bs,
                                              cin, cout, n, ctypes.c_void_p(ws.data_ptr()), _stream(x)),
                "conv1x1 backward")
        return dx, dw.reshape(ctx.wshape), db, None


def conv1x1(x, w, b, relu=False):
    """torch.nn.Conv1d(cin, cout, 1) forward on (bs, cin, n), optional fused ReLU."""
    _cuda(x, w, b, what="Conv1d")
    return _Conv1x1.apply(x, w, b, relu)


def mask_rows(H, mask):
    """mask_embedding: H * mask[:, :, 0] broadcast over features (batch_normalization.py:96-108)."""
    _cuda(H, mask, what="mask_embedding")
    bs, n = mask.shape[0], mask.shape[1]
    return H * mask[:, :, 0].reshape(bs, 1, n)


def masked_mean(H, N_batch, mask):
    """mean_with_padding: sum over (b, n) of H * mask[:, :, 0] / sum(N_batch) (batch_normalization.py:80-93)."""
    _cuda(H, mask, what="mean_with_padding")
    return mask_rows(H, mask).sum(dim=2).sum(dim=0) / N_batch.sum().item()
