"""torch.library custom operators of the network executor (SURVEY.md §8 b).

The eager drop-in modules run hgnn_amd.net's autograd.Function.  These registrations
make the same executor calls visible to PyTorch's tracing stack -- torch.compile,
torch.export, FakeTensor shape propagation -- as two opaque operators:

  hgnn_amd::net_forward(X, W, N_batch, mask, XL?, WL?, Pm?, Pd?, E_batch?, mask_lg?,
                        params[], running[], kind, order, d, n_layers, dim_out, training)
      -> (out (bs, dim_out), workspace (uint8), running'[])
  hgnn_amd::net_backward(dout, workspace, X, W, ..., params[], ..., need_dx, need_dw)
      -> (dX, dW, grads[])

with an autograd formula tying them together (the workspace carries the forward's saved
state, exactly as in the eager path).  Both operators are functional -- an autograd formula
needs that -- so the BN running statistics come back as new tensors (running'[], updated in
training mode) that run_net_ops copies into the module's attributes.  The fake (meta) implementations size every output
from the shapes alone through the C ABI's host-only workspace query, so tracing needs no
GPU work.  GNN_simple / GNN_lg select these operators while torch.compile traces them
(torch.compiler.is_compiling()) or when HGNN_TORCH_OPS=1.
"""

import ctypes
from typing import List, Optional, Tuple

import torch

from . import _lib as L
from . import net as N

Tensor = torch.Tensor


def _cfg(kind, order, d, n_layers, dim_out, training, X, W, XL):
    # int(): symbolic shapes (torch.compile dynamic=True) specialise -- the workspace layout is a
    # host function of the exact sizes
    X, W = _Shape(X), _Shape(W)
    XL = _Shape(XL) if XL is not None else None
    cfg = L.NetConfig()
    cfg.kind = kind
    cfg.order = order
    cfg.bs = X.shape[0]
    cfg.nmax = X.shape[2]
    cfg.emax = XL.shape[2] if (kind == 1 and XL is not None) else 0
    cfg.f_in = X.shape[1]
    cfg.d = d
    cfg.n_layers = n_layers
    cfg.j_tot = W.shape[3]
    cfg.dim_out = dim_out
    cfg.training = 1 if training else 0
    return cfg


class _Shape:
    def __init__(self, t):
        self.shape = tuple(int(k) for k in t.shape)


def _ws_bytes(cfg):
    n = L.lib().hgnn_net_workspace_bytes(ctypes.byref(cfg))
    if n == 0:
        raise RuntimeError("hgnn_amd: unsupported network configuration "
                           f"(bs={cfg.bs}, Nmax={cfg.nmax}, Emax={cfg.emax}, J+2={cfg.j_tot}, d={cfg.d})")
    return n


def _inputs(X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg):
    inp = L.NetInputs()
    inp.d_X = X.data_ptr()
    inp.d_W = W.data_ptr()
    inp.d_N_batch = N_batch.data_ptr()
    inp.d_mask = mask.data_ptr()
    if XL is not None:
        inp.d_XL = XL.data_ptr()
        inp.d_WL = WL.data_ptr()
        inp.d_Pm = Pm.data_ptr()
        inp.d_Pd = Pd.data_ptr()
        inp.d_E_batch = E_batch.data_ptr()
        inp.d_mask_lg = mask_lg.data_ptr()
    return inp


@torch.library.custom_op("hgnn_amd::net_forward", mutates_args=(), device_types="cuda")
def net_forward(X: Tensor, W: Tensor, N_batch: Tensor, mask: Tensor, XL: Optional[Tensor], WL: Optional[Tensor],
                Pm: Optional[Tensor], Pd: Optional[Tensor], E_batch: Optional[Tensor], mask_lg: Optional[Tensor],
                params: List[Tensor], running: List[Tensor], kind: int, order: int, d: int, n_layers: int,
                dim_out: int, training: bool) -> Tuple[Tensor, Tensor, List[Tensor]]:
    cfg = _cfg(kind, order, d, n_layers, dim_out, training, X, W, XL)
    running = [t.clone() for t in running]
    ws = torch.empty(_ws_bytes(cfg), dtype=torch.uint8, device=X.device)
    out = torch.empty(cfg.bs, dim_out, dtype=torch.float32, device=X.device)
    inp = _inputs(X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg)
    with torch.cuda.device(X.device):
        st = L.lib().hgnn_net_forward(ctypes.byref(cfg), ctypes.byref(inp), L.ptr_array(params), L.ptr_array(running),
                                      ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                      L.stream_handle(X.device))
        L.check(st, "network forward")
        N._watch_error_word(cfg, ws)
    return out, ws, running


@net_forward.register_fake
def _net_forward_fake(X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg, params, running, kind, order, d,
                      n_layers, dim_out, training):
    cfg = _cfg(kind, order, d, n_layers, dim_out, training, X, W, XL)
    return (X.new_empty(cfg.bs, dim_out), X.new_empty(_ws_bytes(cfg), dtype=torch.uint8),
            [t.new_empty(t.shape) for t in running])


@torch.library.custom_op("hgnn_amd::net_backward", mutates_args=(), device_types="cuda")
def net_backward(dout: Tensor, ws: Tensor, X: Tensor, W: Tensor, N_batch: Tensor, mask: Tensor, XL: Optional[Tensor],
                 WL: Optional[Tensor], Pm: Optional[Tensor], Pd: Optional[Tensor], E_batch: Optional[Tensor],
                 mask_lg: Optional[Tensor], params: List[Tensor], kind: int, order: int, d: int, n_layers: int,
                 dim_out: int, training: bool, need_dx: bool, need_dw: bool) -> Tuple[Tensor, Tensor, List[Tensor]]:
    cfg = _cfg(kind, order, d, n_layers, dim_out, training, X, W, XL)
    cfg.need_dx = 1 if need_dx else 0
    cfg.need_dw = 1 if need_dw else 0
    grads = [torch.empty_like(p) for p in params]
    dX = torch.empty_like(X) if need_dx else X.new_empty(0)
    dW = torch.empty_like(W) if need_dw else W.new_empty(0)
    inp = _inputs(X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg)
    dout = dout.contiguous()
    with torch.cuda.device(X.device):
        st = L.lib().hgnn_net_backward_ex(ctypes.byref(cfg), ctypes.byref(inp), None, L.ptr_array(params),
                                          ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(dout.data_ptr()),
                                          L.ptr_array(grads), L.ptr(dX if need_dx else None),
                                          L.ptr(dW if need_dw else None), L.stream_handle(X.device), None, None, 0)
    L.check(st, "network backward")
    return dX, dW, grads


@net_backward.register_fake
def _net_backward_fake(dout, ws, X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg, params, kind, order, d,
                       n_layers, dim_out, training, need_dx, need_dw):
    return (X.new_empty(X.shape) if need_dx else X.new_empty(0), W.new_empty(W.shape) if need_dw else W.new_empty(0),
            [p.new_empty(p.shape) for p in params])


def _setup_context(ctx, inputs, output):
    (X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg, params, running, kind, order, d, n_layers, dim_out,
     training) = inputs
    _, ws, _ = output
    ctx.opt = [t is not None for t in (XL, WL, Pm, Pd, E_batch, mask_lg)]
    keep = [t for t in (X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg) if t is not None]
    ctx.save_for_backward(ws, *keep, *params)
    ctx.n_params = len(params)
    ctx.n_running = len(running)
    ctx.meta = (kind, order, d, n_layers, dim_out, training)


def _backward(ctx, dout, dws, drunning):
    saved = list(ctx.saved_tensors)
    ws = saved.pop(0)
    params = saved[len(saved) - ctx.n_params:]
    rest = saved[:len(saved) - ctx.n_params]
    X, W, N_batch, mask = rest[:4]
    it = iter(rest[4:])
    XL, WL, Pm, Pd, E_batch, mask_lg = [next(it) if present else None for present in ctx.opt]
    need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
    dX, dW, grads = torch.ops.hgnn_amd.net_backward(dout, ws, X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg,
                                                     params, *ctx.meta, need_dx, need_dw)
    return (dX if need_dx else None, dW if need_dw else None, None, None, None, None, None, None, None, None,
            list(grads), [None] * ctx.n_running, None, None, None, None, None, None)


net_forward.register_autograd(_backward, setup_context=_setup_context)


def run_net_ops(spec, X, W, N_batch, mask, XL=None, WL=None, Pm=None, Pd=None, E_batch=None, mask_lg=None):
    """GNN_simple / GNN_lg forward through the registered operators (same checks as hgnn_amd.net.run_net)."""
    lg = spec.kind == 1
    dev = N._require_cuda([X, W, N_batch, mask] + ([XL, WL, Pm, Pd, E_batch, mask_lg] if lg else []), "GNN forward")
    X, W, mask = N._f32(X), N._f32(W), N._f32(mask)
    Nb = N._i64(N_batch)
    if lg:
        XL, WL, Pm, Pd, mask_lg = map(N._f32, (XL, WL, Pm, Pd, mask_lg))
        E_batch = N._i64(E_batch)
    else:
        XL = WL = Pm = Pd = E_batch = mask_lg = None
    params = N._checked_params(spec, X.shape[1], W.shape[3], dev)
    out, _, running = torch.ops.hgnn_amd.net_forward(X, W, Nb, mask, XL, WL, Pm, Pd, E_batch, mask_lg, params,
                                                     list(spec.running), spec.kind, spec.order, spec.d,
                                                     spec.n_layers, spec.dim_out, bool(spec.training))
    if spec.training:
        with torch.no_grad():
            torch._foreach_copy_(list(spec.running), list(running))
    return out
