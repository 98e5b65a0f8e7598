"""Autograd binding of the batched CCN executor (hgnn_ccn_* in include/hgnn_amd.h).

The reference builds every receptive field, chi matrix, promotion and the
d^5 tensor product per node in Python (functions/utils_ccn.py:66-324,
functions/contraction.py:106-121) and runs one graph per forward
(models/compnets/model_ccn.py:41-64, 93-105).  Here a whole padded batch of
graphs goes through three device phases (csrc/ccn.hip):

  plan      neighbour lists, degrees, prefix offsets and chi position maps
            (int, bit-exact with _get_chi) -- one small host sync for the
            ragged totals that size the feature workspace;
  forward   per level one kernel (promotion + contraction + Linear + ReLU
            fused; the 2-D contraction uses the closed form of DESIGN.md
            instead of materialising T (x) I), then the readout;
  backward  the adjoint of each phase, gather-formulated (no atomics).

X is (bs, nmax, f) zero-padded, adj (bs, nmax, nmax) with the self loops the
reference's caller adds (scripts/train_ccn.py:36), n_batch (bs,) int64.
"""

import ctypes
import os

import torch

from . import _lib as L
from .net import (_capturing, _require_cuda, _f32, _i64, _raise_bits, check_errors, register_check, strict,
                  watch_word)

# CCN_1D on graphs of <= 64 nodes and CCN_2D on graphs of <= 32 nodes through the one-workgroup-per-graph
# kernels (csrc/ccn_small.hip, csrc/ccn2_small.hip): no plan, no workspace sizing, 1 + 1 dispatches per call
# for one graph.  HGNN_CCN_SMALL=0 (or setting this to False) keeps every call on the general path.
SMALL = os.environ.get("HGNN_CCN_SMALL", "1") != "0"
SMALL2_WS_CAP = 512 << 20  # bytes: the CCN-2D small path's workspace bound per call (CcnSpec.small)

CCN_MAX_DEGREE = {1: 1024, 2: 256}  # csrc/ccn.hip CCN1_MAXD, CCN_BIGD (by order)
CCN2_MAX_CHANNELS = 16  # csrc/ccn.hip C2_CMAX_WIDE: CCN-2D f_in and hidden


class CcnSpec:
    def __init__(self, order, f_in, hidden, layers, n_out):
        self.order = order
        self.f_in = f_in
        self.hidden = hidden
        self.layers = layers
        self.n_out = n_out

    def config(self, bs, nmax):
        return L.CcnConfig(self.order, bs, nmax, self.f_in, self.hidden, self.layers, self.n_out, 0)

    def small(self, bs, nmax):
        """(config, workspace bytes) of the small-graph path for this batch shape, or None."""
        key = (bs, nmax)
        c = self._small.get(key) if hasattr(self, "_small") else None
        if c is None:
            if not hasattr(self, "_small"):
                self._small = {}
            cfg = self.config(bs, nmax)
            lib = L.lib()
            c = (cfg, lib.hgnn_ccn_small_workspace_bytes(ctypes.byref(cfg))) \
                if lib.hgnn_ccn_small_supported(ctypes.byref(cfg)) else False
            # CCN-2D's small path reserves (L + 2) nmax^3 hidden floats per graph for its levels (~0.8 MB
            # per QM9 graph at L = 2, ~30x the rows the graph uses): batches beyond SMALL2_WS_CAP of
            # workspace go to the general path, whose workspace follows the batch's real sum of d^2
            if c and self.order == 2 and c[1] > SMALL2_WS_CAP:
                c = False
            self._small[key] = c
        return c or None

    def param_shapes(self):
        m = 2 if self.order == 1 else 18
        shapes = []
        for l in range(self.layers):
            cin = self.f_in if l == 0 else self.hidden
            shapes += [(self.hidden, m * cin), (self.hidden,)]
        shapes += [(self.n_out, self.f_in + self.layers * self.hidden), (self.n_out,)]
        return shapes


# Workspace bound (elements of the sum-d^2-sized arrays) below which the plan sizes everything from
# the shapes alone (bs nmax^3 >= sum d_i^2 for any content) and needs no host sync: the per-graph
# drop-in path (scripts/train_ccn.py:52, QM9 graphs: 29^3 = 24 K) and small batches.  CCN-2D keeps
# ~13 sum-d^2 arrays per level, so its bound is lower.
ASYNC_PLAN_BOUND = {1: 8 << 20, 2: 1 << 20}


def _plan(cfg, adj, n_batch, stream):
    lib = L.lib()
    dev = adj.device
    bs, nmax = adj.shape[0], adj.shape[1]
    bound = bs * nmax ** 3
    sums = (ctypes.c_longlong * 4)()  # sum d, sum d^2, nodes, max d
    if bound <= ASYNC_PLAN_BOUND[cfg.order]:
        max_d2 = max(bound, 1)
        plan = torch.empty(lib.hgnn_ccn_plan_bytes(ctypes.byref(cfg), max_d2), dtype=torch.uint8, device=dev)
        L.check(lib.hgnn_ccn_plan_async(ctypes.byref(cfg), L.ptr(adj), L.ptr(n_batch), L.ptr(plan), max_d2, sums,
                                        stream), "hgnn_ccn_plan_async")
        base = plan.data_ptr()
        off = int(lib.hgnn_ccn_error_word(ctypes.byref(cfg), ctypes.c_void_p(base), max_d2)) - base
        watch_word(plan[off:off + 4].view(torch.int32))  # checked without a sync (HGNN_STRICT=1: at once)
        return plan, max_d2, sums
    # upper bound of sum_i d_i^2 from the padded adjacency (exact when padding is zero)
    deg = (adj > 0).sum(-1)
    max_d2 = max(int((deg * deg).sum().item()), 1)
    plan = torch.empty(lib.hgnn_ccn_plan_bytes(ctypes.byref(cfg), max_d2), dtype=torch.uint8, device=dev)
    L.check(lib.hgnn_ccn_plan(ctypes.byref(cfg), L.ptr(adj), L.ptr(n_batch), L.ptr(plan), max_d2, sums, stream),
            "hgnn_ccn_plan")
    base = plan.data_ptr()
    off = int(lib.hgnn_ccn_error_word(ctypes.byref(cfg), ctypes.c_void_p(base), max_d2)) - base
    bits = int(plan[off:off + 4].view(torch.int32).item())
    if bits:
        _raise_bits(bits)
    return plan, max_d2, sums


class CcnPlan:
    """The batch's index construction (receptive fields, chi position maps, ragged totals), built
    once: a training loop that replays a captured HIP graph for the step (no host sync inside it)
    plans each batch beforehand and passes the plan to forward_batch."""

    def __init__(self, spec, adj, n_batch):
        _require_cuda([adj, n_batch], "CCN plan")
        bs, nmax = adj.shape[0], adj.shape[1]
        self.cfg = spec.config(bs, nmax)
        self.key = (spec.order, bs, nmax)
        self.plan, self.max_d2, self.sums = _plan(self.cfg, _f32(adj), _i64(n_batch), L.stream_handle(adj.device))


class _CcnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, pl, X, adj, n_batch, *params):
        lib = L.lib()
        bs, nmax, _ = X.shape
        cfg = spec.config(bs, nmax)
        s = L.stream_handle(X.device)
        if pl is not None:
            if pl.key != (spec.order, bs, nmax):
                raise RuntimeError("hgnn_amd: CCN plan was built for another batch shape / order")
            plan, max_d2, sums = pl.plan, pl.max_d2, pl.sums
        else:
            plan, max_d2, sums = _plan(cfg, adj, n_batch, s)
        ws = torch.empty(max(lib.hgnn_ccn_workspace_bytes(ctypes.byref(cfg), sums), 1), dtype=torch.uint8,
                         device=X.device)
        out = torch.empty(bs, spec.n_out, dtype=torch.float32, device=X.device)
        pa = L.ptr_array(params)
        L.check(lib.hgnn_ccn_forward(ctypes.byref(cfg), sums, L.ptr(X), pa, L.ptr(plan), max_d2, L.ptr(ws),
                                     L.ptr(out), s), "hgnn_ccn_forward")
        ctx.cfg, ctx.sums, ctx.plan, ctx.ws, ctx.max_d2 = cfg, sums, plan, ws, max_d2
        ctx.save_for_backward(*params)  # weights: an in-place change before backward raises
        ctx.x_shape = X.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = L.lib()
        dout = dout.contiguous()
        dev = dout.device
        params = ctx.saved_tensors
        grads = [torch.empty_like(p) for p in params]
        dX = torch.empty(ctx.x_shape, dtype=torch.float32, device=dev)
        L.check(lib.hgnn_ccn_backward(ctypes.byref(ctx.cfg), ctx.sums, L.ptr_array(params), L.ptr(ctx.plan),
                                      ctx.max_d2, L.ptr(ctx.ws), L.ptr(dout), L.ptr_array(grads), L.ptr(dX),
                                      L.stream_handle(dev)), "hgnn_ccn_backward")
        return (None, None, dX, None, None, *grads)


class _HostWord:
    """Validation word of the small-graph kernels in host-mapped pinned memory (hgnn_host_word_alloc),
    one per device: a graph with validation bits stores tag * 256 + bits into it (a plain store), so a
    check is a host read -- no copy, no event, nothing enqueued per call.  A nonzero word is an error
    not yet reported: the check reports it and clears the word from the host, so a HIP-graph replay
    (whose captured tag never changes) reports each failing replay again.  Found by the first check
    after that kernel has run (HGNN_STRICT=1 or check_errors() synchronise first); an error stored
    between a check's read and its clear is lost (the check is a host read, not an exchange)."""

    def __init__(self):
        self.words = {}      # device index -> (ctypes int32 view of the host word, device pointer)
        self.tag = 0

    def next(self, dev):
        w = self.words.get(dev.index)
        if w is None:
            h, d = ctypes.c_void_p(), ctypes.c_void_p()
            with torch.cuda.device(dev):
                L.check(L.lib().hgnn_host_word_alloc(ctypes.byref(h), ctypes.byref(d)), "hgnn_host_word_alloc")
            w = (ctypes.c_int32.from_address(h.value), d)
            self.words[dev.index] = w
        # the tag only labels the store (a diagnostic): reporting goes by the word being nonzero
        self.tag = self.tag % ((1 << 23) - 1) + 1
        return w[1], self.tag

    def check(self, block):
        if not self.words:
            return
        if block:
            torch.cuda.synchronize()
        bad = 0
        for hw, _ in self.words.values():
            v = hw.value
            if v:
                hw.value = 0
                bad |= v & 255
        if bad:
            _raise_bits(bad)


_word = _HostWord()
register_check(_word.check)


class _CcnSmallFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, small, X, adj, n_batch, *params):
        lib = L.lib()
        cfg, ws_bytes = small
        bs = X.shape[0]
        s = L.stream_handle(X.device)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=X.device)
        out = torch.empty(bs, spec.n_out, dtype=torch.float32, device=X.device)
        err, tag = _word.next(X.device)
        L.check(lib.hgnn_ccn_small_forward(ctypes.byref(cfg), L.ptr(X), L.ptr(adj), L.ptr(n_batch),
                                           L.ptr_array(params), L.ptr(ws), err, tag, L.ptr(out), s),
                "hgnn_ccn_small_forward")
        if strict() and not _capturing():
            _word.check(True)
        # the backward rebuilds the levels from X, adj, n_batch and the weights: saved through autograd so
        # an in-place change between forward and backward raises instead of giving wrong gradients
        ctx.save_for_backward(X, adj, n_batch, *params)
        ctx.cfg, ctx.ws = cfg, ws
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = L.lib()
        X, adj, nb, *params = ctx.saved_tensors
        dout = dout.contiguous()
        dev = dout.device
        grads = [torch.empty_like(p) for p in params]
        dX = torch.empty(X.shape, dtype=torch.float32, device=dev)
        L.check(lib.hgnn_ccn_small_backward(ctypes.byref(ctx.cfg), L.ptr(X), L.ptr(adj), L.ptr(nb),
                                            L.ptr_array(params), L.ptr(ctx.ws), L.ptr(dout), L.ptr_array(grads),
                                            L.ptr(dX), L.stream_handle(dev)), "hgnn_ccn_small_backward")
        return (None, None, dX, None, None, *grads)


def run_ccn(spec, params, X, adj, n_batch, plan=None):
    """Batched CCN forward: X (bs,nmax,f), adj (bs,nmax,nmax), n_batch (bs,) -> (bs, n_out).
    plan: a CcnPlan of this adj / n_batch (else the plan is built here: without a host sync for
    small shapes, ASYNC_PLAN_BOUND; with one otherwise).  n_batch None: every graph has nmax nodes.
    CCN_1D batches of <= 64-node graphs and CCN_2D batches of <= 32-node graphs (f_in <= 8, hidden <= 2) take
    the small-graph kernels (SMALL; a plan is then unused)."""
    check_errors(block=False)
    # the small-graph kernels need no plan: a batch planned for capture (CcnPlan) takes them too
    if SMALL and X.dim() == 3:
        small = spec.small(X.shape[0], X.shape[1])
        if small is not None:
            _require_cuda([X, adj, n_batch, *params], "CCN")
            _check_shapes(spec, params, X, adj, n_batch)
            return _CcnSmallFn.apply(spec, small, _f32(X), _f32(adj), None if n_batch is None else _i64(n_batch),
                                     *[_f32(p) for p in params])
    if n_batch is None:
        n_batch = torch.full((X.shape[0],), X.shape[1], dtype=torch.int64, device=X.device)
    _require_cuda([X, adj, n_batch, *params], "CCN")
    _check_shapes(spec, params, X, adj, n_batch)
    return _CcnFn.apply(spec, plan, _f32(X), _f32(adj), _i64(n_batch), *[_f32(p) for p in params])


def _check_shapes(spec, params, X, adj, n_batch):
    if X.dim() != 3 or adj.dim() != 3:
        raise RuntimeError(f"hgnn_amd: CCN expects X (bs,nmax,f) and adj (bs,nmax,nmax), got {tuple(X.shape)}, "
                           f"{tuple(adj.shape)}")
    bs, nmax, f = X.shape
    if tuple(adj.shape) != (bs, nmax, nmax) or f != spec.f_in or (n_batch is not None and n_batch.numel() != bs):
        raise RuntimeError(f"hgnn_amd: CCN shape mismatch: X {tuple(X.shape)}, adj {tuple(adj.shape)}, "
                           f"n_batch {None if n_batch is None else tuple(n_batch.shape)}, input_feats {spec.f_in}")
    if not hasattr(spec, "_shapes"):
        spec._shapes = spec.param_shapes()
    for p, shp in zip(params, spec._shapes):
        if tuple(p.shape) != shp:
            raise RuntimeError(f"hgnn_amd: CCN parameter shape {tuple(p.shape)} != {shp}")


def plan_maps(order, X, adj, n_batch):
    """Index construction only (for tests): per-graph (deg, nbr, pos) as numpy, read back from the device plan."""
    import numpy as np
    lib = L.lib()
    bs, nmax, f = X.shape
    cfg = L.CcnConfig(order, bs, nmax, f, 1, 1, 1, 0)
    s = L.stream_handle(X.device)
    plan, max_d2, sums = _plan(cfg, _f32(adj), _i64(n_batch), s)
    offs = (ctypes.c_size_t * 9)()
    L.check(lib.hgnn_ccn_plan_offsets(ctypes.byref(cfg), max_d2, offs), "hgnn_ccn_plan_offsets")
    torch.cuda.synchronize(X.device)
    h = plan.cpu().numpy()

    def arr(i, n):
        return h[offs[i]:offs[i] + 4 * n].view(np.int32)

    nodes = bs * nmax
    node_off = arr(0, bs + 1)
    deg = arr(1, nodes)
    nbr = arr(2, nodes * nmax)
    off2 = arr(6, nodes + 1)
    pos = arr(7, int(sums[1]))
    out = []
    for b in range(bs):
        n0, n1 = int(node_off[b]), int(node_off[b + 1])
        dg = deg[n0:n1].astype(np.int64)
        nb = np.concatenate([nbr[i * nmax:i * nmax + deg[i]] for i in range(n0, n1)]) if n1 > n0 else np.zeros(0)
        ps = pos[off2[n0]:off2[n1]].astype(np.int64)
        out.append((dg, nb.astype(np.int64) - n0, ps))  # plan stores packed node ids
    return out


class _Collapse(torch.autograd.Function):
    @staticmethod
    def forward(ctx, F):
        c, n = F.shape[0], F.shape[1]
        out = torch.empty(n, n, 18 * c, dtype=torch.float32, device=F.device)
        L.check(L.lib().hgnn_collapse6to3(L.ptr(F), L.ptr(out), c, n, L.stream_handle(F.device)),
                "hgnn_collapse6to3")
        ctx.shape = F.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        c, n = ctx.shape[0], ctx.shape[1]
        dF = torch.empty(ctx.shape, dtype=torch.float32, device=dout.device)
        L.check(L.lib().hgnn_collapse6to3_backward(L.ptr(dout.contiguous()), L.ptr(dF), c, n,
                                                   L.stream_handle(dout.device)), "hgnn_collapse6to3_backward")
        return dF


def collapse6to3(F):
    """F (C, n, n, n, n, n) -> (n, n, 18 C), contraction q at channels [q C, (q+1) C)."""
    _require_cuda([F], "collapse6to3")
    if F.dim() != 6 or any(F.shape[i] != F.shape[1] for i in range(1, 6)):
        raise RuntimeError(f"hgnn_amd: collapse6to3 expects (C, n, n, n, n, n), got {tuple(F.shape)}")
    return _Collapse.apply(_f32(F))
