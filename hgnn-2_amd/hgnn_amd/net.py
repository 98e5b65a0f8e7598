"""Autograd binding of the network executor (hgnn_net_forward / _backward).

One torch.autograd.Function runs a whole GNN_lg / GNN_simple forward as a
single enqueue of HIP kernels (include/hgnn_amd.h, hgnn-2_amd/csrc/net.hip) and
its backward as another, so `loss.backward()` in the reference's training
loop (scripts/train_mnb.py:90) works unchanged.

Input validation that needs the batch content (padding of the dense
operators, mask vs N_batch) runs on the device and sets an error word; the
host checks it without stalling the stream: at the next forward, at
`check_errors()`, or immediately when HGNN_STRICT=1.
"""

import ctypes
import os

import torch

from . import _lib as L

_pending = []
_timer = None


TIMER_STAMPS, TIMER_DISPATCH, TIMER_MARKERS = 0, 1, 2  # include/hgnn_amd.h HGNN_TIMER_*


class KernelTimer:
    """Timer of every launch of the selected kernel classes (HGNN_K_*).  mode TIMER_STAMPS: in-kernel
    s_memrealtime stamps per wave (the aggregation and GEMM kernels; the timed kernels run as in an untimed
    step), stamp_words device words (2 per wave of every timed launch); TIMER_DISPATCH: dispatch-bound HIP
    event pairs (every class; a timed dispatch runs slower); None: the library's default (dispatch events,
    or markers with HGNN_TIMER_MARKERS=1)."""

    def __init__(self, max_launches, classes, mode=None, stamp_words=0):
        mask = 0
        for c in classes:
            mask |= 1 << c
        if mode is None:
            self.handle = L.lib().hgnn_timer_create(max_launches, mask)
        else:
            self.handle = L.lib().hgnn_timer_create_ex(max_launches, mask, mode, stamp_words)
        if not self.handle:
            raise RuntimeError("hgnn_amd: could not create the kernel timer")

    def reset(self):
        L.lib().hgnn_timer_reset(self.handle)

    def elapsed(self, kcls):
        ms = ctypes.c_double()
        n = ctypes.c_int()
        L.check(L.lib().hgnn_timer_elapsed(self.handle, kcls, ctypes.byref(ms), ctypes.byref(n)), "timer")
        return ms.value, n.value

    def launches(self, max_launches=65536):
        """Stamp mode: [(class, entry_us, exit_us, stream)] of every timed launch in enqueue order (us from
        the region's first stamp; stream numbered in order of first appearance)."""
        cls = (ctypes.c_int * max_launches)()
        t0 = (ctypes.c_double * max_launches)()
        t1 = (ctypes.c_double * max_launches)()
        sq = (ctypes.c_int * max_launches)()
        n = L.lib().hgnn_timer_launches(self.handle, max_launches, cls, t0, t1, sq)
        if n < 0:
            L.check(-n, "timer launches")
        return [(cls[i], t0[i], t1[i], sq[i]) for i in range(min(n, max_launches))]

    def waves(self, launch, max_waves=1 << 20):
        """Stamp mode: [(entry_us, exit_us)] of every wave of timed launch `launch` (enqueue order), in the
        kernel's wave order (linear block id x waves per block + wave)."""
        t0 = (ctypes.c_double * max_waves)()
        t1 = (ctypes.c_double * max_waves)()
        n = L.lib().hgnn_timer_waves(self.handle, launch, max_waves, t0, t1)
        if n < 0:
            L.check(-n, "timer waves")
        return [(t0[i], t1[i]) for i in range(min(n, max_waves))]

    def close(self):
        if self.handle:
            L.lib().hgnn_timer_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        global _timer
        _timer = self
        return self

    def __exit__(self, *exc):
        global _timer
        _timer = None


def strict():
    return os.environ.get("HGNN_STRICT", "0") == "1"


def _raise_bits(bits):
    raise RuntimeError("hgnn_amd: invalid input batch: " + L.deverr_message(bits))


class _ErrorRing:
    """Pinned host slots the forwards' device error words are copied into asynchronously: a
    check reads a slot only once its copy's event has completed, so it never synchronises the
    stream (reading a device tensor with .item() waited for everything enqueued before it -- the
    host could then not run ahead of the GPU, 0.4 ms per step at config 2)."""

    SLOTS = 256

    def __init__(self):
        self.host = torch.zeros(self.SLOTS, dtype=torch.int32, pin_memory=True)
        self.next = 0

    def take(self):
        i = self.next
        self.next = (i + 1) % self.SLOTS
        for k, (ev, slot) in enumerate(_pending):  # a slot still in flight: retire its check first
            if slot == i:
                ev.synchronize()
                bits = int(self.host[slot])
                del _pending[k]
                if bits:
                    _pending.clear()
                    _raise_bits(bits)
                break
        return i


_ring = None


_checks = []  # further validation words with their own check(block) (hgnn_amd.ccn host-mapped word)


def register_check(fn):
    _checks.append(fn)


def check_errors(block=True):
    """Raise if any enqueued forward found an invalid input batch."""
    if _capturing():
        return
    for fn in _checks:
        fn(block)
    keep = []
    bad = 0
    for ev, slot in _pending:
        if block:
            ev.synchronize()
        if block or ev.query():
            bad |= int(_ring.host[slot])
        else:
            keep.append((ev, slot))
    _pending[:] = keep
    if bad:
        _pending.clear()
        _raise_bits(bad)


def _capturing():
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def _watch_error_word(cfg, ws):
    base = ws.data_ptr()
    addr = L.lib().hgnn_net_error_word(ctypes.byref(cfg), ctypes.c_void_p(base))
    off = int(addr) - base
    watch_word(ws[off:off + 4].view(torch.int32))


def watch_word(err):
    """Check a device error word (int32 view) without synchronising the stream: copied into a
    pinned ring slot behind an event, read by a later check_errors() (HGNN_STRICT=1: at once)."""
    if _capturing():
        # inside a HIP graph capture (bench.py --graph): the batch was validated by the eager
        # warm-up steps; no host-visible check can be part of a replayed graph
        return
    global _ring
    if strict():
        v = int(err.item())
        if v:
            _raise_bits(v)
        return
    if _ring is None:
        _ring = _ErrorRing()
    slot = _ring.take()
    _ring.host[slot:slot + 1].copy_(err, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    _pending.append((ev, slot))


def _require_cuda(tensors, what):
    dev = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(
                f"hgnn_amd: {what} runs on the GPU only; got a CPU tensor (move the batch with .cuda(), "
                "as scripts/train_mnb.py:60 does)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"hgnn_amd: {what}: tensors on different devices ({dev} vs {t.device})")
    return dev


def _f32(t):
    if t is None:
        return None
    if t.dtype != torch.float32:
        raise RuntimeError(f"hgnn_amd: expected float32 tensors, got {t.dtype}")
    return t.contiguous()


def _i64(t):
    return t.to(torch.int64).contiguous()


class NetSpec:
    """Static description of a network call (model hyper-parameters + mode)."""

    def __init__(self, kind, order, d, n_layers, dim_out, params, running, training, dp=None):
        self.dp = dp  # hgnn_amd.dp.LayerBucketAllReduce: flat gradient buffer + per-layer events
        self.kind = kind
        self.order = order
        self.d = d
        self.n_layers = n_layers
        self.dim_out = dim_out
        self.params = params
        self.running = running
        self.training = training


def expected_k(kind, order, f_in, d, n_layers, jt):
    """Input widths (K) of every Conv1d, in ABI parameter order (mirrors net.hip build_program)."""
    ks = []
    c2 = 2 * d
    cn, ce = f_in, 1
    for _ in range(n_layers - 1):
        if kind == 1:
            if order == 1:
                kn, ke = jt * cn + 2 * ce, jt * ce + 2 * c2
            elif order == 2:
                kn, ke = jt * cn + 2 * c2, jt * ce + 2 * cn
            else:
                kn, ke = jt * cn + 2 * ce, jt * ce + 2 * cn
            ks.append((kn, ke))
            cn, ce = c2, c2
        else:
            ks.append((jt * cn,))
            cn = c2
    k_last = jt * cn + (2 * ce if kind == 1 else 0)
    return ks, k_last


class _NetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, tensors, X, W, *params):
        XL, WL, Pm, Pd, Nb, Eb, mask, mask_lg = tensors
        dev = X.device
        lg = spec.kind == 1
        cfg = L.NetConfig()
        cfg.kind = spec.kind
        cfg.order = spec.order
        cfg.bs = X.shape[0]
        cfg.nmax = X.shape[2]
        cfg.emax = XL.shape[2] if lg else 0
        cfg.f_in = X.shape[1]
        cfg.d = spec.d
        cfg.n_layers = spec.n_layers
        cfg.j_tot = W.shape[3]
        cfg.dim_out = spec.dim_out
        cfg.training = 1 if spec.training else 0
        lib = L.lib()
        nbytes = lib.hgnn_net_workspace_bytes(ctypes.byref(cfg))
        if nbytes == 0:
            raise RuntimeError("hgnn_amd: unsupported network configuration "
                               f"(bs={cfg.bs}, Nmax={cfg.nmax}, Emax={cfg.emax}, J+2={cfg.j_tot}, d={cfg.d})")
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        out = torch.empty(cfg.bs, cfg.dim_out, dtype=torch.float32, device=dev)
        inp = L.NetInputs()
        inp.d_X = X.data_ptr()
        inp.d_W = W.data_ptr()
        inp.d_N_batch = Nb.data_ptr()
        inp.d_mask = mask.data_ptr()
        if lg:
            inp.d_XL = XL.data_ptr()
            inp.d_WL = WL.data_ptr()
            inp.d_Pm = Pm.data_ptr()
            inp.d_Pd = Pd.data_ptr()
            inp.d_E_batch = Eb.data_ptr()
            inp.d_mask_lg = mask_lg.data_ptr()
        run = L.ptr_array(spec.running)
        pp = L.ptr_array(params)
        args = (ctypes.byref(cfg), ctypes.byref(inp), pp, run, ctypes.c_void_p(ws.data_ptr()),
                ctypes.c_void_p(out.data_ptr()), L.stream_handle(dev))
        if _timer is not None:
            st = lib.hgnn_net_forward_timed(*args, ctypes.c_void_p(_timer.handle))
        else:
            st = lib.hgnn_net_forward(*args)
        L.check(st, "network forward")
        _watch_error_word(cfg, ws)
        ctx.cfg = cfg
        ctx.ws = ws
        ctx.inp = inp  # device pointers of the inputs below, read again by the backward
        ctx.param_ptrs = pp  # the parameters' pointers (saved below: an in-place change raises)
        ctx.spec = spec
        # saved through autograd: an in-place change of an input or a weight between forward and
        # backward raises the usual version error instead of giving wrong gradients
        ctx.save_for_backward(X, W, XL, WL, Pm, Pd, Nb, Eb, mask, mask_lg, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        cfg = ctx.cfg
        saved = ctx.saved_tensors
        X, W = saved[0], saved[1]
        params = saved[10:]
        dout = dout.contiguous().to(torch.float32)
        grads, evs, nev = _grad_targets(ctx.spec, params)
        dX = torch.empty_like(X) if ctx.needs_input_grad[2] else None
        dW = torch.empty_like(W) if ctx.needs_input_grad[3] else None
        cfg.need_dx = 1 if dX is not None else 0
        cfg.need_dw = 1 if dW is not None else 0
        with torch.cuda.device(X.device):
            st = L.lib().hgnn_net_backward_ex(
                ctypes.byref(cfg), ctypes.byref(ctx.inp), None, ctx.param_ptrs,
                ctypes.c_void_p(ctx.ws.data_ptr()), ctypes.c_void_p(dout.data_ptr()), L.ptr_array(grads), L.ptr(dX),
                L.ptr(dW), L.stream_handle(X.device), ctypes.c_void_p(_timer.handle) if _timer is not None else None,
                evs, nev)
        L.check(st, "network backward")
        return (None, None, dX, dW, *grads)


def _grad_targets(spec, params):
    """Gradient buffers for the backward: views into the data-parallel flat buffer (with its
    per-layer events) when a LayerBucketAllReduce is attached, else fresh tensors."""
    dp = spec.dp
    if dp is not None and len(dp.views) == len(params) and all(
            v.shape == p.shape and v.device == p.device for v, p in zip(dp.views, params)):
        views, use_events = dp.grad_targets()
        if use_events:
            evs = (ctypes.c_void_p * max(1, len(dp.event_handles)))(*dp.event_handles)
            return list(views), evs, len(dp.event_handles)
        # some p.grad present: fresh tensors, accumulated by autograd (dp.py, gradient accumulation)
    # one allocation for all of them (50 empty_like calls were ~0.1 ms of host time per step), cut into the
    # parameters' shapes in one C++ call (split + view per parameter in Python cost ~0.3 ms per step)
    flat = torch.empty(sum(p.numel() for p in params), dtype=torch.float32, device=params[0].device)
    return list(torch._C._nn.unflatten_dense_tensors(flat, params)), None, 0


def run_net(spec, X, W, N_batch, mask, XL=None, WL=None, Pm=None, Pd=None, E_batch=None, mask_lg=None):
    """Forward of GNN_simple (kind 0) / GNN_lg (kind 1) through the HIP executor."""
    check_errors(block=False)
    lg = spec.kind == 1
    tensors_in = [X, W, N_batch, mask] + ([XL, WL, Pm, Pd, E_batch, mask_lg] if lg else [])
    dev = _require_cuda(tensors_in, "GNN forward")
    X = _f32(X)
    W = _f32(W)
    mask = _f32(mask)
    Nb = _i64(N_batch)
    bs, f_in, nmax = X.shape
    if W.dim() != 4 or W.shape[:3] != (bs, nmax, nmax):
        raise RuntimeError(f"hgnn_amd: W must be (bs, Nmax, Nmax, J+2) = ({bs}, {nmax}, {nmax}, .), got {tuple(W.shape)}")
    if mask.shape != (bs, nmax, nmax) or Nb.shape != (bs,):
        raise RuntimeError("hgnn_amd: mask must be (bs, Nmax, Nmax) and N_batch (bs,)")
    if lg:
        XL, WL, Pm, Pd, mask_lg = map(_f32, (XL, WL, Pm, Pd, mask_lg))
        Eb = _i64(E_batch)
        emax = XL.shape[2]
        jt = W.shape[3]
        if XL.shape != (bs, 1, emax):
            raise RuntimeError(f"hgnn_amd: XL must be (bs, 1, Emax), got {tuple(XL.shape)}")
        if WL.shape != (bs, emax, emax, jt):
            raise RuntimeError(f"hgnn_amd: WL must be (bs, Emax, Emax, J+2), got {tuple(WL.shape)}")
        if Pm.shape != (bs, nmax, emax) or Pd.shape != (bs, nmax, emax):
            raise RuntimeError("hgnn_amd: Pm/Pd must be (bs, Nmax, Emax)")
        if mask_lg.shape != (bs, emax, emax) or Eb.shape != (bs,):
            raise RuntimeError("hgnn_amd: mask_lg must be (bs, Emax, Emax) and E_batch (bs,)")
    else:
        Eb = None
    params = _checked_params(spec, f_in, W.shape[3], dev)
    tensors = (XL, WL, Pm, Pd, Nb, Eb, mask, mask_lg)
    with torch.cuda.device(dev):
        return _NetFn.apply(spec, tensors, X, W, *params)


_checked_last = [None, None]  # (signature, parameter list) of the last call that passed the checks


def _checked_params(spec, f_in, jt, dev):
    """Every parameter's shape against the widths the executor will read (the C ABI gets bare
    pointers: a mismatch would be an out-of-bounds device read), dtype and device.  A call with the same
    parameter objects at the same storage addresses, shapes, dtypes, contiguity, widths and device as the
    last one that passed returns its list without re-checking (~70 us of host time per forward)."""
    params = spec.params
    # shape, dtype and contiguity too: an in-place metadata change at the same address (p.data = a view,
    # resize_, a dtype view) must not hit the cache
    sig = (spec.kind, spec.order, spec.d, spec.n_layers, spec.dim_out, f_in, jt, dev,
           tuple(map(id, params)),
           tuple((p.data_ptr(), tuple(p.shape), p.dtype, p.is_contiguous()) for p in params))
    if _checked_last[0] == sig:
        return _checked_last[1]
    out = _check_params(spec, f_in, jt, dev)
    if all(a is b for a, b in zip(out, params)):  # contiguous as given: nothing copied, safe to reuse
        _checked_last[0], _checked_last[1] = sig, out
    return out


def _check_params(spec, f_in, jt, dev):
    lg = spec.kind == 1
    ks, k_last = expected_k(spec.kind, spec.order, f_in, spec.d, spec.n_layers, jt)
    params = list(spec.params)
    per = 12 if lg else 6
    if len(params) != per * len(ks) + 2:
        raise RuntimeError(f"hgnn_amd: expected {per * len(ks) + 2} parameters, got {len(params)}")
    for l, kk in enumerate(ks):
        convs = [(0, kk[0]), (2, kk[0])] + ([(6, kk[1]), (8, kk[1])] if lg else [])
        for off, k in convs:
            w = params[l * per + off]
            if w.shape != (spec.d, k, 1):
                raise RuntimeError(f"hgnn_amd: layer {l} conv weight {tuple(w.shape)} != ({spec.d}, {k}, 1)")
            if params[l * per + off + 1].shape != (spec.d,):
                raise RuntimeError(f"hgnn_amd: layer {l} conv bias {tuple(params[l * per + off + 1].shape)}")
        for off in ((4, 5, 10, 11) if lg else (4, 5)):
            if params[l * per + off].numel() != 1:
                raise RuntimeError(f"hgnn_amd: layer {l} BN affine parameters must be scalars")
    if params[-2].shape != (spec.dim_out, k_last, 1):
        raise RuntimeError(f"hgnn_amd: fc weight {tuple(params[-2].shape)} != ({spec.dim_out}, {k_last}, 1)")
    if params[-1].shape != (spec.dim_out,):
        raise RuntimeError(f"hgnn_amd: fc bias {tuple(params[-1].shape)} != ({spec.dim_out},)")
    for p in params:
        if p.device != dev or p.dtype != torch.float32:
            raise RuntimeError("hgnn_amd: parameters must be float32 on the input device (call model.cuda())")
    return [p if p.is_contiguous() else p.contiguous() for p in params]


def _csr_config(spec, batch):
    cfg = L.NetConfig()
    cfg.kind = spec.kind
    cfg.order = spec.order
    cfg.bs = batch.bs
    cfg.nmax = batch.nmax
    cfg.emax = batch.emax if spec.kind == 1 else 0
    cfg.f_in = batch.f_in
    cfg.d = spec.d
    cfg.n_layers = spec.n_layers
    cfg.j_tot = batch.j_tot
    cfg.dim_out = spec.dim_out
    cfg.training = 1 if spec.training else 0
    return cfg


class _NetCsrFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, batch, x, *params):
        dev = batch.device
        cfg = _csr_config(spec, batch)
        lib = L.lib()
        nbytes = lib.hgnn_net_workspace_bytes(ctypes.byref(cfg))
        if nbytes == 0:
            raise RuntimeError("hgnn_amd: unsupported network configuration for this CSR batch")
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        out = torch.empty(cfg.bs, cfg.dim_out, dtype=torch.float32, device=dev)
        L.check(lib.hgnn_net_forward_csr(ctypes.byref(cfg), ctypes.byref(batch.view), L.ptr_array(params),
                                         L.ptr_array(spec.running), ctypes.c_void_p(ws.data_ptr()),
                                         ctypes.c_void_p(out.data_ptr()), L.stream_handle(dev)),
                "network forward (csr)")
        ctx.cfg, ctx.ws, ctx.batch, ctx.spec = cfg, ws, batch, spec
        ctx.save_for_backward(*params)  # weights: an in-place change before backward raises
        return out

    @staticmethod
    def backward(ctx, dout):
        cfg = ctx.cfg
        batch = ctx.batch
        dout = dout.contiguous().to(torch.float32)
        params = ctx.saved_tensors
        grads, evs, nev = _grad_targets(ctx.spec, params)
        dX = torch.empty(batch.nodes, batch.f_in, dtype=torch.float32, device=batch.device) \
            if ctx.needs_input_grad[2] else None
        cfg.need_dx = 1 if dX is not None else 0
        cfg.need_dw = 0
        with torch.cuda.device(batch.device):
            st = L.lib().hgnn_net_backward_ex(ctypes.byref(cfg), None, ctypes.byref(batch.view), L.ptr_array(params),
                                              ctypes.c_void_p(ctx.ws.data_ptr()), ctypes.c_void_p(dout.data_ptr()),
                                              L.ptr_array(grads), L.ptr(dX), None, L.stream_handle(batch.device),
                                              None, evs, nev)
        L.check(st, "network backward (csr)")
        return (None, None, dX, *grads)


def run_net_csr(spec, batch):
    """GNN_simple / GNN_lg forward on a hgnn_amd.csr.CsrBatch.  The differentiable node
    input is batch.x (packed (nodes, f_in)); set batch.x.requires_grad_() for dX."""
    if not batch.image.is_cuda:
        raise RuntimeError("hgnn_amd: the CSR batch must be on the GPU (CsrBatch(..., device='cuda'))")
    if spec.kind == 1 and not batch.dual:
        raise RuntimeError("hgnn_amd: GNN_lg needs a CSR batch built with dual=True")
    params = _checked_params(spec, batch.f_in, batch.j_tot, batch.device)
    with torch.cuda.device(batch.device):
        return _NetCsrFn.apply(spec, batch, batch.x, *params)
