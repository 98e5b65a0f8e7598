"""Device-resident training step.

The reference's step (scripts/train_mnb.py:41-91) runs, per batch: prepare_batch
on the host, normalize_data(T), forward, nn.MSELoss, .item() twice for the
RunningAverage logs (two host syncs), backward and torch.optim.Adamax -- with
the optimizer re-created every epoch (scripts/main_gnn_qm9.py:185), which
resets its state.  TrainStep does the same arithmetic with every piece on the
device and no host synchronisation:

  forward      the network executor (dense inputs or a CsrBatch)
  loss         hgnn_mse_loss: normalised targets, MSE, MAE, the dloss seed and
               both RunningAverages, in one kernel
  backward     the executor's backward (autograd seeded with dloss)
  all-reduce   optional gradient bucket all-reduce (hgnn_amd.dp.GradAllReduce)
  optimizer    hgnn_adamax_step: Adamax over every parameter in one launch

Classification (the reference's `mean == 0` branch, scripts/train_mnb.py:50-51: T cast to
class indices, the drivers' nn.CrossEntropyLoss, scripts/main_generate.py:147) uses
hgnn_xent_loss instead; the MAE meters stay untouched as in the reference.
"""

import ctypes
import os

import torch

from . import _lib as L


class TrainStep:
    """One train_with_mnb minibatch step for a GNN_lg / GNN_simple drop-in model.

    step(batch) with batch = the 11-tuple of prepare_batch (on the model's device)
    or a hgnn_amd.csr.CsrBatch with targets.  Returns the device tensor `stats`:
    [loss, mae, running loss, running mae] (read it when you log, not per step).
    """

    def __init__(self, model, lr=3e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, t_mean=None, t_std=1.0,
                 grad_allreduce=None, classification=None):
        self.model = model
        # the reference's rule (train_mnb.py:50-51): mean == 0 marks generated (classification) data --
        # inferred only from an explicitly passed t_mean; TrainStep(model) is the regression step
        if classification is None:
            classification = t_mean is not None and float(t_mean) == 0.0
        self.classification = bool(classification)
        t_mean = 0.0 if t_mean is None else t_mean
        self.params = [p for p in model.parameters()]
        self.lr = float(lr)
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.weight_decay = float(weight_decay)
        self.t_mean = float(t_mean)
        self.t_std = float(t_std)
        self.allreduce = grad_allreduce
        dev = self.params[0].device
        if dev.type != "cuda":
            raise RuntimeError("hgnn_amd: TrainStep runs on the GPU only (call model.cuda() first)")
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise RuntimeError("hgnn_amd: TrainStep needs contiguous float32 parameters")
        self.stats = torch.zeros(4, dtype=torch.float32, device=dev)
        self._err = torch.zeros(1, dtype=torch.int32, device=dev)
        # the class-target error word, copied to pinned memory behind an event and checked at the
        # next step without synchronising the stream (HGNN_STRICT=1: checked at once)
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._err_ev = None
        self._numel = (ctypes.c_int64 * len(self.params))(*[p.numel() for p in self.params])
        self.reset_optimizer()

    def reset_optimizer(self):
        """The reference builds a new Adamax every epoch (scripts/main_gnn_qm9.py:185): zero state, step 0."""
        self.exp_avg = [torch.zeros_like(p) for p in self.params]
        self.exp_inf = [torch.zeros_like(p) for p in self.params]
        self.step_count = 0

    def reset_running(self):
        """New RunningAverage meters (one pair per train_with_mnb call, scripts/train_mnb.py:34-35)."""
        self.stats.zero_()

    def _forward(self, batch):
        from .csr import CsrBatch
        m = self.model
        if isinstance(batch, CsrBatch):
            if batch.T is None:
                raise RuntimeError("hgnn_amd: TrainStep needs a CsrBatch built with targets")
            return m.forward_csr(batch), batch.T
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = batch
        if m.dual:
            out = m([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        else:
            out = m([X, W], Nb, mask)
        return out, T

    def _poll_targets(self, block):
        ev = self._err_ev
        if ev is None:
            return
        if block:
            ev.synchronize()
        elif not ev.query():
            return
        self._err_ev = None
        if int(self._err_host[0]):
            self._err.zero_()
            self._err_host.zero_()
            raise RuntimeError("hgnn_amd: class target outside [0, dim_output) or not an integer "
                               "(the rows were left out of the loss and gradients)")

    def __call__(self, batch):
        lib = L.lib()
        self._poll_targets(block=False)
        self.model.train()
        for p in self.params:
            p.grad = None
        out, T = self._forward(batch)
        T = T.to(torch.float32).contiguous()
        stream = L.stream_handle(out.device)
        dout = torch.empty_like(out)
        if self.classification:
            if out.shape[1] < 2:
                raise RuntimeError("hgnn_amd: classification needs dim_output >= 2 (cross-entropy over one "
                                   "class is identically 0); pass t_mean != 0 or classification=False")
            if T.numel() != out.shape[0]:
                raise RuntimeError(f"hgnn_amd: class targets {tuple(T.shape)} do not match {out.shape[0]} rows")
            L.check(lib.hgnn_xent_loss(L.ptr(out.detach()), L.ptr(T), out.shape[0], out.shape[1], L.ptr(self.stats),
                                       L.ptr(dout), L.ptr(self._err), stream), "cross-entropy loss")
            if os.environ.get("HGNN_STRICT", "0") == "1":
                self._err_ev = None
                if int(self._err.item()):
                    self._err.zero_()
                    raise RuntimeError("hgnn_amd: class target outside [0, dim_output) or not an integer")
            elif not torch.cuda.is_current_stream_capturing():
                self._err_host.copy_(self._err, non_blocking=True)
                self._err_ev = torch.cuda.Event()
                self._err_ev.record()
        else:
            if T.numel() != out.numel():
                raise RuntimeError(f"hgnn_amd: targets {tuple(T.shape)} do not match the output {tuple(out.shape)}")
            L.check(lib.hgnn_mse_loss(L.ptr(out.detach()), L.ptr(T), out.numel(), self.t_mean, self.t_std,
                                      L.ptr(self.stats), L.ptr(dout), stream), "mse loss")
        torch.autograd.backward(out, dout)
        if self.allreduce is not None:
            self.allreduce()
        grads = [p.grad for p in self.params]
        if any(g is None for g in grads):
            raise RuntimeError("hgnn_amd: a parameter received no gradient")
        self.step_count += 1
        L.check(lib.hgnn_adamax_step(len(self.params), L.ptr_array(self.params), L.ptr_array(grads),
                                     L.ptr_array(self.exp_avg), L.ptr_array(self.exp_inf), self._numel, self.lr,
                                     self.betas[0], self.betas[1], self.eps, self.weight_decay, self.step_count,
                                     stream), "adamax step")
        return self.stats

    def check_targets(self):
        """Raise if a classification step saw a target outside [0, dim_output) (host sync)."""
        self._poll_targets(block=True)
        if int(self._err.item()):
            self._err.zero_()
            raise RuntimeError("hgnn_amd: class target outside [0, dim_output) or not an integer")
