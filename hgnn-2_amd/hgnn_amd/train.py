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

import torch

from . import _lib as L


class TrainStep:
    """One train_with_mnb minibatch step for a GNN_lg / GNN_simple drop-in model.

    step(batch) with batch = the 11-tuple of prepare_batch (on the model's device)
    or a hgnn_amd.csr.CsrBatch with targets.  Returns the device tensor `stats`:
    [loss, mae, running loss, running mae] (read it when you log, not per step).
    """

    def __init__(self, model, lr=3e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, t_mean=0.0, t_std=1.0,
                 grad_allreduce=None, classification=None):
        self.model = model
        # the reference's rule: mean == 0 marks generated (classification) data
        self.classification = (float(t_mean) == 0.0) if classification is None else bool(classification)
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

    def __call__(self, batch):
        lib = L.lib()
        self.model.train()
        for p in self.params:
            p.grad = None
        out, T = self._forward(batch)
        T = T.to(torch.float32).contiguous()
        stream = L.stream_handle(out.device)
        dout = torch.empty_like(out)
        if self.classification:
            if T.numel() != out.shape[0]:
                raise RuntimeError(f"hgnn_amd: class targets {tuple(T.shape)} do not match {out.shape[0]} rows")
            L.check(lib.hgnn_xent_loss(L.ptr(out.detach()), L.ptr(T), out.shape[0], out.shape[1], L.ptr(self.stats),
                                       L.ptr(dout), L.ptr(self._err), stream), "cross-entropy loss")
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
        if int(self._err.item()):
            raise RuntimeError("hgnn_amd: class target outside [0, dim_output) or not an integer")
