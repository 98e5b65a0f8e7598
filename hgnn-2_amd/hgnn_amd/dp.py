"""Batch-axis data parallelism for the drop-in models (SURVEY.md §8 e).

Graphs are independent except for the batch statistics of BN and the padded
sizes Nmax/Emax, so the natural shard is the batch axis: every rank runs the
full network on its own graphs and the only exchange is one all-reduce of the
gradients (torch.distributed "nccl" = RCCL over xGMI on MI355X; "gloo" in the
CPU tests).  With gradient-only all-reduce each rank normalises BN over its
own shard: the result equals "world reference batches, gradients averaged",
which is what tests/test_dp_cpu.py checks.

The gradient set is small (2.1 MB at d = 64, 8.4 MB at d = 128), so it goes as
one flat bucket: one latency-bound collective per step instead of one per
parameter.
"""

import torch
import torch.distributed as dist


class GradAllReduce:
    """Average .grad of `params` across ranks with one flat all-reduce."""

    def __init__(self, params, group=None):
        self.params = [p for p in params]
        self.group = group
        self._flat = None

    def __call__(self):
        if not dist.is_available() or not dist.is_initialized():
            return
        world = dist.get_world_size(self.group)
        if world == 1:
            return
        grads = []
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            grads.append(p.grad)
        # one concatenation, one collective, one multi-tensor copy back: a handful of launches
        # instead of two copies per parameter (49 tensors for GNN_lg)
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat, group=self.group)  # SUM on every backend (gloo has no AVG)
        flat.div_(world)
        views = []
        off = 0
        for g in grads:
            k = g.numel()
            views.append(flat[off:off + k].view_as(g))
            off += k
        torch._foreach_copy_(grads, views)
