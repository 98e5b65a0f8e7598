"""Batch-axis data parallelism for the drop-in models (SURVEY.md §8 e).

Graphs are independent except for the batch statistics of BN and the padded
sizes Nmax/Emax, so the natural shard is the batch axis: every rank runs the
full network on its own graphs and the only exchange is the gradient
all-reduce (torch.distributed "nccl" = RCCL over xGMI on MI355X; "gloo" in the
CPU tests).  With gradient-only all-reduce each rank normalises BN over its
own shard: the result equals "world reference batches, gradients averaged"
(the reference itself has one batch, models/layers/batch_normalization.py:80-93),
which tests/test_dp_cpu.py and tests/test_gpu_dp.py check.

* shard_graphs: the global batch split into `world` shards balanced by the
  per-graph work N + M (nodes + edge slots, the rows every kernel walks),
  longest-processing-time first, so ragged graphs do not leave a rank idle.
* LayerBucketAllReduce: one gradient bucket per layer (layerlast.fc rides with
  the last layer).  The network executor records two HIP events per layer in
  its backward (hgnn_net_backward_ex: main stream and the weight-GEMM side
  stream); a communication stream waits on them and all-reduces that layer's
  bucket while the earlier layers are still being differentiated.  The
  gradients are written by the executor straight into one flat buffer, so the
  collective needs no packing copies.
* BN running statistics (plain attributes, not state, batch_normalization.py:30-38)
  averaged across ranks in every step -- LayerBucketAllReduce carries them in the
  last layer's bucket, average_running_stats is the stand-alone collective -- so
  every rank, and a checkpoint written by rank 0, holds the same eval-mode
  statistics.
* GradAllReduce: the single flat all-reduce for any module (used by TrainStep
  when no executor events are available).
"""

import weakref

import torch
import torch.distributed as dist

# model -> its LayerBucketAllReduce (kept outside the module so torch.save(model) stays the
# reference's plain whole-module pickle, functions/logs.py:99-111)
_ATTACHED = weakref.WeakKeyDictionary()


def attached(model):
    return _ATTACHED.get(model)


def graph_cost(X, A):
    """Work of one graph for balancing: nodes + edge slots (M = nnz(A), functions/operators.py:36)."""
    return int(X.shape[0]) + int((A != 0).sum())


def shard_graphs(costs, world):
    """Split graph indices into `world` shards of near-equal total cost (LPT: longest first onto
    the least-loaded shard; ties to the lower rank).  Each shard keeps the original order."""
    costs = list(costs)
    loads = [0] * world
    owner = [0] * len(costs)
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        r = min(range(world), key=lambda k: (loads[k], k))
        owner[i] = r
        loads[r] += costs[i]
    return [[i for i in range(len(costs)) if owner[i] == r] for r in range(world)]


def _world(group):
    if not dist.is_available() or not dist.is_initialized():
        return 1
    return dist.get_world_size(group)


class GradAllReduce:
    """Average .grad of `params` across ranks with one flat all-reduce."""

    def __init__(self, params, group=None):
        self.params = [p for p in params]
        self.group = group

    def __call__(self):
        world = _world(self.group)
        if world == 1:
            return
        grads = []
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            grads.append(p.grad)
        # one concatenation, one collective, one multi-tensor copy back
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


def running_stats(model):
    """The BN running statistics tensors of a GNN_lg / GNN_simple drop-in (bn1, bn2 per layer)."""
    out = []
    for layer in model._layers():
        for nm in ("bn1", "bn2"):
            bn = getattr(layer, nm, None)
            if bn is not None:
                out += [bn.running_mean, bn.running_std]
    return out


def average_running_stats(model, group=None):
    world = _world(group)
    if world == 1:
        return
    ts = running_stats(model)
    flat = torch.cat([t.reshape(-1) for t in ts])
    dist.all_reduce(flat, group=group)
    flat.div_(world)
    off = 0
    views = []
    for t in ts:
        views.append(flat[off:off + t.numel()].view_as(t))
        off += t.numel()
    torch._foreach_copy_(ts, views)


class LayerBucketAllReduce:
    """Per-layer gradient buckets of a drop-in GNN, reduced during the executor's backward.

    Attaches itself to `model` (dp.attached(model)): the executor then writes every parameter gradient
    into self.flat and records the per-layer events.  Call the object after loss.backward():
    it enqueues, last layer first, a wait on the layer's events and the all-reduce of its
    bucket on a communication stream, then joins that stream and divides by the world size.
    sync_running=True also averages the BN running statistics: they are copied into the tail of the
    flat buffer (the last layer's bucket, reduced first) and back after the division, so the step
    has no collective beyond the gradient buckets.

    Gradient accumulation: the overlapped path needs every p.grad to be None at backward time
    (optimizer.zero_grad(), whose default is set_to_none=True).  When a p.grad is present
    (zero_grad(set_to_none=False), or several backwards per step) the executor writes fresh
    gradient tensors that autograd adds to p.grad as usual; the call then copies the accumulated
    gradients into the flat buffer and all-reduces it in one collective after the backward.
    """

    HW_QUEUE_NOTE = ("hgnn_amd.dp: GPU_MAX_HW_QUEUES is {} -- with a process group's streams the executor's side stream "
                     "can share the main stream's hardware queue and run serialised with it (~20 % per step); set "
                     "GPU_MAX_HW_QUEUES=8 before the process starts HIP (DESIGN.md §6)")

    def __init__(self, model, group=None, sync_running=True, force=False, single=False):
        self.model = model
        # single: one collective over the whole buffer after the backward instead of one per layer (fewer host-side
        # collective calls; no overlap with the backward)
        self.single = single
        # force: run the bucketed collectives even in a group of one rank (an RCCL group of world size 1 on a
        # one-GPU box exercises the communication stream, the per-layer events and the RCCL kernels)
        self.force = force
        self.group = group
        self.sync_running = sync_running
        spec = model._spec(next(model.parameters()).device)
        self.params = list(spec.params)
        dev = self.params[0].device
        self.device = dev
        per = 12 if spec.kind == 1 else 6
        n_layers = spec.n_layers - 1
        sizes = [p.numel() for p in self.params]
        # the BN running statistics ride at the end of the buffer, in the last layer's bucket (the first
        # one reduced): averaged by the gradients' own collectives, no second collective per step
        self.n_run = sum(t.numel() for t in running_stats(model)) if sync_running else 0
        self.n_grad = sum(sizes)
        self.flat = torch.zeros(self.n_grad + self.n_run, dtype=torch.float32, device=dev)
        self.run_tail = self.flat[self.n_grad:]
        self.views = []
        off = 0
        for p, k in zip(self.params, sizes):
            self.views.append(self.flat[off:off + k].view_as(p))
            off += k
        # bucket l = layer l's parameters; the fc pair and the running statistics join the last layer's bucket
        self.buckets = []
        off = 0
        for l in range(n_layers):
            last = l == n_layers - 1
            n = sum(sizes[l * per:(l + 1) * per]) + (sizes[-2] + sizes[-1] + self.n_run if last else 0)
            self.buckets.append((off, n))
            off += n
        assert off == self.flat.numel()
        self.events = []
        if dev.type == "cuda":
            cur = torch.cuda.current_stream(dev)
            for _ in range(2 * n_layers):
                ev = torch.cuda.Event()
                ev.record(cur)  # materialise the HIP event; the executor re-records it
                self.events.append(ev)
            self.comm = torch.cuda.Stream(dev)
        self.event_handles = [int(e.cuda_event) for e in self.events]
        self.ptrs = [v.data_ptr() for v in self.views]
        # RCCL (and NCCL) average in the collective itself; gloo sums, then the buffer is divided
        self.avg = None
        import os
        import warnings
        q = os.environ.get("GPU_MAX_HW_QUEUES")
        if dev.type == "cuda" and (q is None or (q.isdigit() and int(q) < 8)):
            warnings.warn(self.HW_QUEUE_NOTE.format(q or "unset (4)"), RuntimeWarning, stacklevel=2)
        # set by the executor's backward (net._grad_targets): True when the gradients went to fresh
        # tensors (some p.grad present), i.e. no per-layer events were recorded this step
        self.fresh = False
        # optional timing (bench.py, N > 1): per call, HIP events on the main stream when the call is
        # made (backward enqueued), on the communication stream when the first bucket's collective
        # starts (the last layer's gradients final) and when the last one ends
        self.timing = False
        self.marks = []
        _ATTACHED[model] = self

    def grad_targets(self):
        """(views, use_events): views of the flat buffer and True when every p.grad is None, else
        (None, False) -- the executor then writes fresh tensors for autograd to accumulate.  The views are
        made fresh for every backward and referenced nowhere else, so autograd's AccumulateGrad takes each
        one as p.grad as it is (a gradient tensor with another live reference is cloned instead: 50 copies
        per step, ~0.5 ms of host time at config 2)."""
        self.fresh = any(p.grad is not None for p in self.params)
        if self.fresh:
            return None, False
        return torch._C._nn.unflatten_dense_tensors(self.flat[:self.n_grad], self.params), True

    def __call__(self):
        world = _world(self.group)
        fresh = self.fresh
        if fresh:
            # accumulation: autograd summed fresh gradients into p.grad -- gathered into the views
            for p, v in zip(self.params, self.views):
                if p.grad is None:
                    v.zero_()  # a parameter without a gradient this step
                elif p.grad.data_ptr() != v.data_ptr():
                    v.copy_(p.grad)
                p.grad = v
        else:
            # the executor wrote into the flat buffer and autograd took its views as p.grad; a gradient that
            # does not alias the buffer (autograd cloned it) is copied in and replaced by the view
            for p, v, q in zip(self.params, self.views, self.ptrs):
                g = p.grad
                if g is None or g.data_ptr() != q:
                    if g is not None:
                        v.copy_(g)
                    p.grad = v
        self.fresh = False
        if world == 1 and not self.force:
            return
        if self.avg is None:
            self.avg = dist.get_backend(self.group) == "nccl"
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        run = running_stats(self.model) if self.n_run else []
        if run and sum(t.numel() for t in run) != self.n_run:
            raise RuntimeError("LayerBucketAllReduce: the model's BN running statistics changed size")

        def pack_running():
            # the running statistics are final once the forward has run (the executor updates them in place)
            if run:
                torch._foreach_copy_(self._tail_views(run), run)
        cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        if self.single and cur is not None and not fresh:
            # one collective on the caller's stream, after the backward it follows in stream order
            pack_running()
            dist.all_reduce(self.flat, op=op, group=self.group)
        elif fresh or cur is None:
            # no per-layer events this step: one collective over the whole buffer after the backward
            if cur is not None:
                self.comm.wait_stream(cur)
                with torch.cuda.stream(self.comm):
                    pack_running()
                    dist.all_reduce(self.flat, op=op, group=self.group)
                cur.wait_stream(self.comm)
            else:
                pack_running()
                dist.all_reduce(self.flat, op=op, group=self.group)
        else:
            mk = None
            if self.timing:
                mk = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                mk[0].record(cur)
            for l in reversed(range(len(self.buckets))):
                # the events are recorded in the backward, after the forward that wrote the running statistics
                self.comm.wait_event(self.events[2 * l])
                self.comm.wait_event(self.events[2 * l + 1])
                if mk is not None and l == len(self.buckets) - 1:
                    mk[1].record(self.comm)
                off, n = self.buckets[l]
                with torch.cuda.stream(self.comm):
                    if l == len(self.buckets) - 1:
                        pack_running()
                    dist.all_reduce(self.flat[off:off + n], op=op, group=self.group)
            if mk is not None:
                mk[2].record(self.comm)
            cur.wait_stream(self.comm)
            if mk is not None:
                mk[3].record(cur)
                self.marks.append(mk)
        if not self.avg:
            self.flat.div_(world)
        if run:
            torch._foreach_copy_(run, self._tail_views(run))

    def _tail_views(self, run):
        out = []
        off = 0
        for t in run:
            out.append(self.run_tail[off:off + t.numel()].view_as(t))
            off += t.numel()
        return out

    def timing_summary(self):
        """Mean over the timed calls (ms): 'span' from the first bucket's collective start to the
        last one's end on the communication stream, 'exposed' from the backward's end on the main
        stream to the main stream's join (the all-reduce time not hidden behind the backward)."""
        if not self.marks:
            return None
        torch.cuda.synchronize(self.device)
        span = sum(m[1].elapsed_time(m[2]) for m in self.marks) / len(self.marks)
        exposed = sum(max(0.0, m[0].elapsed_time(m[3])) for m in self.marks) / len(self.marks)
        n = len(self.marks)
        self.marks = []
        return {"allreduce_span_ms": round(span, 4), "allreduce_exposed_ms": round(exposed, 4), "calls": n,
                "buckets": len(self.buckets), "bytes": int(self.flat.numel() * 4)}

    def detach(self):
        if _ATTACHED.get(self.model) is self:
            del _ATTACHED[self.model]
