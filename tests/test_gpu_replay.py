"""Replay of launch-bound executor calls (csrc/net.hip: a call met a third time with the same configuration
and device pointers is captured once into a HIP graph and replayed).  The replayed calls must give what the
eager enqueue gives -- bit for bit, since the same kernels run on the same buffers -- and must read the
buffers' current contents (inputs changed in place, parameters updated by an optimizer)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(graphs):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    return [t.cuda() for t in prepare_batch(data, 0, 1)]


def _simple_step(model, X, W, Nb, mask, T):
    for p in model.parameters():
        p.grad = None
    X.grad = W.grad = None
    out = model([X, W], Nb, mask)
    torch.nn.MSELoss()(out, T).backward()
    return (out.detach().clone(), X.grad.clone(), W.grad.clone(),
            [p.grad.clone() for p in model.parameters()])


def _same(a, b, what):
    assert torch.equal(a, b), f"{what}: max diff {(a - b).abs().max().item():.3g}"


def test_replayed_steps_equal_eager_steps_config1_shape():
    """Config 1's shape (GNN_simple L=20, 32 SBM-50 graphs, below the replay bound): steps 3.. replay the
    captured forward and backward; every step's output, dX, W.grad, parameter grads and the BN running
    statistics equal a twin model whose inputs sit at fresh addresses every step (never replayed)."""
    import copy

    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_simple
    torch.manual_seed(3)
    model = GNN_simple(0, 2, 20, 5, 1, 1).cuda()
    twin = copy.deepcopy(model)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _batch(dg.sbm_dataset(32, n=50, seed=3))
    T = T[:, :1].contiguous()
    X.requires_grad_(True)
    W.requires_grad_(True)
    keep = []
    for it in range(6):
        got = _simple_step(model, X, W, Nb, mask, T)
        Xf, Wf = X.detach().clone().requires_grad_(True), W.detach().clone().requires_grad_(True)
        keep.append((Xf, Wf))  # alive: the twin's pointers never repeat
        ref = _simple_step(twin, Xf, Wf, Nb, mask, T)
        _same(got[0], ref[0], f"step {it} output")
        _same(got[1], ref[1], f"step {it} dX")
        _same(got[2], ref[2], f"step {it} dW")
        for k, (g, r) in enumerate(zip(got[3], ref[3])):
            _same(g, r, f"step {it} grad {k}")
    for (n, b), (_, rb) in zip(model.named_buffers(), twin.named_buffers()):
        _same(b, rb, f"buffer {n}")


def test_replay_reads_current_contents():
    """After the capture, inputs changed in place and parameters updated by Adamax are what the replay
    reads; eval mode (another configuration) is its own entry."""
    import copy

    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    torch.manual_seed(5)
    model = GNN_lg(0, 16, 4, 5, 1, 1, 2).cuda()
    twin = copy.deepcopy(model)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _batch(dg.qm9_shape_dataset(48, seed=5))
    opt = torch.optim.Adamax(model.parameters(), lr=1e-2)
    opt2 = torch.optim.Adamax(twin.parameters(), lr=1e-2)
    keep = []
    for it in range(6):
        if it == 4:
            with torch.no_grad():
                X.mul_(1.5)
                XL.add_(0.25)
        opt.zero_grad()
        out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        torch.nn.MSELoss()(out, T).backward()
        opt.step()
        fresh = [t.clone() for t in (X, XL, W, WL, Pm, Pd, mask, mask_lg)]
        keep.append(fresh)
        opt2.zero_grad()
        ref = twin([fresh[0], fresh[1], fresh[2], fresh[3], fresh[4], fresh[5]], Nb, fresh[6], Eb, fresh[7])
        torch.nn.MSELoss()(ref, T).backward()
        opt2.step()
        _same(out.detach(), ref.detach(), f"step {it} output")
        for (n, p), (_, q) in zip(model.named_parameters(), twin.named_parameters()):
            _same(p.detach(), q.detach(), f"step {it} param {n}")
    model.eval()
    twin.eval()
    with torch.no_grad():
        for it in range(4):
            o = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
            fresh = [t.clone() for t in (X, XL, W, WL, Pm, Pd, mask, mask_lg)]
            keep.append(fresh)
            r = twin([fresh[0], fresh[1], fresh[2], fresh[3], fresh[4], fresh[5]], Nb, fresh[6], Eb, fresh[7])
            _same(o, r, f"eval {it}")
