"""HIP-graph replay of whole training steps (launch-bound configurations: cfg1's 20-layer
GNN_simple, cfg3's CCN-1D): a replay computes exactly what the eager step computes.

The executor enqueues everything without host synchronisation (device-side totals, the side
stream forks/joins with events), so torch.cuda.graph captures the forward, the loss and the
backward -- the CCN index plan is built once beforehand (CcnPlan), as its ragged totals size
the workspace on the host.
"""

import pytest
import torch

import fixture_util as fu

pytestmark = pytest.mark.gpu


def _capture(step):
    """Warm-up on a side stream, then capture.  The steps keep their outputs as values only
    (out.detach()): an output kept with its grad_fn keeps the eager step's autograd nodes alive,
    among them the parameters' AccumulateGrad nodes with the stream they were created on, and the
    capture then meets a cross-stream sync with that (default) stream -- capture_end crashed on
    the box that way (tools/graph_diag.py with DIAG_KEEP=1)."""
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    return g


def _batch(graphs):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    return [t.cuda() for t in prepare_batch(data, 0, 1)]


@pytest.mark.parametrize("kind", ["simple", "lg"])
def test_graph_replay_equals_eager_step(kind):
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg, GNN_simple
    if kind == "simple":
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _batch(dg.sbm_dataset(8, n=30, seed=11))
        model = GNN_simple(0, 2, 20, 5, 1, 1).cuda()
    else:
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _batch(dg.qm9_shape_dataset(64, seed=12))
        model = GNN_lg(0, 16, 4, 5, 1, 1, 2).cuda()
    fu.det_init(model, 13)
    X.requires_grad_(True)
    out_buf = {}

    def step():
        for p in model.parameters():
            p.grad = None
        X.grad = None
        out = model([X, W], Nb, mask) if kind == "simple" else model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        torch.nn.MSELoss()(out, T).backward()
        out_buf["out"] = out.detach()

    step()
    torch.cuda.synchronize()
    ref_out = out_buf["out"].detach().clone()
    ref = {k: p.grad.clone() for k, p in model.named_parameters()}
    ref_dx = X.grad.clone()
    g = _capture(step)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out_buf["out"].detach(), ref_out)
    for k, p in model.named_parameters():
        assert torch.equal(p.grad, ref[k]), k
    assert torch.equal(X.grad, ref_dx)


@pytest.mark.parametrize("small", [False, True])
def test_ccn1_graph_replay_with_plan_equals_eager(small, monkeypatch):
    """Captured CCN-1D step (general path with a CcnPlan, or the small-graph kernels that need none)
    replays bit-identically to the eager step."""
    import hgnn_amd.ccn as HC
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D
    monkeypatch.setattr(HC, "SMALL", small)
    graphs = [(x, a + torch.eye(a.shape[0]), t) for x, a, t in dg.qm9_shape_dataset(32, seed=14)]
    bs, nmax = len(graphs), max(x.shape[0] for x, _, _ in graphs)
    X = torch.zeros(bs, nmax, 5)
    A = torch.zeros(bs, nmax, nmax)
    T = torch.zeros(bs, 1)
    for b, (x, a, t) in enumerate(graphs):
        X[b, :x.shape[0]] = x
        A[b, :x.shape[0], :x.shape[0]] = a
        T[b, 0] = t[0]
    nb = torch.tensor([x.shape[0] for x, _, _ in graphs], dtype=torch.int64).cuda()
    X, A, T = X.cuda().requires_grad_(True), A.cuda(), T.cuda()
    net = CCN_1D(5, 1, 2, 2).cuda()
    fu.det_init(net, 15)
    plan = net.plan(A, nb)
    buf = {}

    def step():
        for p in net.parameters():
            p.grad = None
        X.grad = None
        out = net.forward_batch(X, A, nb, plan)
        ((out - T) ** 2).sum().backward()
        buf["out"] = out.detach()

    step()
    torch.cuda.synchronize()
    ref_out = buf["out"].detach().clone()
    ref = {k: p.grad.clone() for k, p in net.named_parameters()}
    ref_dx = X.grad.clone()
    # the eager step without a plan computes the same
    with torch.no_grad():
        assert torch.equal(net.forward_batch(X, A, nb), ref_out)
    torch.cuda.synchronize()
    g = _capture(step)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(buf["out"].detach(), ref_out)
    for k, p in net.named_parameters():
        assert torch.equal(p.grad, ref[k]), k
    assert torch.equal(X.grad, ref_dx)
