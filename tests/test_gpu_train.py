"""Device-resident training step (hgnn_amd.train.TrainStep) vs the reference's step.

The reference step (scripts/train_mnb.py:41-91): T' = normalize_data(T, mean, std),
out = model(...), MSELoss, backward, torch.optim.Adamax.step; RunningAverage
logs of loss and MAE.  Here the same model (copied weights) runs both ways for
several steps; parameters must agree after every step.
Each step starts from equal parameters and optimizer state (re-synchronised after
the comparison).  Tolerance: parameters |d| <= 1e-5 * max(1, |p|) per step (Adamax steps are
lr-sized; summation-order noise in the gradients shows up only below that),
losses within 1e-5 relative.  Elements whose gradient is analytically zero
(cv2 / cv4 biases; ReLU channels active on every row) carry fp32 noise that
Adamax amplifies to lr-sized steps on both sides (the reference against itself
at another thread count does the same): for elements whose reference gradient
is below the noise floor (1e-4 max|g|) only |d| <= 2 lr holds.
"""

import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(graphs):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    return [t.cuda() for t in prepare_batch(data, 0, 1)]


@pytest.mark.parametrize("csr", [False, True])
def test_train_step_matches_torch_adamax_loop(csr):
    import hgnn_amd.datagen as dg
    from functions.utils import normalize_data
    from hgnn_amd.csr import prepare_batch_csr
    from hgnn_amd.train import TrainStep
    from models.gnns.model_mnb import GNN_lg
    torch.manual_seed(11)
    model = GNN_lg(0, 16, 4, 5, 1, 1, 2).cuda()
    ref = copy.deepcopy(model)
    mean, std, lr = 0.3, 1.7, 1e-3
    opt = torch.optim.Adamax(ref.parameters(), lr=lr)
    crit = torch.nn.MSELoss()
    step = TrainStep(model, lr=lr, t_mean=mean, t_std=std)
    batches = [dg.qm9_shape_dataset(64, seed=500 + i) for i in range(4)]
    run_loss = None
    k = 0
    noisy = {}
    for graphs in batches:
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _batch(graphs)
        opt.zero_grad()
        out = ref([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        loss = crit(out, normalize_data(T, mean, std))
        loss.backward()
        opt.step()
        lv = loss.item()
        run_loss = lv if run_loss is None else 0.9 * lv + 0.1 * run_loss
        if csr:
            inst = [[x, a, t] for x, a, t in graphs]
            stats = step(prepare_batch_csr(inst, 0, 1))
        else:
            stats = step([X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb])
        s = stats.cpu()
        assert abs(s[0].item() - lv) <= 1e-5 * max(1.0, abs(lv)), (s[0].item(), lv)
        assert abs(s[2].item() - run_loss) <= 1e-5 * max(1.0, abs(run_loss))
        k += 1
        gmax = max(q.grad.abs().max().item() for q in ref.parameters())
        for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
            # elements whose reference gradient is at the fp32 noise floor (analytically zero:
            # a BN mean subtraction follows a linear or all-active ReLU channel)
            # have no defined sign, and Adamax turns any |g| >> eps into a full lr-sized step
            noisy[n] = noisy.get(n, torch.zeros_like(q, dtype=torch.bool)) | (q.grad.abs() <= 1e-4 * gmax)
            err = (p.detach() - q.detach()).abs()
            tight = err[~noisy[n]]
            assert tight.numel() == 0 or tight.max().item() <= 1e-5 * max(1.0, q.abs().max().item()), \
                (n, tight.max().item())
            assert err.max().item() <= 2 * lr, (n, err.max().item())
        # re-synchronise (params + Adamax state) so every step is compared from equal states:
        # noise-driven lr-sized differences would otherwise compound across batches
        with torch.no_grad():
            for i, (p, q) in enumerate(zip(model.parameters(), ref.parameters())):
                p.copy_(q)
                st = opt.state[q]
                step.exp_avg[i].copy_(st["exp_avg"])
                step.exp_inf[i].copy_(st["exp_inf"])
        noisy = {}


def test_train_step_vs_fp64_oracle_two_steps():
    """TrainStep against the fp64 oracle (oracle/ref_mnb.py) with torch's Adamax on the oracle's
    parameters: two steps of scripts/train_mnb.py:41-91 on different batches, no re-synchronisation.
    Adamax's first steps move a parameter by ~lr * sign(g): every element whose oracle gradient is
    above the noise floor (1e-4 max|g|) must land within 1e-5 * max(1, |p|) of the oracle's; the
    others (analytically zero gradients) within 2 lr per step."""
    import hgnn_amd.datagen as dg
    from functions.utils import normalize_data
    from hgnn_amd.train import TrainStep
    from models.gnns.model_mnb import GNN_lg
    from oracle import ref_mnb as R
    torch.manual_seed(31)
    L, order, mean, std, lr = 4, 2, 0.3, 1.7, 1e-3
    model = GNN_lg(0, 16, L, 5, 1, 1, order).cuda()
    p64 = {k: v.detach().cpu().double().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    names = [k for k, _ in model.named_parameters()]
    opt = torch.optim.Adamax([p64[k] for k in names], lr=lr)
    st = R.bn_states(L, 2 * model.n_features, dtype=torch.float64)
    step = TrainStep(model, lr=lr, t_mean=mean, t_std=std)
    noisy = {k: torch.zeros_like(p64[k], dtype=torch.bool) for k in names}
    for i in range(2):
        b = _batch(dg.qm9_shape_dataset(48, seed=900 + i))
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cpu() for t in b]
        opt.zero_grad()
        out = R.gnn_lg(p64, [X.double(), XL.double(), W.double(), WL.double(), Pm.double(), Pd.double()], Nb,
                       mask.double(), Eb, mask_lg.double(), L, order, st, True)
        loss = torch.nn.MSELoss()(out, normalize_data(T.double(), mean, std))
        loss.backward()
        gmax = max(p64[k].grad.abs().max().item() for k in names)
        for k in names:
            noisy[k] |= p64[k].grad.abs() <= 1e-4 * gmax
        opt.step()
        s = step(b).cpu()
        assert abs(s[0].item() - loss.item()) <= 1e-5 * max(1.0, abs(loss.item())), (i, s[0].item(), loss.item())
        for k, p in model.named_parameters():
            q = p64[k].detach()
            err = (p.detach().cpu().double() - q).abs()
            tight = err[~noisy[k]]
            assert tight.numel() == 0 or tight.max().item() <= 1e-5 * max(1.0, q.abs().max().item()), \
                (i, k, tight.max().item())
            assert err.max().item() <= 2 * lr * (i + 1) + 1e-6, (i, k, err.max().item())


def test_adamax_kernel_matches_torch_exactly_on_fixed_grads():
    """The optimizer alone, on identical gradients: elementwise agreement to 1 ulp-scale."""
    from hgnn_amd import _lib as L
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(64, 271, 1), (64,), (), (1, 640, 1), (5000,)]
    ps = [torch.randn(s, generator=g).cuda() for s in shapes]
    qs = [p.clone().requires_grad_(True) for p in ps]
    opt = torch.optim.Adamax(qs, lr=3e-4, weight_decay=0.01)
    m = [torch.zeros_like(p) for p in ps]
    u = [torch.zeros_like(p) for p in ps]
    import ctypes
    numel = (ctypes.c_int64 * len(ps))(*[p.numel() for p in ps])
    for t in range(1, 6):
        grads = [torch.randn(s, generator=g).cuda() for s in shapes]
        for q, gr in zip(qs, grads):
            q.grad = gr.clone()
        opt.step()
        L.check(L.lib().hgnn_adamax_step(len(ps), L.ptr_array(ps), L.ptr_array(grads), L.ptr_array(m),
                                         L.ptr_array(u), numel, 3e-4, 0.9, 0.999, 1e-8, 0.01, t,
                                         L.stream_handle(ps[0].device)), "adamax")
        for p, q in zip(ps, qs):
            assert torch.allclose(p, q.detach(), rtol=0, atol=1e-7 * max(1.0, q.abs().max().item()))


def test_train_step_classification_matches_cross_entropy_adamax():
    """mean == 0 (generated data): T -> class indices, nn.CrossEntropyLoss (scripts/train_mnb.py:50-51,
    scripts/main_generate.py:147); the device step against torch's loss + Adamax from equal states."""
    import hgnn_amd.datagen as dg
    from hgnn_amd.train import TrainStep
    from models.gnns.model_mnb import GNN_lg
    torch.manual_seed(21)
    model = GNN_lg(0, 16, 4, 5, 3, 1, 2).cuda()  # dim_output = 3 classes
    ref = copy.deepcopy(model)
    lr = 1e-3
    opt = torch.optim.Adamax(ref.parameters(), lr=lr)
    crit = torch.nn.CrossEntropyLoss()
    step = TrainStep(model, lr=lr, t_mean=0.0)
    assert step.classification
    run_loss = None
    for i in range(3):
        graphs = dg.qm9_shape_dataset(48, seed=700 + i)
        b = _batch(graphs)
        b[2] = torch.randint(0, 3, (48, 1), generator=torch.Generator().manual_seed(i)).float().cuda()
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = b
        opt.zero_grad()
        out = ref([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        loss = crit(out, T.squeeze().long())
        loss.backward()
        opt.step()
        lv = loss.item()
        run_loss = lv if run_loss is None else 0.9 * lv + 0.1 * run_loss
        s = step(b).cpu()
        step.check_targets()
        assert abs(s[0].item() - lv) <= 1e-5 * max(1.0, abs(lv)), (s[0].item(), lv)
        assert abs(s[2].item() - run_loss) <= 1e-5 * max(1.0, abs(run_loss))
        assert s[1].item() == 0.0 and s[3].item() == 0.0  # no MAE for classes
        gmax = max(q.grad.abs().max().item() for q in ref.parameters())
        for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
            quiet = q.grad.abs() > 1e-4 * gmax
            err = (p.detach() - q.detach()).abs()
            assert err[quiet].numel() == 0 or err[quiet].max().item() <= 1e-5 * max(1.0, q.abs().max().item()), n
            assert err.max().item() <= 2 * lr, n
        with torch.no_grad():
            for k, (p, q) in enumerate(zip(model.parameters(), ref.parameters())):
                p.copy_(q)
                st = opt.state[q]
                step.exp_avg[k].copy_(st["exp_avg"])
                step.exp_inf[k].copy_(st["exp_inf"])
    bad = _batch(dg.qm9_shape_dataset(4, seed=9))
    bad[2] = torch.tensor([[0.0], [5.0], [1.0], [2.0]]).cuda()
    # HGNN_STRICT=1 (conftest): the step raises at once
    with pytest.raises(RuntimeError, match="class target"):
        step(bad)
    # asynchronous check: the rejected row's dout is zero (finite parameters), the next check raises
    os.environ["HGNN_STRICT"] = "0"
    try:
        step(bad)
        torch.cuda.synchronize()
        assert all(torch.isfinite(p).all() for p in model.parameters())
        with pytest.raises(RuntimeError, match="class target"):
            step.check_targets()
        step.check_targets()  # the error word was consumed
    finally:
        os.environ["HGNN_STRICT"] = "1"


def test_train_step_defaults_to_regression():
    """TrainStep(model) with no t_mean is the MSE step; classification over one class is refused."""
    from hgnn_amd.train import TrainStep
    from models.gnns.model_mnb import GNN_lg
    model = GNN_lg(0, 8, 3, 5, 1, 1, 2).cuda()
    assert not TrainStep(model).classification
    assert TrainStep(model, t_mean=0.0).classification
    import hgnn_amd.datagen as dg
    b = _batch(dg.qm9_shape_dataset(4, seed=19))
    with pytest.raises(RuntimeError, match="dim_output >= 2"):
        TrainStep(model, t_mean=0.0)(b)
