"""GPU parity at the BASELINE.json sizes (SURVEY.md §8 c policy, oracle/parity.py).

* config 2 at its real size: GNN_lg order 2, d=64, L=5 on the 512-graph QM9-shape batch;
* config 4's per-rank share: GNN_lg d=128, L=5 on 512 graphs;
* the executor's J > 1 instantiations (J+2 = 4 and 5 operator slices,
  functions/operators.py:25-29) for every order and for GNN_simple.

Outputs: two legs -- the reference-order fp32 oracle (per-graph torch.mm loops,
oracle/ref_mnb.py, forward only) and the fp64 oracle.  Gradients: against the
fp64 oracle, batched leg (oracle/ref_mnb.py graph_oper_fast, pinned to the loop
leg by tests/test_oracle.py::test_oracle_fast_leg_equals_loop_leg).
"""

import pytest
import torch

import fixture_util as fu
from oracle import parity as PP
from oracle import ref_mnb as R

pytestmark = pytest.mark.gpu


def _batch(graphs, J=1):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    data = [[X, A, t, *graph_operators([X, A], J, True)] for X, A, t in graphs]
    return list(prepare_batch(data, 0, J))


def _oracle(model, b, L, order, dtype, fast, grads=True, kind="lg"):
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = b
    p = {k: v.detach().cpu().to(dtype).requires_grad_(grads) for k, v in model.state_dict().items()}
    st = R.bn_states(L, 2 * model.n_features, kind=kind, dtype=dtype)
    Xo = X.to(dtype).requires_grad_(grads)
    Wo = W.to(dtype).requires_grad_(grads)
    with torch.set_grad_enabled(grads):
        if kind == "lg":
            out = R.gnn_lg(p, [Xo, XL.to(dtype), Wo, WL.to(dtype), Pm.to(dtype), Pd.to(dtype)], Nb,
                           mask.to(dtype), Eb, mask_lg.to(dtype), L, order, st, True, fast=fast)
        else:
            out = R.gnn_simple(p, [Xo, Wo], Nb, mask.to(dtype), L, st, True, fast=fast)
        loss = torch.nn.MSELoss()(out, T.to(dtype))
        if not grads:
            return out.detach(), loss.item(), None, None, None
        loss.backward()
    return out.detach(), loss.item(), {k: v.grad for k, v in p.items()}, Xo.grad, Wo.grad


def _gpu(model, b, kind="lg"):
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cuda() for t in b]
    X.requires_grad_(True)
    W.requires_grad_(True)
    out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg) if kind == "lg" else model([X, W], Nb, mask)
    loss = torch.nn.MSELoss()(out, T)
    loss.backward()
    torch.cuda.synchronize()
    return out.detach(), loss.item(), {k: p.grad for k, p in model.named_parameters()}, X.grad, W.grad


def _check(model, b, L, order, kind="lg", factor=2.0):
    out, loss, g, dx, dw = _gpu(model, b, kind)
    r32, l32, _, _, _ = _oracle(model, b, L, order, torch.float32, fast=False, grads=False, kind=kind)
    r64, l64, g64, dx64, dw64 = _oracle(model, b, L, order, torch.float64, fast=True, kind=kind)
    o = PP.outputs_two_leg(out, r32, r64, factor)
    assert o["pass"], o
    assert abs(loss - l32) <= 1e-5 * max(1.0, abs(l32)), (loss, l32)
    gr = PP.grads_global(g, g64)
    assert gr["pass"], gr
    dwr = PP.grads_global({"dW": dw}, {"dW": dw64})
    assert dwr["pass"], dwr
    err = (dx.cpu().double() - dx64).abs().max().item()
    # strict at every width since round 5: d = 128 / 256 dX at 0.04 / 0.002 of this bound with the split-bf16
    # GEMMs (tools/parity_margins.py, profiles/r05_parity_margins.jsonl)
    bound = 1e-4 * max(1.0, dx64.abs().max().item())
    assert err <= bound, (err, bound)
    return o, gr


def test_config2_full_batch_512_vs_oracle():
    """The headline workload itself: 512 QM9-shape graphs, GNN_lg(0, 64, 5, 5, 1, 1, 2)."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    b = _batch(dg.qm9_shape_dataset(512, seed=1000))
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).cuda()
    fu.det_init(model, 2)
    _check(model, b, 5, 2)


def test_config4_rank_share_d128_512_vs_oracle():
    """Config 4's per-GPU share: GNN_lg d = 128 (2d = 256 channels), L = 5, 512 graphs."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    b = _batch(dg.qm9_shape_dataset(512, seed=1004))
    model = GNN_lg(0, 128, 5, 5, 1, 1, 2).cuda()
    fu.det_init(model, 4)
    # the plain §8(c) dX bound (measured round 5 at 0.037 of it, profiles/r05_parity_margins.jsonl; the
    # round-2..4 fallback to twice the reference's fp32 error is no longer taken)
    _check(model, b, 5, 2)


@pytest.mark.parametrize("J,order", [(2, 1), (2, 2), (2, 3), (3, 2)])
def test_executor_more_operator_slices_vs_oracle(J, order):
    """J = 2 / 3: W = [I, D, A, A^2(, A^4)] (functions/operators.py:25-29) -> the jtot 4 / 5 kernels."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    b = _batch(dg.qm9_shape_dataset(64, seed=60 + 10 * J + order), J=J)
    assert b[1].shape[3] == J + 2
    model = GNN_lg(0, 16, 4, 5, 1, J, order).cuda()
    fu.det_init(model, 20 + J)
    _check(model, b, 4, order)


def test_gnn_simple_j2_vs_oracle():
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_simple
    b = _batch(dg.sbm_dataset(24, n=50, seed=5), J=2)
    model = GNN_simple(0, 8, 6, 5, 1, 2).cuda()
    fu.det_init(model, 61)
    # outputs reach |y| = 412 here (SBM-50, A^2 slice): measured |gpu - ref64| = 1.33e-3 against the
    # reference fp32's own 5.2e-4 (3.2e-6 vs 1.3e-6 relative), inside the first leg (1e-5 relative) but
    # 2.6x the reference's error, so the fp64 leg is held at 3x here (re-measured round 5: 1.34x the
    # strict 2x bound, profiles/r05_parity_margins.jsonl).  Where it enters (round 6,
    # tools/parity_order_spread.py -> profiles/r06_parity_order_spread.txt): the reference's OWN fp32 error on
    # these graphs moves 0.53x-3.07x (median 1.08x) with a mere relabelling of the nodes -- the same function,
    # only the order of the graph_oper / BN sums changed -- 3 of 12 relabellings above 2x: the summation order
    # of the aggregation sets it, not a kernel, so the 3x leg stays
    _check(model, b, 6, 0, kind="simple", factor=3.0)


@pytest.mark.parametrize("d", [1, 3])
@pytest.mark.parametrize("order", [1, 2, 3])
def test_gnn_lg_odd_widths_vs_oracle(d, order):
    """2d = 2 / 6 output channels (n_features = 1 is the reference driver's default,
    scripts/main_gnn_qm9.py:78, and scripts/exp_lggnn_qm9.sh's h=1): the padded-stride path of
    the Conv1d-pair GEMMs (dY and the repacked WT at a row stride of 2d rounded up to 4, the
    scalar BN-backward apply zeroing the padding) against the oracle -- outputs on the two-leg
    bound, loss, every parameter grad, dX and the dense W.grad (model_mnb.py:69-129)."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    b = _batch(dg.qm9_shape_dataset(64, seed=500 + 10 * d + order))
    model = GNN_lg(0, d, 5, 5, 1, 1, order).cuda()
    fu.det_init(model, 510 + 10 * d + order)
    _check(model, b, 5, order)


@pytest.mark.parametrize("d", [1, 3])
def test_gnn_simple_odd_widths_vs_oracle(d):
    """GNN_simple at 2d = 2 / 6 (scripts/main_gnn.py with --h 1 / 3) on 24 SBM-50 graphs."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_simple
    b = _batch(dg.sbm_dataset(24, n=50, seed=520 + d))
    model = GNN_simple(0, d, 5, 5, 1, 1).cuda()
    fu.det_init(model, 530 + d)
    _check(model, b, 5, 0, kind="simple")


def test_gnn_lg_d256_readout_row_beyond_64kb_lds():
    """2d = 512 (d = 256, the widest valid_config width) with W.requires_grad: the readout-row dense
    dW kernel needs ~66 KB of LDS at QM9 Nmax = 29 (allowed per kernel up to the CU's 160 KB)."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    b = _batch(dg.qm9_shape_dataset(16, seed=256))
    model = GNN_lg(0, 256, 3, 5, 1, 1, 2).cuda()
    fu.det_init(model, 256, scale=0.05)
    _check(model, b, 3, 2)


def test_gnn_simple_large_nmax_readout_fallback():
    """Nmax = 400 (SBM-400) at 2d = 128: the readout-row kernels' LDS (rows of the graph) exceeds
    160 KB, so the executor takes the materialised [rows][K] readout gradient instead -- still every
    gradient incl. W.grad against the oracle."""
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_simple
    b = _batch(dg.sbm_dataset(3, n=400, seed=400))
    assert b[0].shape[2] == 400
    model = GNN_simple(0, 64, 3, 5, 1, 1).cuda()
    fu.det_init(model, 400, scale=0.05)
    _check(model, b, 3, 0, kind="simple")
