"""Checkpoint compatibility: whole-module checkpoints written by the
reference (torch.save(model), functions/logs.py:99-111; reloaded with torch.load,
scripts/main_gnn_qm9.py:149-151) load into the drop-in classes.

The fixture tests/golden/ckpt_lg_ref.pt was written by tests/golden/make_ckpt.py with
the reference's own classes (a GNN_lg after one Adamax step, so its BN running
statistics are non-trivial); it is our generated file, loaded with weights_only=False.
"""

import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
CKPT = os.path.join(HERE, "golden", "ckpt_lg_ref.pt")


def load_ref_checkpoint():
    return torch.load(CKPT, map_location="cpu", weights_only=False)


def test_reference_checkpoint_loads_into_dropin_classes(golden):
    import models.gnns.model_mnb as mm
    import models.layers.batch_normalization as bnm
    z = golden("ckpt_lg_ref")
    model = load_ref_checkpoint()
    assert type(model) is mm.GNN_lg
    assert model.dual and model.J == 1 and model.order == 2 and model.n_layers == 3
    sd = model.state_dict()
    keys = sorted(k[3:] for k in z.files if k.startswith("sd."))
    assert sorted(sd.keys()) == keys
    for k in keys:
        assert np.array_equal(sd[k].numpy(), z["sd." + k]), k
    bns = [m for _, m in model.named_modules() if isinstance(m, bnm.BN)]
    assert len(bns) == 4
    for i, m in enumerate(bns):
        assert not m.running_mean.requires_grad
        assert np.array_equal(m.running_mean.numpy(), z[f"run.{i}.running_mean"])
        assert np.array_equal(m.running_std.numpy(), z[f"run.{i}.running_std"])


def test_dropin_checkpoint_round_trip(tmp_path):
    """torch.save(model) / torch.load of the drop-in itself (what Logger.save_model does)."""
    from models.gnns.model_mnb import GNN_lg
    m = GNN_lg(0, 8, 3, 5, 1, 1, 2)
    p = tmp_path / "gnn.pt"
    torch.save(m, p)
    m2 = torch.load(p, weights_only=False)
    for (n, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), n


@pytest.mark.gpu
def test_reference_checkpoint_runs_on_gpu(golden):
    """Eval-mode output of the reloaded reference checkpoint equals the reference's own."""
    import fixture_util as fu
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    z = golden("ckpt_lg_ref")
    model = load_ref_checkpoint().cuda().eval()
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in fu.unpack_graphs(z)]
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cuda() for t in prepare_batch(data, 0, 1)]
    with torch.no_grad():
        out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg).cpu().numpy()
    ref = z["out_eval"]
    assert np.abs(out - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max()), np.abs(out - ref).max()
