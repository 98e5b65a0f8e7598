#!/usr/bin/env python3
"""Checkpoint-compatibility fixture, generated from the REAL reference.

The reference saves whole modules with torch.save(model) (functions/logs.py:99-111)
and reloads them with torch.load(path) (scripts/main_gnn_qm9.py:149-151).  This
script builds a reference GNN_lg (its own classes: models.gnns.model_mnb,
models.layers.*), trains it one step on CPU so the BN running statistics are
non-trivial, saves the whole module as the reference does, and records the
module's eval-mode and train-mode outputs on a fixture batch.  The drop-in
package has the same import paths, so the pickle resolves to the drop-in classes
when loaded beside it (tests/test_checkpoint.py, tests/test_gpu_checkpoint.py).

Run once in the survey container (where /root/reference exists):
    python tests/golden/make_ckpt.py
Writes tests/golden/ckpt_lg_ref.pt and tests/golden/ckpt_lg_ref.npz.
"""

import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, "/root/reference")
sys.path.insert(0, HERE)

import fixture_util as fu  # noqa: E402

spec = importlib.util.spec_from_file_location("datagen", os.path.join(REPO, "hgnn-2_amd", "hgnn_amd", "datagen.py"))
dg = importlib.util.module_from_spec(spec)
spec.loader.exec_module(dg)

from functions import batching as r_batch  # noqa: E402
from functions import operators as r_ops  # noqa: E402
from models.gnns import model_mnb as r_model  # noqa: E402


def main():
    torch.manual_seed(0)
    graphs = dg.qm9_shape_dataset(24, seed=909)
    data = [[X, A, t, *r_ops.graph_operators([X, A], 1, True)] for X, A, t in graphs]
    b = r_batch.prepare_batch(data, 0, 1)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = b
    model = r_model.GNN_lg(0, 8, 3, 5, 1, 1, 2)
    fu.det_init(model, 4242)
    opt = torch.optim.Adamax(model.parameters(), lr=1e-3)
    model.train()
    out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    torch.nn.MSELoss()(out, T).backward()
    opt.step()
    torch.save(model, os.path.join(HERE, "ckpt_lg_ref.pt"))
    with torch.no_grad():
        model.eval()
        out_eval = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    sd = {k: v.numpy() for k, v in model.state_dict().items()}
    np.savez_compressed(os.path.join(HERE, "ckpt_lg_ref.npz"), out_eval=out_eval.numpy(),
                        **fu.pack_graphs(graphs), **{"sd." + k: v for k, v in sd.items()},
                        **{f"run.{i}.{n}": getattr(m, n).detach().numpy()
                           for i, m in enumerate(mm for _, mm in model.named_modules() if hasattr(mm, "running_std"))
                           for n in ("running_mean", "running_std")})
    print("wrote ckpt_lg_ref.pt / .npz", out_eval.view(-1)[:4])


if __name__ == "__main__":
    main()
