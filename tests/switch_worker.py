"""Worker of tests/test_gpu_switches.py (run as a child process: the library reads its HGNN_* kernel switches once
per process).  One fwd+bwd of GNN_lg (order 2, d = 64, L = 4, 48 QM9-shape graphs, X and W requiring grad) and of
GNN_simple (d = 32, L = 3, 16 SBM-24 graphs, X and W requiring grad) on cuda:0; outputs, losses, every parameter
gradient, dX and dW saved to the .npz named on the command line."""

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "tests", "golden"), os.path.join(REPO, "hgnn-2_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def batches():
    import hgnn_amd.datagen as dg
    from functions.batching import prepare_batch
    from functions.operators import graph_operators

    def mk(graphs, dual):
        data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
        return list(prepare_batch(data, 0, 1))
    return mk(dg.qm9_shape_dataset(48, seed=4242), True), mk(dg.sbm_dataset(16, n=24, seed=4343), False)


def models():
    import fixture_util as fu
    from models.gnns.model_mnb import GNN_lg, GNN_simple
    lg = GNN_lg(0, 64, 4, 5, 1, 1, 2)
    fu.det_init(lg, 8181)
    sm = GNN_simple(0, 32, 3, 5, 1, 1)
    fu.det_init(sm, 8282)
    return lg, sm


def main(out):
    os.environ.setdefault("HGNN_STRICT", "1")
    blg, bsm = batches()
    lg, sm = models()
    res = {}
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cuda() for t in blg]
    lg = lg.cuda()
    X.requires_grad_(True)
    W.requires_grad_(True)
    o = lg([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    loss = torch.nn.MSELoss()(o, T)
    loss.backward()
    res["lg.out"] = o.detach().cpu().numpy()
    res["lg.loss"] = np.array(loss.item())
    res["lg.dX"] = X.grad.cpu().numpy()
    res["lg.dW"] = W.grad.cpu().numpy()
    for k, p in lg.named_parameters():
        res["lg.grad." + k] = p.grad.cpu().numpy()
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cuda() for t in bsm]
    sm = sm.cuda()
    X.requires_grad_(True)
    W.requires_grad_(True)
    o = sm([X, W], Nb, mask)
    loss = torch.nn.MSELoss()(o, T)
    loss.backward()
    res["sm.out"] = o.detach().cpu().numpy()
    res["sm.loss"] = np.array(loss.item())
    res["sm.dX"] = X.grad.cpu().numpy()
    res["sm.dW"] = W.grad.cpu().numpy()
    for k, p in sm.named_parameters():
        res["sm.grad." + k] = p.grad.cpu().numpy()
    torch.cuda.synchronize()
    from hgnn_amd.net import check_errors
    check_errors()
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1])
