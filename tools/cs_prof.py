"""Phase cycles of the small-graph CCN forward (HGNN_CCN_SMALL_PROF=1 build hook): one QM9 graph, repeated."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO, os.path.join(REPO, "tools")]
import torch  # noqa: E402


def main():
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D
    g = dg.qm9_shape_dataset(4, seed=7)
    net = CCN_1D(5, 1, 2, 2).cuda()
    for X, A, _ in g:
        x, a = X.cuda(), (A + torch.eye(A.shape[0])).cuda()
        for _ in range(3):
            with torch.no_grad():
                net(x, a)
            torch.cuda.synchronize()
    # a batch of 256
    from tools_bc import ccn_pad
    X, A, nb = ccn_pad(dg.qm9_shape_dataset(256, seed=8))
    for _ in range(3):
        with torch.no_grad():
            net.forward_batch(X, A, nb)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
