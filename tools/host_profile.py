"""cProfile of the headline step's host side (what the CPU does per eager step).
usage: python tools/host_profile.py [--steps 30]"""
import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from models.gnns.model_mnb import GNN_lg
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).to(dev)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.to(dev) for t in bench.make_batch(512, 1000, 1, 0)]
    X.requires_grad_(True)
    W.requires_grad_(True)
    crit = torch.nn.MSELoss()
    params = list(model.parameters())

    def step():
        for p in params:
            p.grad = None
        X.grad = None
        W.grad = None
        crit(model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg), T).backward()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    n = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 30
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
