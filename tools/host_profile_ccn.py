"""cProfile of the per-graph CCN drop-in step's host side (config cfg3_pergraph: net(X, A + I), MSE,
backward, Adamax per graph, as scripts/train_ccn.py:31-73 runs it).
usage: python tools/host_profile_ccn.py [--order 1] [--graphs 256]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO, os.path.join(REPO, "tools")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", type=int, default=1)
    ap.add_argument("--graphs", type=int, default=256)
    args = ap.parse_args()
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D, CCN_2D
    graphs = dg.qm9_shape_dataset(args.graphs, seed=7)
    torch.manual_seed(0)
    net = (CCN_1D if args.order == 1 else CCN_2D)(5, 1, 2, 2).cuda()
    opt = torch.optim.Adamax(net.parameters(), lr=1e-3)
    crit = torch.nn.MSELoss()
    data = [(x.cuda(), (a + torch.eye(a.shape[0])).cuda(), t[0].view(1).cuda()) for x, a, t in graphs]

    def epoch():
        for x, a, t in data:
            opt.zero_grad()
            loss = crit(net(x, a), t)
            loss.backward()
            opt.step()

    for _ in range(3):
        epoch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        epoch()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / (3 * len(data))
    print(f"per graph {ms:.4f} ms (no profiler)", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    epoch()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(35)


if __name__ == "__main__":
    main()
