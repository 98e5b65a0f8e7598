"""Same-process A/B of the per-graph CCN-1D drop-in step (scripts/train_ccn.py:31-73 shape): epochs over
the same 256 QM9-shape graphs alternate between the general path and the small-graph path
(hgnn_amd.ccn.SMALL); per path the min and median ms per graph over the epochs.  Also the batched
config-3 step (256 graphs fwd+bwd) the same way."""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO, os.path.join(REPO, "tools")]
import torch  # noqa: E402


def main():
    import hgnn_amd.ccn as HC
    import hgnn_amd.datagen as dg
    from models.compnets.model_ccn import CCN_1D
    from tools_bc import ccn_pad
    graphs = dg.qm9_shape_dataset(256, seed=7)
    torch.manual_seed(0)
    net = CCN_1D(5, 1, 2, 2).cuda()
    opt = torch.optim.Adamax(net.parameters(), lr=1e-3)
    crit = torch.nn.MSELoss()
    data = [(x.cuda(), (a + torch.eye(a.shape[0])).cuda(), t[0].view(1).cuda()) for x, a, t in graphs]
    X, A, nb = ccn_pad(graphs)
    T = torch.stack([t[0] for _, _, t in graphs]).view(-1, 1).cuda()

    def epoch():
        for x, a, t in data:
            opt.zero_grad()
            loss = crit(net(x, a), t)
            loss.backward()
            opt.step()

    def batched():
        net.zero_grad(set_to_none=True)
        out = net.forward_batch(X, A, nb)
        ((out - T) ** 2).sum().backward()

    res = {}
    for name, fn, reps, per in (("pergraph", epoch, 1, 256), ("batched", batched, 20, 1)):
        times = {0: [], 1: []}
        for it in range(12):
            for sm in (0, 1):
                HC.SMALL = bool(sm)
                fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    fn()
                torch.cuda.synchronize()
                if it >= 2:
                    times[sm].append((time.perf_counter() - t0) * 1e3 / reps / per)
        for sm in (0, 1):
            res[f"{name}_{'small' if sm else 'general'}_ms"] = {"min": round(min(times[sm]), 4),
                                                               "median": round(statistics.median(times[sm]), 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
