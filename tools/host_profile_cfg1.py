"""cProfile of config 1's eager step (GNN_simple(0, 2, 20, 5, 1, 1), 32 SBM-50 graphs): where the host
time of a launch-bound step goes.  usage: python tools/host_profile_cfg1.py [--steps 30]"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO, os.path.join(REPO, "tools")]
import torch  # noqa: E402


def main():
    from bench_configs import lg_batch
    from models.gnns.model_mnb import GNN_simple
    torch.manual_seed(0)
    model = GNN_simple(0, 2, 20, 5, 1, 1).cuda()
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = lg_batch(32, 1000, sbm_n=50)
    X.requires_grad_(True)
    W.requires_grad_(True)
    crit = torch.nn.MSELoss()

    def step():
        for p in model.parameters():
            p.grad = None
        X.grad = W.grad = None
        crit(model([X, W], Nb, mask), T).backward()

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    n = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 30
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"eager: host enqueue {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step")
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
