"""Where the headline's fp64 parity leg is spent: the bench batch (512 QM9-shape graphs, d = 64, order 2,
training-mode BN) through GNN_lg truncated to L = 2..5 layers, each on the GPU executor, the fp32 oracle
(the reference's op order) and the fp64 oracle.  Per depth: max |gpu - ref64|, max |ref32 - ref64| and
their ratio against bench.py's bound (2 max|ref32 - ref64| + 1e-6), plus the graphs where the GPU error
is largest.  usage: python tools/parity_depth.py [--depths 2,3,4,5] [--bs 512]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depths", default="2,3,4,5")
    ap.add_argument("--bs", type=int, default=512)
    ap.add_argument("--d", type=int, default=64)
    a = ap.parse_args()
    import bench
    from models.gnns.model_mnb import GNN_lg
    from oracle import ref_mnb as R
    batch_cpu = bench.make_batch(a.bs, 1000)
    dev = torch.device("cuda", 0)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.to(dev) for t in batch_cpu]
    for L in [int(x) for x in a.depths.split(",")]:
        torch.manual_seed(0)
        model = GNN_lg(0, a.d, L, 5, 1, 1, 2).to(dev)
        with torch.no_grad():
            gpu = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg).double().cpu()
        sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}

        def run(dtype, fast):
            p = {k: v.to(dtype) for k, v in sd.items()}
            st = R.bn_states(L, 2 * a.d, dtype=dtype)
            Xc, Wc, _, XLc, WLc, Pmc, Pdc, mc, mlc, Nbc, Ebc = batch_cpu
            with torch.no_grad():
                return R.gnn_lg(p, [Xc.to(dtype), XLc.to(dtype), Wc.to(dtype), WLc.to(dtype), Pmc.to(dtype),
                                    Pdc.to(dtype)], Nbc, mc.to(dtype), Ebc, mlc.to(dtype), L, 2, st, True,
                                fast=fast).double()

        r32 = run(torch.float32, False)
        r64 = run(torch.float64, True)
        eg = (gpu - r64).abs().view(-1)
        er = (r32 - r64).abs().view(-1)
        bound = 2 * er.max().item() + 1e-6
        top = torch.topk(eg, 5)
        print(json.dumps({"layers": L, "max_abs_gpu_vs_ref64": eg.max().item(), "max_abs_ref32_vs_ref64": er.max().item(),
                          "frac_of_bound": eg.max().item() / bound, "max_abs_gpu_vs_ref32": (gpu - r32).abs().max().item(),
                          "mean_abs_gpu_vs_ref64": eg.mean().item(), "mean_abs_ref32_vs_ref64": er.mean().item(),
                          "max_abs_out": r64.abs().max().item(),
                          "worst_graphs": [[int(i), round(float(v), 9), round(float(er[i]), 9), round(float(r64.view(-1)[i]), 4)]
                                           for v, i in zip(top.values, top.indices)],
                          "env": {k: v for k, v in os.environ.items() if k.startswith("HGNN_")}}), flush=True)


if __name__ == "__main__":
    main()
