#!/usr/bin/env python3
"""How much the reference's OWN fp32 error moves with the summation order (review r05 #8).

The two-leg output policy (SURVEY.md §8 c) bounds |gpu - ref64| by 2 x max|ref32 - ref64|: the GPU's fp32 error may be
twice the reference fp32's.  For the two relaxed cases (GNN_lg J = 4, GNN_simple J = 2 on SBM-50) this tool runs the
reference restatement (oracle/ref_mnb.py, the reference's op order) in fp32 and fp64 on the same graphs with their nodes
relabelled by random permutations -- the same function of the same graphs (the networks are permutation-equivariant),
only the order of every graph_oper / P_multi / BN summation changes -- and prints max|ref32 - ref64| per relabelling as
a ratio to the identity order's.  A spread of these ratios above 2 means the factor-2 bound fails the reference itself
under an equally valid summation order: the error is set by cancellation in the aggregation sums (A^8 entries of the
weighted QM9 adjacencies reach ~1e8 against BN'd inputs of mean 0), not by any kernel.  CPU only.

usage: python tools/parity_order_spread.py [--perms 12]"""
import argparse
import os
import statistics as st
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO, os.path.join(REPO, "tests", "golden")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--perms", type=int, default=12)
    a = ap.parse_args()
    import fixture_util as fu
    import hgnn_amd.datagen as dg
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    from models.gnns.model_mnb import GNN_lg, GNN_simple
    from oracle import ref_mnb as R

    cases = [
        # (name, graphs, J, model, layers, kind) -- the GPU tests' own cases
        ("GNN_lg J=4 d=16 L=4 order 2, 32 QM9-shape graphs (test_large_J_vs_oracle_fp64)",
         dg.qm9_shape_dataset(32, seed=44), 4, ("lg", 16, 4, 504)),
        ("GNN_simple J=2 d=8 L=6, 24 SBM-50 graphs (test_gnn_simple_j2_vs_oracle)",
         dg.sbm_dataset(24, n=50, seed=5), 2, ("simple", 8, 6, 61)),
    ]
    for name, graphs, J, (kind, d, L, seed) in cases:
        model = GNN_lg(0, d, L, 5, 1, J, 2) if kind == "lg" else GNN_simple(0, d, L, 5, 1, J)
        fu.det_init(model, seed)
        sd = model.state_dict()

        def err(gs):
            data = [[X, A, t, *graph_operators([X, A], J, True)] for X, A, t in gs]
            X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = list(prepare_batch(data, 0, J))

            def run(dtype):
                p = {k: v.detach().to(dtype) for k, v in sd.items()}
                with torch.no_grad():
                    if kind == "lg":
                        return R.gnn_lg(p, [X.to(dtype), XL.to(dtype), W.to(dtype), WL.to(dtype), Pm.to(dtype),
                                            Pd.to(dtype)], Nb, mask.to(dtype), Eb, mask_lg.to(dtype), L, 2,
                                        R.bn_states(L, 2 * d, dtype=dtype), True, fast=True)
                    return R.gnn_simple(p, [X.to(dtype), W.to(dtype)], Nb, mask.to(dtype), L,
                                        R.bn_states(L, 2 * d, "simple", dtype), True, fast=True)
            r64 = run(torch.float64).double()
            r32 = run(torch.float32).double()
            return (r32 - r64).abs().max().item(), r64.abs().max().item()

        e0, m0 = err(graphs)
        print(f"{name}\n  identity order: max|ref32 - ref64| = {e0:.4g} (max|out| {m0:.4g})", flush=True)
        gen = torch.Generator().manual_seed(7)
        rs = []
        for t in range(a.perms):
            gp = []
            for X, A, tt in graphs:
                p = torch.randperm(X.shape[0], generator=gen)
                gp.append((X[p], A[p][:, p], tt))
            e, _ = err(gp)
            rs.append(e / e0)
            print(f"  relabelling {t:2d}: max|ref32 - ref64| = {e:.4g}  ratio {e / e0:.2f}", flush=True)
        print(f"  ratio over {a.perms} relabellings: min {min(rs):.2f}, median {st.median(rs):.2f}, max {max(rs):.2f}; "
              f"{sum(r > 2 for r in rs)} of {a.perms} above the policy's factor 2", flush=True)


if __name__ == "__main__":
    main()
