#!/usr/bin/env python3
"""Round-5 re-measurement of the three relaxed parity legs against the plain
SURVEY.md §8(c) policy, on the tests' own batches and weights:
  a) d = 128 dX (tests/test_gpu_fullsize.py::test_config4_rank_share_d128_512_vs_oracle,
     tests/test_gpu_net.py::test_gnn_lg_d128_config4_model_vs_oracle_fp64): |dX - dX64| vs 1e-4 max|dX64|;
  b) GNN_simple J = 2 (test_gnn_simple_j2_vs_oracle): the fp64 leg vs 2 |ref32 - ref64| + 1e-6;
  c) J = 4, 5 (test_large_J_vs_oracle_fp64): GNN_lg outputs vs the two-leg bound.
Prints one JSON line per case with the measured errors, the strict bounds and err / bound."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hgnn-2_amd"), os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import fixture_util as fu  # noqa: E402
import test_gpu_fullsize as F  # noqa: E402
import test_gpu_net as G  # noqa: E402
from oracle import parity as PP  # noqa: E402


def out(d):
    print(json.dumps(d), flush=True)


def case_d128_fullsize():
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    b = F._batch(dg.qm9_shape_dataset(512, seed=1004))
    model = GNN_lg(0, 128, 5, 5, 1, 1, 2).cuda()
    fu.det_init(model, 4)
    o, loss, g, dx, dw = F._gpu(model, b)
    _, _, _, dx64, _ = F._oracle(model, b, 5, 2, torch.float64, fast=True)
    _, _, _, dx32, _ = F._oracle(model, b, 5, 2, torch.float32, fast=True)
    err = (dx.cpu().double() - dx64).abs().max().item()
    strict = 1e-4 * max(1.0, dx64.abs().max().item())
    r32 = (dx32.double() - dx64).abs().max().item()
    out({"case": "d128 dX fullsize (512 graphs)", "err": err, "strict_bound": strict, "err_over_strict": err / strict,
         "ref32_err": r32, "ref32_over_strict": r32 / strict})


def case_d128_net():
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    b = G._batch(dg.qm9_shape_dataset(48, seed=12))
    model = GNN_lg(0, 128, 4, 5, 1, 1, 2).cuda()
    fu.det_init(model, 128)
    ref_out, ref_loss, ref_g, ref_dx = G._oracle_lg(model, b, 4, 2)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = G._cuda(b)
    X.requires_grad_(True)
    o = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    torch.nn.MSELoss()(o, T).backward()
    err = (X.grad.cpu().double() - ref_dx).abs().max().item()
    _, _, _, dx32 = G._oracle_lg(model, b, 4, 2, dtype=torch.float32)
    r32 = (dx32.double() - ref_dx).abs().max().item()
    strict = 1e-4 * max(1.0, ref_dx.abs().max().item())
    out({"case": "d128 dX net (48 graphs, L=4)", "err": err, "strict_bound": strict, "err_over_strict": err / strict,
         "ref32_err": r32, "ref32_over_strict": r32 / strict})


def case_d256():
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    b = F._batch(dg.qm9_shape_dataset(16, seed=256))
    model = GNN_lg(0, 256, 3, 5, 1, 1, 2).cuda()
    fu.det_init(model, 256, scale=0.05)
    o, loss, g, dx, dw = F._gpu(model, b)
    _, _, _, dx64, _ = F._oracle(model, b, 3, 2, torch.float64, fast=True)
    _, _, _, dx32, _ = F._oracle(model, b, 3, 2, torch.float32, fast=True)
    err = (dx.cpu().double() - dx64).abs().max().item()
    strict = 1e-4 * max(1.0, dx64.abs().max().item())
    r32 = (dx32.double() - dx64).abs().max().item()
    out({"case": "d256 dX (16 graphs, L=3)", "err": err, "strict_bound": strict, "err_over_strict": err / strict,
         "ref32_err": r32, "ref32_over_strict": r32 / strict})


def case_simple_j2():
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_simple
    b = F._batch(dg.sbm_dataset(24, n=50, seed=5), J=2)
    model = GNN_simple(0, 8, 6, 5, 1, 2).cuda()
    fu.det_init(model, 61)
    o, loss, g, dx, dw = F._gpu(model, b, "simple")
    r32 = F._oracle(model, b, 6, 0, torch.float32, fast=False, grads=False, kind="simple")[0]
    r64 = F._oracle(model, b, 6, 0, torch.float64, fast=True, grads=False, kind="simple")[0]
    res = PP.outputs_two_leg(o, r32, r64, 2.0)
    res.update({"case": "GNN_simple J=2 fp64 leg", "leg64_over_strict": res["max_abs_vs_ref64"] / res["bound_ref64"],
                "leg32_over_bound": res["max_abs_vs_ref32"] / res["bound_ref32"]})
    out(res)


def case_large_j(J):
    import hgnn_amd.datagen as dg
    from models.gnns.model_mnb import GNN_lg
    b = G._batch(dg.qm9_shape_dataset(32, seed=40 + J), J)
    model = GNN_lg(0, 16, 4, 5, 1, J, 2).cuda()
    fu.det_init(model, 500 + J)
    ref_out = G._oracle_lg(model, b, 4, 2)[0]
    with torch.no_grad():
        ref32 = G._oracle_lg(model, b, 4, 2, dtype=torch.float32, grads=False)[0]
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = G._cuda(b)
    with torch.no_grad():
        o = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
    res = PP.outputs_two_leg(o, ref32, ref_out, 2.0)
    res.update({"case": f"GNN_lg J={J} two-leg", "leg64_over_strict": res["max_abs_vs_ref64"] / res["bound_ref64"],
                "leg32_over_bound": res["max_abs_vs_ref32"] / res["bound_ref32"]})
    out(res)


if __name__ == "__main__":
    case_d128_fullsize()
    case_d128_net()
    case_d256()
    case_simple_j2()
    for J in (4, 5):
        case_large_j(J)
