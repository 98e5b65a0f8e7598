"""Every kept kernel alternate of the executor under a parity test (review r05 #9).

The library reads its HGNN_* switches once per process (static initialisers), so each setting runs in a child
process (tests/switch_worker.py: GNN_lg order 2 at d = 64 and GNN_simple at d = 32, X and W requiring grad --
widths where the split-bf16 GEMMs and the diagonal I / D columns are active), and every setting is checked
against the fp64 oracle (oracle/ref_mnb.py) on SURVEY.md §8 c's bounds: outputs on the two-leg policy, every
parameter gradient, dX and dW on the gradient bound.  HGNN_DIAG_ID=1 (the I / D columns built by the GEMMs from the
half's input instead of aggregated) must give the default's results bit for bit: it hands the GEMMs the same
operand values.
"""

import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import parity as PP
from oracle import ref_mnb as R

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# groups of switches that do not shadow each other; each group is one child process
GROUPS = {
    "default": {},
    "diag_id_on": {"HGNN_DIAG_ID": "1"},
    "fp32_gemms": {"HGNN_FWD_BF3": "0", "HGNN_DA_BF3": "0", "HGNN_DW_BF3": "0", "HGNN_FWD_XCD": "0",
                   "HGNN_DA_XCD": "0", "HGNN_DW_XCD": "0", "HGNN_FWD_G5": "2"},
    "fp32_gemms_b": {"HGNN_FWD_BF3": "0", "HGNN_DA_BF3": "0", "HGNN_DW_BF3": "0", "HGNN_GEMM_DMA": "0",
                     "HGNN_FWD_G5": "0"},
    "alt_a": {"HGNN_DW_RING": "2", "HGNN_AGG_RPW": "1", "HGNN_BN_BWD2": "1", "HGNN_EXTRACT_REG": "0",
              "HGNN_DWD_GRID": "0", "HGNN_BWD_TAIL": "0", "HGNN_EVENT_FENCE": "1", "HGNN_READOUT_ROW": "0",
              "HGNN_SERIAL_BWD": "1", "HGNN_DW_NARROW": "0", "HGNN_BN_ACC": "0"},
    "alt_b": {"HGNN_DW_RING": "3", "HGNN_AGG_RPW": "4", "HGNN_SIDE": "0", "HGNN_EXTRACT_REG": "0",
              "HGNN_EXTRACT_LDS": "0", "HGNN_BN_BWD2": "0", "HGNN_EXEC_GRAPH": "0", "HGNN_EXTRACT_SPLIT": "1",
              "HGNN_BN_FWD_FIN": "0"},
}


def _run(name, env_extra, tmp):
    out = os.path.join(tmp, f"{name}.npz")
    env = dict(os.environ)
    for k in list(env):
        if k.startswith("HGNN_") and k != "HGNN_STRICT":
            del env[k]
    env.update(env_extra)
    env["HGNN_STRICT"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "switch_worker.py"), out], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, (name, r.stderr[-2000:])
    return dict(np.load(out))


def _oracle():
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import switch_worker as SW
    blg, bsm = SW.batches()
    lg, sm = SW.models()
    res = {}
    for dtype, grads in ((torch.float64, True), (torch.float32, False)):
        tag = "64" if dtype == torch.float64 else "32"
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = blg
        p = {k: v.detach().to(dtype).requires_grad_(grads) for k, v in lg.state_dict().items()}
        Xo, Wo = X.to(dtype).requires_grad_(grads), W.to(dtype).requires_grad_(grads)
        with torch.set_grad_enabled(grads):
            o = R.gnn_lg(p, [Xo, XL.to(dtype), Wo, WL.to(dtype), Pm.to(dtype), Pd.to(dtype)], Nb, mask.to(dtype), Eb,
                         mask_lg.to(dtype), 4, 2, R.bn_states(4, 128, dtype=dtype), True, fast=dtype == torch.float64)
        res["lg.out" + tag] = o.detach()
        if grads:
            torch.nn.MSELoss()(o, T.to(dtype)).backward()
            res["lg.g"] = {k: v.grad for k, v in p.items()}
            res["lg.dX"], res["lg.dW"] = Xo.grad, Wo.grad
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = bsm
        p = {k: v.detach().to(dtype).requires_grad_(grads) for k, v in sm.state_dict().items()}
        Xo, Wo = X.to(dtype).requires_grad_(grads), W.to(dtype).requires_grad_(grads)
        with torch.set_grad_enabled(grads):
            o = R.gnn_simple(p, [Xo, Wo], Nb, mask.to(dtype), 3, R.bn_states(3, 64, "simple", dtype), True)
        res["sm.out" + tag] = o.detach()
        if grads:
            torch.nn.MSELoss()(o, T.to(dtype)).backward()
            res["sm.g"] = {k: v.grad for k, v in p.items()}
            res["sm.dX"], res["sm.dW"] = Xo.grad, Wo.grad
    return res


def _check(name, got, ref):
    for m in ("lg", "sm"):
        o = PP.outputs_two_leg(torch.from_numpy(got[m + ".out"]), ref[m + ".out32"], ref[m + ".out64"])
        assert o["pass"], (name, m, o)
        g = ref[m + ".g"]
        gmax = max(v.abs().max().item() for v in g.values())
        for k, v in g.items():
            err = (torch.from_numpy(got[f"{m}.grad.{k}"]).double() - v).abs()
            assert torch.all(err <= 1e-4 * gmax + 1e-5 * v.abs()), (name, m, k, err.max().item(), gmax)
        for k in ("dX", "dW"):
            r = ref[f"{m}.{k}"]
            err = (torch.from_numpy(got[f"{m}.{k}"]).double() - r).abs().max().item()
            assert err <= 1e-4 * max(1.0, r.abs().max().item()), (name, m, k, err)


def test_kernel_switches_vs_oracle(tmp_path):
    ref = _oracle()
    runs = {name: _run(name, env, str(tmp_path)) for name, env in GROUPS.items()}
    for name, got in runs.items():
        _check(name, got, ref)
    a, b = runs["default"], runs["diag_id_on"]
    diff = [k for k in a if not np.array_equal(a[k], b[k])]
    assert not diff, f"diagonal I / D columns not bitwise equal to the general aggregation: {diff}"
