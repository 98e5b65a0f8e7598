"""Host-side drop-ins (CPU): operator construction, batching, index lists, ABI library surface."""

import ctypes
import os
import re
import time

import numpy as np
import pytest
import torch

import fixture_util as fu
from oracle import ref_mnb as R

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_graph_operators_bit_exact_vs_reference(golden):
    from functions.operators import graph_operators
    z = golden("operators")
    graphs = fu.unpack_graphs(z)
    for k, ((X, A, _), J) in enumerate(zip(graphs, z["J"])):
        W, WL, Pm, Pd = graph_operators([X, A], int(J), True)
        Wonly = graph_operators([X, A], int(J), False)
        assert torch.equal(W, Wonly)
        for nm, v in (("W", W), ("WL", WL), ("Pm", Pm), ("Pd", Pd)):
            ref = z[f"{nm}_{k}"]
            assert v.shape == ref.shape, (k, nm)
            assert v.dtype == torch.float32
            assert np.array_equal(v.numpy(), ref), (k, nm)


def test_graph_operators_random_vs_oracle():
    """Seeded random graphs (weights, self loops, isolated nodes) against the loop restatement."""
    from functions.operators import graph_operators
    g = torch.Generator().manual_seed(7)
    for trial in range(40):
        n = int(torch.randint(2, 14, (1,), generator=g))
        A = (torch.rand(n, n, generator=g) < 0.35).float()
        A = torch.triu(A, 1)
        wts = torch.tensor([1.0, 1.5, 2.0, 3.0])[torch.randint(0, 4, (n, n), generator=g)]
        A = A * wts
        A = A + A.t()
        if trial % 5 == 0:
            A[0, 0] = 1.0
        X = torch.zeros(n, 5)
        J = 1 + trial % 2
        got = graph_operators([X, A], J, True)
        ref = R.graph_operators([X, A], J, True)
        for a, b in zip(got, ref):
            assert torch.equal(a, b)


def test_graph_operators_faster_than_loops():
    from functions.operators import graph_operators
    import hgnn_amd.datagen as dg
    X, A, _ = dg.sbm_dataset(1, n=50, seed=3)[0]
    t0 = time.perf_counter()
    graph_operators([X, A], 1, True)
    assert time.perf_counter() - t0 < 0.5


def test_prepare_batch_bit_exact_vs_reference(golden):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    z = golden("batch")
    data = []
    for X, A, t in fu.unpack_graphs(z):
        W, WL, Pm, Pd = graph_operators([X, A], 1, True)
        data.append([X, A, t, W, WL, Pm, Pd])
    out = prepare_batch(data, 0, 1)
    names = ["X", "W", "T", "XL", "WL", "Pm", "Pd", "mask", "mask_lg", "N_batch", "E_batch"]
    for nm, v in zip(names, out):
        assert v.dtype == torch.from_numpy(z[nm]).dtype, nm
        assert np.array_equal(v.numpy(), z[nm]), nm


def test_get_batches_index_lists(golden):
    from functions.batching import get_batches
    z = golden("batch")
    flat = list(z["batches_23_5"])
    sep = flat.index(-1)
    idx, lens = flat[:sep], flat[sep + 1:]
    got = get_batches(23, 5, None, False, False)
    assert [len(b) for b in got] == lens
    assert [i for b in got for i in b] == idx


def test_normalize_data_semantics():
    from functions.utils import normalize_data, RunningAverage
    x = torch.tensor([1.0, 2.0, 3.0])
    assert torch.equal(normalize_data(x, 1.0, 1e-6), x - 1.0)  # std < 1e-5: mean only (Q14)
    assert torch.allclose(normalize_data(x, 2.0, 2.0), (x - 2.0) / 2.0)
    r = RunningAverage()
    r.update(4.0)
    r.update(2.0)
    assert r.val == pytest.approx(0.9 * 2.0 + 0.1 * 4.0)


# ----------------------------------------------------------------------------- C ABI surface
def _header_functions():
    src = open(os.path.join(REPO, "include", "hgnn_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hgnn_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from hgnn_amd import _lib
    lib = _lib.lib()
    names = _header_functions()
    assert len(names) >= 10
    for nm in names:
        assert hasattr(lib, nm), nm
    assert lib.hgnn_abi_version() == 1
    assert set(names) <= set(_lib.SIGNATURES), set(names) - set(_lib.SIGNATURES)


def _cfg(**kw):
    from hgnn_amd import _lib
    c = _lib.NetConfig()
    base = dict(kind=1, order=2, bs=512, nmax=29, emax=70, f_in=5, d=64, n_layers=5, j_tot=3, dim_out=1, training=1)
    base.update(kw)
    for k, v in base.items():
        setattr(c, k, v)
    return c


def test_workspace_and_counts_host_only():
    from hgnn_amd import _lib
    lib = _lib.lib()
    c = _cfg()
    assert lib.hgnn_net_param_count(ctypes.byref(c)) == 12 * 4 + 2
    assert lib.hgnn_net_bn_count(ctypes.byref(c)) == 8
    ws = lib.hgnn_net_workspace_bytes(ctypes.byref(c))
    assert 100e6 < ws < 4e9
    s = _cfg(kind=0, emax=0, n_layers=20, d=2)
    assert lib.hgnn_net_param_count(ctypes.byref(s)) == 6 * 19 + 2
    assert lib.hgnn_net_workspace_bytes(ctypes.byref(s)) > 0
    for bad in (dict(j_tot=9), dict(n_layers=1), dict(order=4), dict(bs=0), dict(d=300)):
        assert lib.hgnn_net_workspace_bytes(ctypes.byref(_cfg(**bad))) == 0
        assert lib.hgnn_net_param_count(ctypes.byref(_cfg(**bad))) == -1


def test_expected_k_matches_reference_shapes():
    from hgnn_amd.net import expected_k
    from models.gnns.model_mnb import GNN_lg, GNN_simple
    for order in (1, 2, 3):
        m = GNN_lg(0, 16, 4, 5, 1, 1, order)
        ks, kl = expected_k(1, order, 5, 16, 4, 3)
        for l, (kn, ke) in enumerate(ks):
            layer = m._layers()[l]
            assert layer.cv1.weight.shape == (16, kn, 1)
            assert layer.cv3.weight.shape == (16, ke, 1)
        assert m.layerlast.fc.weight.shape == (1, kl, 1)
    m = GNN_simple(0, 2, 5, 5, 1, 1)
    ks, kl = expected_k(0, 0, 5, 2, 5, 3)
    assert m.layer0.cv1.weight.shape == (2, ks[0][0], 1)
    assert m.layerlast.fc.weight.shape == (1, kl, 1)


def test_state_dict_matches_reference_layout(golden):
    """Same parameter names and shapes as the reference (fixture grads are keyed by them)."""
    from models.gnns.model_mnb import GNN_lg
    z = golden("lg_d64_o2")
    m = GNN_lg(0, 64, 5, 5, 1, 1, 2)
    names = {k[5:]: z[k].shape for k in z.files if k.startswith("grad.")}
    sd = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert sd == {k: tuple(v) for k, v in names.items()}


def test_gpu_ops_refuse_cpu_tensors():
    from models.gnns.model_mnb import GNN_lg
    from functions.operators import graph_operators
    from functions.batching import prepare_batch
    import hgnn_amd.datagen as dg
    graphs = dg.qm9_shape_dataset(4, seed=5)
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = prepare_batch(data, 0, 1)
    m = GNN_lg(0, 8, 3, 5, 1, 1, 2)
    with pytest.raises(RuntimeError, match="GPU"):
        m([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)


def test_compnet_utils_1d_surface_matches_reference(golden):
    """CompnetUtils (functions/utils_ccn.py drop-in) reproduces the reference's 1-D pipeline and chi matrices."""
    import fixture_util as fu
    from functions.utils_ccn import CompnetUtils
    from test_oracle import ccn_graphs, ccn_params
    z = golden("ccn")
    for k, (X, adj, _) in enumerate(ccn_graphs(z)):
        net, _ = ccn_params("1d", k)
        u = CompnetUtils(False)
        F = [u.get_F0_1D(X, adj)]
        for l in range(2):
            F.append(u.update_F_1D(F[-1], net._modules[f"w{l + 1}"]))
        out = net.fc(torch.cat([sum(v.sum(0) for v in f) for f in F], 0))
        assert torch.allclose(out.detach(), torch.from_numpy(z[f"1d_out_{k}"]), rtol=1e-5, atol=1e-5), k
        pos = []
        for i in range(adj.shape[0]):
            for j in range(adj.shape[0]):
                if adj[i, j] > 0:
                    chi = u.chis[i][j]
                    pos += [int(r.nonzero()[0]) if r.any() else -1 for r in chi]
        assert np.array_equal(np.array(pos), z[f"pos_{k}"]), k
        assert fu is not None


def test_ccn_state_dict_layout():
    from models.compnets.model_ccn import CCN_1D, CCN_2D
    s1 = {k: tuple(v.shape) for k, v in CCN_1D(5, 1, 2, 2).state_dict().items()}
    s2 = {k: tuple(v.shape) for k, v in CCN_2D(5, 1, 2, 2).state_dict().items()}
    assert s1 == {"w1.weight": (2, 10), "w1.bias": (2,), "w2.weight": (2, 4), "w2.bias": (2,),
                  "fc.weight": (1, 9), "fc.bias": (1,)}
    assert s2 == {"w1.weight": (2, 90), "w1.bias": (2,), "w2.weight": (2, 36), "w2.bias": (2,),
                  "fc.weight": (1, 9), "fc.bias": (1,)}
    assert CCN_2D(5, 1, 3, 2).hidden_size == 2


def test_ccn_cpu_tensors_raise():
    from models.compnets.model_ccn import CCN_1D
    net = CCN_1D(5, 1, 2, 2)
    with pytest.raises(RuntimeError, match="GPU only"):
        net(torch.zeros(3, 5), torch.eye(3))


def test_small_ccn_validation_word_reported_and_cleared():
    """Host side of the small-graph CCN validation word (hgnn_amd.ccn._HostWord): a nonzero word raises
    once with its bits and is cleared by the check; the same word stored again (a HIP-graph replay
    keeps its captured tag) raises again; clean checks do not raise; per-device words are independent."""
    import ctypes

    import hgnn_amd.ccn as HC
    w = HC._HostWord()
    word, word1 = ctypes.c_int32(0), ctypes.c_int32(0)
    w.words = {0: (word, None), 1: (word1, None)}
    w.check(False)
    word.value = (5 << 8) | 0x20
    with pytest.raises(RuntimeError, match="not symmetric"):
        w.check(False)
    assert word.value == 0
    w.check(False)                  # reported and cleared
    word.value = (5 << 8) | 0x20    # a replay of the same captured call fails again
    with pytest.raises(RuntimeError, match="not symmetric"):
        w.check(False)
    word1.value = (2 << 8) | 0x8    # the other device's word
    with pytest.raises(RuntimeError, match="self loop"):
        w.check(False)
    w.check(False)


def test_spec_params_and_checked_params_cache():
    """The executor's parameter list (read through the modules' dicts) is the modules' parameters in ABI
    order, the same objects attribute access gives; the cached parameter check re-checks a replaced
    parameter and raises on a wrong shape."""
    import hgnn_amd.net as N
    from models.gnns.model_mnb import GNN_lg, GNN_simple
    m = GNN_lg(0, 16, 4, 5, 1, 1, 2)
    dev = torch.device("cpu")
    spec = m._spec(dev)
    ref = []
    for layer in m._layers():
        for sub in ("cv1", "cv2", "bn1", "cv3", "cv4", "bn2"):
            mod = getattr(layer, sub)
            ref += [mod.weight, mod.bias]
    ref += [m.layerlast.fc.weight, m.layerlast.fc.bias]
    assert len(spec.params) == len(ref) and all(a is b for a, b in zip(spec.params, ref))
    assert len(GNN_simple(0, 2, 5, 5, 1, 1)._spec(dev).params) == 4 * 6 + 2  # layer0 + 3 mid layers, fc
    first = N._checked_params(spec, 5, 3, dev)
    again = N._checked_params(m._spec(dev), 5, 3, dev)
    assert again is first  # same objects at the same addresses: the cached list
    m.layer0.cv1.weight = torch.nn.Parameter(torch.zeros(16, 3, 1))
    with pytest.raises(RuntimeError, match="conv weight"):
        N._checked_params(m._spec(dev), 5, 3, dev)


def test_roofline_trace_cross_check(tmp_path):
    """bench.py's frac_trace: the stamp-timed algorithmic rate rescaled to the committed kernel trace's launch
    time of the class (launch-weighted over its kernels), absent without a trace file."""
    import json
    from hgnn_amd import roofline as RF
    path = tmp_path / "kernel_trace.json"
    path.write_text(json.dumps({
        "k_gemm_bf3_tn_ring<4, false>": {"avg_us": 40.0, "launches_per_step": 6.0},
        "k_gemm_bf3_tn_ring<4, true>": {"avg_us": 20.0, "launches_per_step": 2.0},
        "k_agg_fwd_rpw<3, 2, 2, true, 2, 0>": {"avg_us": 16.0, "launches_per_step": 8.0},
    }))
    assert RF.trace_avg_us(RF.K_GEMM_DW, str(path)) == 35.0
    assert RF.trace_avg_us(RF.K_AGG_FWD, str(path)) == 16.0
    assert RF.trace_avg_us(RF.K_GEMM_DA, str(path)) is None
    assert RF.trace_avg_us(RF.K_GEMM_DW, str(tmp_path / "absent.json")) is None
    counts = dict(nodes=9530, edges=22750, nnz_w=40000, nnz_wl=90000, nnz_p=45500)  # batch_counts' layout
    e = RF.roofline_entry(RF.K_GEMM_DW, 8 * 30e-3, 8, counts, 2, 5, 64, 5, 1, trace_path=str(path))
    assert e["avg_launch_us"] == 30.0 and e["trace_avg_launch_us"] == 35.0
    assert abs(e["frac_trace"] - e["frac"] * 30.0 / 35.0) < 1e-3
    assert "frac_trace" not in RF.roofline_entry(RF.K_GEMM_DW, 8 * 30e-3, 8, counts, 2, 5, 64, 5, 1)
