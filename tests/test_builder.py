"""Native operator builder and sparse batcher (csrc/builder.cpp), on the CPU.

* hgnn_graph_operators (behind functions.operators.graph_operators) is pinned
  bit-exactly to the reference's fixtures in test_host.py; here it is also
  checked against the oracle's literal loop restatement on QM9-shape and SBM
  graphs, and timed against it.
* CsrBatch (hgnn_csr_batch_plan / _build) must hold exactly the row lists the
  device extraction (csrc/struct.hip k_extract) produces from the dense
  prepare_batch tensors: same rows, same ascending columns, same values, same
  packed X / XL / offsets -- emulated here in numpy on the dense batch.
"""

import time

import numpy as np
import pytest
import torch

from oracle import ref_mnb as R


def _graphs(n_qm9=12, n_sbm=2, seed=5):
    import hgnn_amd.datagen as dg
    gs = dg.qm9_shape_dataset(n_qm9, seed=seed) + dg.sbm_dataset(n_sbm, n=24, seed=seed)
    # edge cases: a self loop (an empty edge slot, Q2), an isolated node, a single node
    X, A, t = gs[0]
    A = A.clone()
    A[0, 0] = 1.0
    gs[0] = (X, A, t)
    X, A, t = gs[1]
    A = A.clone()
    A[-1, :] = 0
    A[:, -1] = 0
    gs[1] = (X, A, t)
    gs.append((torch.eye(1, 5), torch.zeros(1, 1), torch.randn(13)))
    return gs


def test_graph_operators_native_vs_loop_oracle():
    from functions.operators import graph_operators
    for X, A, _ in _graphs():
        if X.shape[0] == 1:
            continue  # the reference's torch.diag(d.squeeze()) raises on a 1-node graph
        for J in (1, 2, 3, 4, 5):
            got = graph_operators([X, A], J, True)
            ref = R.graph_operators([X, A], J, True)
            for a, b in zip(got, ref):
                assert a.shape == b.shape
                if J <= 3:
                    assert torch.equal(a, b), J
                else:  # A^8, A^16 of weighted adjacencies: the reference's fp32 matmul rounds per product
                    # and sum, the builder squares in fp64 and rounds once (parity within fp32, unpinned bits)
                    assert torch.allclose(a, b, rtol=2e-6, atol=0), J


def test_graph_operators_native_speed():
    """The reference's O(M^2) Python loop takes ~1.7 s per SBM-50 graph."""
    import hgnn_amd.datagen as dg
    from functions.operators import graph_operators
    X, A, _ = dg.sbm_dataset(1, n=50, seed=3)[0]
    t0 = time.perf_counter()
    for _ in range(5):
        graph_operators([X, A], 1, True)
    native = (time.perf_counter() - t0) / 5
    assert native < 0.05, native


def _extract(dense_rows, jt):
    """Emulation of k_extract on one dense (R, C, jt) block: per row, ascending nonzero columns."""
    out = []
    for r in range(dense_rows.shape[0]):
        nz = np.nonzero((dense_rows[r] != 0).any(axis=-1))[0]
        out.append([(int(c), dense_rows[r, c]) for c in nz])
    return out


def _check_kind(rows, ent, want, row0, col0, ncoef):
    for r, items in enumerate(want):
        start, count = rows[row0 + r]
        assert count == len(items), (r, count, len(items))
        for e, (c, v) in enumerate(items):
            q = ent[start + e]
            assert q[:1].view(np.int32)[0] == col0 + c
            assert np.array_equal(q[1:1 + ncoef], np.asarray(v, dtype=np.float32).reshape(-1)[:ncoef])


@pytest.mark.parametrize("J", [1, 2])
def test_csr_batch_equals_device_extraction_of_dense_batch(J):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    from hgnn_amd.csr import CsrBatch
    gs = _graphs()
    data = [[X, A, t, *graph_operators([X, A], J, True)] for X, A, t in gs]
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.numpy() for t in prepare_batch(data, 0, J)]
    b = CsrBatch([(X_, A_) for X_, A_, _ in gs], J=J, dual=True, device="cpu")
    lists = b.lists()
    jt = J + 2
    assert b.nodes == Nb.sum() and b.edges == Eb.sum() and b.nmax == W.shape[1] and b.emax == WL.shape[1]
    assert np.array_equal(b.N_batch.numpy(), Nb) and np.array_equal(b.E_batch.numpy(), Eb)
    n0 = e0 = 0
    xl = b._f32(b.layout.off_xl, b.edges).numpy()
    for g in range(len(gs)):
        n, e = int(Nb[g]), int(Eb[g])
        assert np.array_equal(b.x.numpy()[n0:n0 + n], X[g, :, :n].T)
        assert np.array_equal(xl[e0:e0 + e], XL[g, 0, :e])
        w = W[g, :n, :n]
        wl = WL[g, :e, :e]
        p = np.stack([Pm[g, :n, :e], Pd[g, :n, :e]], -1)
        _check_kind(*lists[0], _extract(w, jt), n0, n0, jt)
        _check_kind(*lists[1], _extract(w.transpose(1, 0, 2), jt), n0, n0, jt)
        _check_kind(*lists[2], _extract(wl, jt), e0, e0, jt)
        _check_kind(*lists[3], _extract(wl.transpose(1, 0, 2), jt), e0, e0, jt)
        _check_kind(*lists[4], _extract(p, 2), n0, e0, 2)
        _check_kind(*lists[5], _extract(p.transpose(1, 0, 2), 2), e0, n0, 2)
        n0 += n
        e0 += e


def test_csr_batch_is_smaller_than_dense():
    import hgnn_amd.datagen as dg
    from hgnn_amd.csr import CsrBatch
    gs = dg.qm9_shape_dataset(256, seed=0)
    b = CsrBatch([(X, A) for X, A, _ in gs], device="cpu")
    nmax, emax = b.nmax, b.emax
    dense = 4 * 256 * (nmax * nmax * 3 + emax * emax * 3 + 2 * nmax * emax + nmax * nmax + emax * emax + 5 * nmax + emax)
    assert b.layout.bytes * 4 < dense, (b.layout.bytes, dense)


def test_csr_batch_rejects_bad_input():
    from hgnn_amd.csr import CsrBatch
    with pytest.raises(RuntimeError):
        CsrBatch([(torch.zeros(3, 5), torch.zeros(2, 2))], device="cpu")


def _real_weight_graphs(seed=9):
    """Graphs whose A weights are not dyadic: interatomic-distance-like values (model_mnb.py:82 documents
    distances as the alternative edge feature) and real-valued SBM weights."""
    import hgnn_amd.datagen as dg
    g = torch.Generator().manual_seed(seed)
    out = []
    for X, A, t in dg.qm9_shape_dataset(6, seed=seed) + dg.sbm_dataset(2, n=24, seed=seed):
        W = torch.rand(A.shape, generator=g) * 1.3 + 0.7
        W = torch.triu(W, 1)
        W = W + W.T
        out.append((X, torch.where(A != 0, W, torch.zeros_like(W)), t))
    return out


def test_graph_operators_real_valued_weights_within_reference_rounding():
    """The bit-exact claim needs dyadic weights (bond orders 1, 1.5, 2, 3: every partial sum exact in
    fp32).  With real-valued weights the builder rounds each degree / A^2 entry once from an exact
    double sum, while the reference rounds torch.sum / torch.matmul partial sums in fp32: the two may
    differ by the reference's own rounding, |d| <= n * 2^-24 * sum|terms| (n = N terms per entry).
    Copies of A (the A slice, WL's weights, Pm / Pd) stay bit-exact."""
    # the rounding rule is actually exercised: some entries do differ (72 with this seed)
    assert _real_weight_check() > 0


def _real_weight_check():
    from functions.operators import graph_operators
    n_diff = 0
    for X, A, _ in _real_weight_graphs():
        N = A.shape[0]
        for J in (1, 2):
            got = graph_operators([X, A], J, True)
            ref = R.graph_operators([X, A], J, True)
            W, WL, Pm, Pd = got
            Wr, WLr, Pmr, Pdr = ref
            assert torch.equal(Pm, Pmr) and torch.equal(Pd, Pdr)
            assert torch.equal(W[:, :, :1], Wr[:, :, :1]) and torch.equal(W[:, :, 2], Wr[:, :, 2])
            assert torch.equal(WL[:, :, :1], WLr[:, :, :1])
            Aa = A.double().abs()
            bound = {1: torch.diag(Aa.sum(1)) * N * 2.0 ** -24}
            if J == 2:
                bound[3] = (Aa @ Aa) * N * 2.0 ** -24
            for j, b in bound.items():
                d = (W[:, :, j].double() - Wr[:, :, j].double()).abs()
                assert (d <= b).all(), (j, d.max().item())
                n_diff += int((d > 0).sum())
            # the line graph's slices: the same rule on its own weights
            M = WL.shape[0]
            ALa = WLr[:, :, 2].double().abs()
            assert torch.equal(WL[:, :, 2], WLr[:, :, 2])
            d = (WL[:, :, 1].double() - WLr[:, :, 1].double()).abs()
            assert (d <= torch.diag(ALa.sum(1)) * M * 2.0 ** -24).all()
            if J == 2:
                d = (WL[:, :, 3].double() - WLr[:, :, 3].double()).abs()
                assert (d <= (ALa @ ALa) * M * 2.0 ** -24).all()
    return n_diff


def test_high_j_operators_vs_reference_fixture():
    """J = 3, 4, 5 operators against the reference's own graph_operators output (tests/golden/operators_hij.npz,
    functions/operators.py:25-29, fp32 torch.matmul powers on the fixture machine's BLAS).  J = 3 (A^4) stays in
    fp32's exact range for these weights: bit-exact.  J >= 4 (A^8, A^16) leaves it, so the reference's bits depend
    on its BLAS's summation order; the builder rounds each power once from an fp64 accumulation (the correctly
    rounded square of its fp32 input).  Measured: J = 4 differs in 27 of 407 220 entries (26 by 1 ulp, one by 2);
    J = 5 (A^16, squared from the already rounded A^8) in 8 556 of 652 267, by 1-6 ulp.  The restated
    oracle (oracle/ref_mnb.py, torch.matmul like the reference) is bit-exact at every J."""
    import os

    import fixture_util as fu
    from functions.operators import graph_operators
    GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    z = np.load(os.path.join(GOLD, "operators_hij.npz"))
    for J, max_diff, max_ulp in ((3, 0, 0), (4, 64, 2), (5, 12000, 8)):
        gs = fu.unpack_graphs(z, f"J{J}.")
        nd = 0
        for k, (X, A, _t) in enumerate(gs):
            W, WL, _, _ = graph_operators([X, A], J, True)
            Wo, WLo, _, _ = R.graph_operators([X, A], J, True)
            for got, orc, key in ((W, Wo, f"J{J}.W_{k}"), (WL, WLo, f"J{J}.WL_{k}")):
                ref = torch.from_numpy(z[key])
                assert torch.equal(orc, ref), (J, key)
                d = got != ref
                nd += int(d.sum())
                if d.any():
                    ulps = (got[d].view(torch.int32).long() - ref[d].view(torch.int32).long()).abs()
                    assert int(ulps.max()) <= max_ulp, (J, key, int(ulps.max()))
        assert nd <= max_diff, (J, nd)
