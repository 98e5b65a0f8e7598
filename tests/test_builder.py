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
        for J in (1, 2):
            got = graph_operators([X, A], J, True)
            ref = R.graph_operators([X, A], J, True)
            for a, b in zip(got, ref):
                assert a.shape == b.shape and torch.equal(a, b)


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
