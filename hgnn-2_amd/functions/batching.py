"""Drop-in for functions/batching.py of the reference.

get_batches / _divide_batch / _get_unsorted_batches keep the reference's index
semantics (functions/batching.py:26-74).  prepare_batch (77-185) returns the
same 11 tensors bit for bit -- zero padding to the batch maxima Nmax / Emax,
XL = diag(WL[:, :, 1]) (the line-graph degree, Q4), masks with ones on the
real block, N_batch = nodes, E_batch = nnz(A) -- but writes each graph into
preallocated tensors by slicing instead of the reference's chain of
torch.cat + copy per graph.
"""

from random import shuffle

import numpy as np
import torch

from functions.operators import graph_operators  # noqa: F401  (reference import surface)

dtype = torch.FloatTensor
dtype_l = torch.LongTensor


def _divide_batch(nb_samples_in, batch_size, idx):
    """List of index lists, the last one possibly short (reference 26-40)."""
    if nb_samples_in % batch_size == 0:
        nb_batches = nb_samples_in // batch_size
    else:
        nb_batches = (nb_samples_in // batch_size) + 1
    idx_list = []
    for i in range(0, nb_batches):
        if i == nb_batches - 1:
            idx_list.append(idx[i * batch_size:])
        else:
            idx_list.append(idx[i * batch_size:(i + 1) * batch_size])
    return idx_list


def _get_unsorted_batches(nb_samples_in, batch_size, shuffle_batch=False):
    idx = list(range(nb_samples_in))
    if shuffle_batch:
        shuffle(idx)
    return _divide_batch(nb_samples_in, batch_size, idx)


def get_batches(nb_samples_in, batch_size, data, shuffle_batch=False, sort_batch=False):
    """Batch index lists; optionally grouped by graph size (reference 52-74)."""
    if not sort_batch:
        return _get_unsorted_batches(nb_samples_in, batch_size, shuffle_batch)
    sample_sizes = np.zeros(nb_samples_in)
    for i in range(len(data)):
        sample_sizes[i] = data[i][0].shape[0]
    sm_to_lg = np.argsort(sample_sizes)
    idx_list = _divide_batch(nb_samples_in, batch_size, sm_to_lg)
    if shuffle_batch:
        shuffle(idx_list)
    return idx_list


def prepare_batch(batch, task, J=1):
    """bs instances [x, A, t, W, WL, Pm, Pd] -> (X, W, T, XL, WL, Pm, Pd, mask, mask_lg, N_batch, E_batch).

    X (bs, f, Nmax), W (bs, Nmax, Nmax, J+2), T (bs, 1), XL (bs, 1, Emax),
    WL (bs, Emax, Emax, J+2), Pm / Pd (bs, Nmax, Emax), mask (bs, Nmax, Nmax),
    mask_lg (bs, Emax, Emax), N_batch / E_batch (bs,) int64.
    """
    bs = len(batch)
    n_features = batch[0][0].shape[1]
    N_batch = torch.zeros(bs, dtype=torch.int64)
    E_batch = torch.zeros(bs, dtype=torch.int64)
    for i in range(bs):
        N_batch[i] = batch[i][0].shape[0]
        E_batch[i] = int((batch[i][1] != 0).sum().item())
    Nmax = int(torch.max(N_batch).item())
    Emax = int(torch.max(E_batch).item())
    mask = torch.zeros(bs, Nmax, Nmax)
    mask_lg = torch.zeros(bs, Emax, Emax)
    X = torch.zeros(bs, n_features, Nmax)
    W = torch.zeros(bs, Nmax, Nmax, J + 2)
    T = torch.zeros(bs, 1)
    XL = torch.zeros(bs, 1, Emax)
    WL = torch.zeros(bs, Emax, Emax, J + 2)
    Pm = torch.zeros(bs, Nmax, Emax)
    Pd = torch.zeros(bs, Nmax, Emax)
    for i in range(bs):
        x, A, t, w, wl, pm, pd = batch[i]
        n = int(N_batch[i])
        e = int(E_batch[i])
        X[i, :, :n].copy_(x.transpose(1, 0))
        T[i, 0] = t[task]
        W[i, :n, :n, :].copy_(w)
        WL[i, :e, :e, :].copy_(wl)
        XL[i, 0, :e].copy_(torch.diagonal(wl[:, :, 1]))
        Pm[i, :n, :e].copy_(pm)
        Pd[i, :n, :e].copy_(pd)
        mask[i, :n, :n] = 1
        mask_lg[i, :e, :e] = 1
    return X, W, T, XL, WL, Pm, Pd, mask, mask_lg, N_batch, E_batch


def prepare_batch_csr(batch, task, J=1, device="cuda"):
    """Native sparse counterpart of prepare_batch for the executor (hgnn_amd.csr.CsrBatch):
    operators built from each instance's A by csrc/builder.cpp, no dense padding."""
    from hgnn_amd.csr import prepare_batch_csr as _p
    return _p(batch, task, J, device)
