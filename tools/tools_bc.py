"""Small helpers shared by the diagnostic tools."""
import torch


def ccn_pad(graphs):
    bs = len(graphs)
    nmax = max(X.shape[0] for X, _, _ in graphs)
    f = graphs[0][0].shape[1]
    X = torch.zeros(bs, nmax, f)
    A = torch.zeros(bs, nmax, nmax)
    nb = torch.zeros(bs, dtype=torch.int64)
    for b, (x, a, _) in enumerate(graphs):
        n = x.shape[0]
        X[b, :n] = x
        A[b, :n, :n] = a + torch.eye(n)
        nb[b] = n
    return X.cuda(), A.cuda(), nb.cuda()
