"""ORACLE -- test infrastructure only.  Never imported by the product path.

CPU restatement of the reference's covariant compositional networks, one graph
at a time, with the reference's ragged per-node tensors and the literal d^5
tensor product T (x) chi_ii followed by the 18 contractions.  Autograd through
it gives the gradients the reference's loss.backward() produces.  Pinned by
tests/test_oracle.py against tests/golden/ccn.npz (generated from the
reference by tests/golden/make_golden.py).

Reference line map (all under /root/reference):
  receptive fields, chi      functions/utils_ccn.py:66-106, 148-222
  _promote / _promote_1D     functions/utils_ccn.py:225-252
  update_F / update_F_1D     functions/utils_ccn.py:281-324
  python_contract/tensorprod functions/utils_ccn.py:37-45, 57-63
  collapse6to3               functions/contraction.py:21-121
  CCN_1D / CCN_2D forward    models/compnets/model_ccn.py:41-64, 93-105
Closed / vectorised forms for the sizes the literal loops cannot reach: ccn2_forward_closed
(CCN-2D, SBM-200) and ccn1_forward_vec (CCN-1D, SBM-400..1000), each pinned to ccn_forward.
"""

import torch
import torch.nn.functional as Fn


def receptive_fields(adj):
    """deg_i = #(A[i] > 0), nbr_i ascending (utils_ccn.py:159-163)."""
    n = adj.shape[0]
    nbrs = [[j for j in range(n) if adj[i, j] > 0] for i in range(n)]
    return nbrs


def positions(nbrs, i, j):
    """p[x] = index of nbr_i[x] in nbr_j, -1 if absent (the nonzero of chi_ij row x, utils_ccn.py:78-82)."""
    where = {v: k for k, v in enumerate(nbrs[j])}
    return [where.get(v, -1) for v in nbrs[i]]


def collapse6to3(F):
    """F (C, n, n, n, n, n) -> (n, n, 18C); contraction.py:44-121 restated with einsum diagonals."""
    P = F.permute(1, 2, 3, 4, 5, 0)  # [a, b, c, d, e, ch] (contraction.py:114)
    qs = [
        torch.einsum("abcdeh->abh", P),   # fix a,b
        torch.einsum("abcdeh->adh", P),   # fix a,d
        torch.einsum("abcdeh->bch", P),   # fix b,c
        torch.einsum("abcdeh->bdh", P),   # fix b,d
        torch.einsum("abcdeh->deh", P),   # fix d,e
        torch.einsum("abcceh->abh", P),   # case 6: c == d, sum e
    ]
    qs += [torch.einsum("abcddh->abh", P)] * 9   # cases 7-15: identity permutation, d == e
    qs += [
        torch.einsum("abbdbh->adh", P),   # case 16: b == c == e
        torch.einsum("abadah->bdh", P),   # case 17: a == c == e
        torch.einsum("aaadeh->deh", P),   # case 18: a == b == c
    ]
    return torch.cat(qs, 2)


def _promote_1d(Fj, p):
    rows = [Fj[q] if q >= 0 else torch.zeros_like(Fj[0]) for q in p]
    return torch.stack(rows, 0)


def _promote_2d(Fj, p):
    d = len(p)
    out = torch.zeros(d, d, Fj.shape[2], dtype=Fj.dtype)
    for x in range(d):
        for y in range(d):
            if p[x] >= 0 and p[y] >= 0:
                out[x, y] = Fj[p[x], p[y]]
    return out


def _linear(p, name, x):
    return x @ p[name + ".weight"].t() + p[name + ".bias"]


def ccn_forward(p, X, adj, order, layers):
    """CCN_1D (order 1) / CCN_2D (order 2) forward for one graph; p = state-dict-like params."""
    n = X.shape[0]
    nbrs = receptive_fields(adj)
    if order == 1:
        F = [X[i].view(1, -1).expand(len(nbrs[i]), -1) for i in range(n)]
    else:
        F = [X[i].view(1, 1, -1).expand(len(nbrs[i]), len(nbrs[i]), -1) for i in range(n)]
    levels = [F]
    for l in range(layers):
        new = []
        for i in range(n):
            ps = [positions(nbrs, i, j) for j in nbrs[i]]
            if order == 1:
                T = torch.stack([_promote_1d(F[j], pj) for j, pj in zip(nbrs[i], ps)], 0)
                coll = torch.cat([T.sum(0), T.sum(1)], 1)
            else:
                T = torch.stack([_promote_2d(F[j], pj) for j, pj in zip(nbrs[i], ps)], 0)
                d = len(nbrs[i])
                eye = torch.eye(d, dtype=T.dtype)  # chi_ii
                H = T.permute(3, 0, 1, 2).unsqueeze(4).unsqueeze(5) * eye
                coll = collapse6to3(H)
            new.append(Fn.relu(_linear(p, "w{}".format(l + 1), coll)))
        F = new
        levels.append(F)
    if order == 1:
        summed = [sum(v.sum(0) for v in f) for f in levels]
    else:
        summed = [sum(v.sum(0).sum(0) for v in f) for f in levels]
    return _linear(p, "fc", torch.cat(summed, 0))


def ccn2_forward_closed(p, X, adj, layers):
    """CCN_2D forward for one graph with collapse6to3(T (x) chi_ii) in its O(n^3 C) closed form
    (utils_ccn.py:281-300, contraction.py:106-121): the same function as
    ccn_forward(..., order=2) without the d^5 intermediate, so it runs at SBM N = 200 (config 5),
    which the reference itself cannot (5.65 GB per node).  Pinned against ccn_forward on small
    graphs by tests/test_oracle.py; vectorised per node, any dtype (fp64 for parity)."""
    n_nodes = X.shape[0]
    nbrs = [torch.nonzero(adj[i] > 0).view(-1) for i in range(n_nodes)]
    deg = [len(v) for v in nbrs]
    idx = torch.full((n_nodes, n_nodes), -1, dtype=torch.long)  # idx[j, v] = position of v in nbr_j
    for j in range(n_nodes):
        idx[j, nbrs[j]] = torch.arange(deg[j])
    F = [X[i].view(1, 1, -1).expand(deg[i], deg[i], -1) for i in range(n_nodes)]
    levels = [F]
    dmax = max(deg) if deg else 0
    for l in range(layers):
        new = []
        # (nodes, dmax, dmax, C) zero-padded, autograd through it
        Fp = torch.stack([Fn.pad(f, (0, 0, 0, dmax - f.shape[1], 0, dmax - f.shape[0])) for f in F], 0)
        for i in range(n_nodes):
            n = deg[i]
            J = nbrs[i]
            P = idx[J][:, J]                              # P[a][x] = position of nbr_i[x] in nbr_{j_a}
            q = P.clamp(min=0)
            valid = (P >= 0).to(X.dtype)
            # T[a][b][c] = F_{j_a}[p_a(b)][p_a(c)], 0 where either position is absent
            T = Fp[J.view(-1, 1, 1), q.unsqueeze(2), q.unsqueeze(1)] * (valid.unsqueeze(2) * valid.unsqueeze(1)).unsqueeze(-1)
            Sc = T.sum(2)                                 # [a][b]
            Sa = T.sum(0)                                 # [b][c]
            q1 = Sc.sum(1)                                # [a]
            q3 = Sa.sum(1)                                # [b]
            tot = Sc.sum((0, 1))
            ar = torch.arange(n)
            d3 = T[ar, ar, ar].sum(0)
            eye = torch.eye(n, dtype=T.dtype).unsqueeze(-1)
            nf = float(n)
            blocks = [nf * Sc, q1.view(n, 1, -1).expand(n, n, -1), nf * Sa, q3.view(n, 1, -1).expand(n, n, -1),
                      eye * tot, Sc]
            blocks += [nf * Sc] * 9
            blocks += [T[:, ar, ar],                      # q15[x][y] = T[x][y][y]
                       T[ar, :, ar].transpose(0, 1),      # q16[x][y] = T[y][x][y]
                       eye * d3]
            coll = torch.cat(blocks, 2)                   # (n, n, 18 C), channel q * C + ch
            new.append(Fn.relu(_linear(p, "w{}".format(l + 1), coll)))
        F = new
        levels.append(F)
    summed = [sum(v.sum(0).sum(0) for v in f) for f in levels]
    return _linear(p, "fc", torch.cat(summed, 0))


def ccn1_forward_vec(p, X, adj, layers):
    """CCN_1D forward for one graph, vectorised per node: the same function as
    ccn_forward(..., order=1) (utils_ccn.py:185-222, 242-252, 303-324) with the chi position maps
    from one dense index table instead of per-pair Python dicts, so it runs on SBM graphs of
    N = 400-1000 (degrees ~70-200).  Pinned against ccn_forward by tests/test_oracle.py."""
    n_nodes = X.shape[0]
    nbrs = [torch.nonzero(adj[i] > 0).view(-1) for i in range(n_nodes)]
    deg = [len(v) for v in nbrs]
    idx = torch.full((n_nodes, n_nodes), -1, dtype=torch.long)  # idx[j, v] = position of v in nbr_j
    for j in range(n_nodes):
        idx[j, nbrs[j]] = torch.arange(deg[j])
    F = [X[i].view(1, -1).expand(deg[i], -1) for i in range(n_nodes)]
    levels = [F]
    for l in range(layers):
        new = []
        Fp = torch.nn.utils.rnn.pad_sequence(F, batch_first=True)  # (nodes, dmax, C), autograd through it
        for i in range(n_nodes):
            J = nbrs[i]
            P = idx[J][:, J]                                   # P[a][x] = position of nbr_i[x] in nbr_{j_a}
            T = Fp[J.view(-1, 1), P.clamp(min=0)] * (P >= 0).to(X.dtype).unsqueeze(2)   # (d, d, C): T[a][x]
            coll = torch.cat([T.sum(0), T.sum(1)], 1)
            new.append(Fn.relu(_linear(p, "w{}".format(l + 1), coll)))
        F = new
        levels.append(F)
    summed = [sum(v.sum(0) for v in f) for f in levels]
    return _linear(p, "fc", torch.cat(summed, 0))
