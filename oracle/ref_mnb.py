"""ORACLE -- test infrastructure only.  Never imported by the product path.

CPU restatement, op for op, of the reference's batched message-passing path,
used (1) as the checker in tests/ and __graft_entry__.smoke(), and (2) as the
`cpu_baseline` leg of bench.py (kind "port": the reference's own Python cannot
travel to the GPU box).  It keeps the reference's dense padded tensors, its
per-graph / per-slice torch.mm loops with slice assignment into zero buffers,
torch Conv1d and its masked BN, so its cost profile is the reference's.

Pinned against the reference by tests/test_oracle.py on the golden fixtures
that tests/golden/make_golden.py generated from /root/reference
(bit-exact operators and batches; outputs/grads within fp32 round-off).

Reference line map (all under /root/reference):
  graph_operators        functions/operators.py:11-83
  prepare_batch          functions/batching.py:77-185
  graph_oper / P_multi   models/layers/layers_mnb.py:391-434
  BN / sb_normalization  models/layers/batch_normalization.py:23-108
  layer_simple / last    models/layers/layers_mnb.py:25-95
  layer_with_lg_{1,2,3}  models/layers/layers_mnb.py:157-358
  layer_last_lg          models/layers/layers_mnb.py:361-388
  GNN_simple / GNN_lg    models/gnns/model_mnb.py:19-129
"""

import torch
import torch.nn.functional as F


# --------------------------------------------------------------------------- operators
def graph_operators(graph, J=1, dual=False):
    """Loop restatement of functions/operators.py:11-83 (small graphs only: O(M^2) Python)."""
    V, A = graph
    N = V.shape[0]
    ops = torch.zeros(N, N, J + 2)
    ops[:, :, 0] = torch.eye(N)
    d = torch.sum(A, dim=1)
    ops[:, :, 1] = torch.diag(d.squeeze())
    ops[:, :, 2].copy_(A)
    C = A.clone()
    for j in range(1, J):
        C = torch.matmul(C, C)
        ops[:, :, j + 2].copy_(C)
    if not dual:
        return ops
    M = A.nonzero().shape[0]
    lg = torch.zeros(M, M, J + 2)
    lg[:, :, 0] = torch.eye(M)
    AL = torch.zeros(M, M)
    Pm = torch.zeros(N, M)
    Pd = torch.zeros(N, M)
    edges = torch.zeros(M, 3)
    e = 0
    for i in range(N):
        for j in range(i + 1, N):
            if A[i, j] != 0:
                Pm[i, e] = 1
                Pm[j, e] = 1
                Pd[i, e] = 1
                Pd[j, e] = -1
                edges[e, 0] = i
                edges[e, 1] = j
                edges[e, 2] = A[i, j]
                e = e + 1          # once per bond ...
                Pm[i, e] = 1       # ... but the reverse slot is written at the new e too (Q1)
                Pm[j, e] = 1
                Pd[i, e] = -1
                Pd[j, e] = 1
                edges[e, 0] = j
                edges[e, 1] = i
                edges[e, 2] = A[i, j]
    for m1 in range(M):
        for m2 in range(M):
            if edges[m1, 1] == edges[m2, 0] and edges[m1, 0] != edges[m2, 1]:
                AL[m1, m2] = edges[m2, 2]
    dl = torch.sum(AL, dim=1)
    lg[:, :, 1] = torch.diag(dl)
    lg[:, :, 2].copy_(AL)
    CL = AL.clone()
    for j in range(1, J):
        CL = torch.matmul(CL, CL)
        lg[:, :, j + 2].copy_(CL)
    return ops, lg, Pm, Pd


def prepare_batch(batch, task, J=1):
    """Restatement of functions/batching.py:77-185 (cat-based padding, as the reference)."""
    bs = len(batch)
    nf = batch[0][0].shape[1]
    N_batch = torch.zeros(bs, dtype=torch.int64)
    E_batch = torch.zeros(bs, dtype=torch.int64)
    for i in range(bs):
        N_batch[i] = batch[i][0].shape[0]
        E_batch[i] = batch[i][1].nonzero().shape[0]
    Nmax = int(torch.max(N_batch).item())
    Emax = int(torch.max(E_batch).item())
    mask = torch.zeros(bs, Nmax, Nmax)
    mask_lg = torch.zeros(bs, Emax, Emax)
    X = torch.zeros(bs, nf, Nmax)
    W = torch.zeros(bs, Nmax, Nmax, J + 2)
    T = torch.zeros(bs, 1)
    XL = torch.zeros(bs, 1, Emax)
    WL = torch.zeros(bs, Emax, Emax, J + 2)
    Pm = torch.zeros(bs, Nmax, Emax)
    Pd = torch.zeros(bs, Nmax, Emax)
    for i in range(bs):
        x, A, t, w, wl, pm, pd = batch[i]
        n, e = int(N_batch[i]), int(E_batch[i])
        pn, pe = Nmax - n, Emax - e
        if pn > 0:
            x = torch.cat((x, torch.zeros(pn, nf)), 0)
            w = torch.cat((torch.cat((w, torch.zeros(n, pn, J + 2)), 1), torch.zeros(pn, Nmax, J + 2)), 0)
            pm = torch.cat((pm, torch.zeros(pn, e)), 0)
            pd = torch.cat((pd, torch.zeros(pn, e)), 0)
        if pe > 0:
            wl = torch.cat((torch.cat((wl, torch.zeros(e, pe, J + 2)), 1), torch.zeros(pe, Emax, J + 2)), 0)
            pm = torch.cat((pm, torch.zeros(Nmax, pe)), 1)
            pd = torch.cat((pd, torch.zeros(Nmax, pe)), 1)
        X[i].copy_(x.transpose(1, 0))
        T[i, 0] = t[task]
        XL[i].copy_(torch.diag(wl[:, :, 1]))
        W[i].copy_(w)
        WL[i].copy_(wl)
        Pm[i].copy_(pm)
        Pd[i].copy_(pd)
        mask[i, :n, :n] = 1
        mask_lg[i, :e, :e] = 1
    return X, W, T, XL, WL, Pm, Pd, mask, mask_lg, N_batch, E_batch


# --------------------------------------------------------------------------- ops
def graph_oper(A, X):
    bs, N, _, J = A.shape
    nf = X.shape[1]
    out = torch.zeros(bs, J * nf, N, dtype=X.dtype)
    for b in range(bs):
        for j in range(J):
            out[b, nf * j:nf * (j + 1), :] = torch.mm(A[b, :, :, j], X[b].transpose(1, 0)).transpose(1, 0)
    return out


def p_multi(P, X):
    bs, N = P.shape[0], P.shape[1]
    out = torch.zeros(bs, X.shape[1], N, dtype=X.dtype)
    for b in range(bs):
        out[b] = torch.mm(P[b], X[b].transpose(1, 0)).transpose(1, 0)
    return out


def graph_oper_fast(A, X):
    """graph_oper as one batched contraction (same sums, other fp order); the fast oracle leg that
    keeps the full-size parity tests cheap.  tests/test_oracle.py pins it to graph_oper."""
    bs, N, _, J = A.shape
    return torch.einsum("bnmj,bfm->bjfn", A, X).reshape(bs, J * X.shape[1], N)


def p_multi_fast(P, X):
    """p_multi as one bmm (see graph_oper_fast)."""
    return torch.bmm(X, P.transpose(1, 2))


def _ops(fast):
    return (graph_oper_fast, p_multi_fast) if fast else (graph_oper, p_multi)


def mask_embedding(H, mask):
    bs, N = mask.shape[0], mask.shape[1]
    return H * mask[:, :, 0].view(bs, 1, N).repeat(1, H.shape[1], 1)


def mean_with_padding(t, N_batch, mask):
    t = mask_embedding(t, mask)
    return torch.sum(torch.sum(t, dim=2), dim=0) / torch.sum(N_batch).item()


def bn(X, N_batch, mask, w, b, state, training, momentum=0.1):
    """BN.forward; `state` = dict with running_mean / running_std (updated in training)."""
    H = mask_embedding(X, mask)
    if training:
        mean = mean_with_padding(H, N_batch, mask)
        var = 10 ** -5 + mean_with_padding((H.transpose(2, 1) - mean).transpose(2, 1) ** 2, N_batch, mask)
        std = var ** 0.5
        state["running_mean"] = (1 - momentum) * mean.detach() + momentum * state["running_mean"]
        state["running_std"] = (1 - momentum) * std.detach() + momentum * state["running_std"]
    else:
        mean, std = state["running_mean"], state["running_std"]
    H = ((H.transpose(2, 1) - mean) / std).transpose(2, 1)
    return w * H + b


def conv(x, p, name):
    return F.conv1d(x, p[name + ".weight"], p[name + ".bias"])


# --------------------------------------------------------------------------- models
def _lg_node(p, pre, X, XL_like, W, Pm, Pd, N_batch, mask, st, training, fast=False):
    go, pm = _ops(fast)
    x1 = torch.cat((go(W, X), pm(Pm, XL_like), pm(Pd, XL_like)), 1)
    zb = torch.cat((conv(x1, p, pre + "cv2"), F.relu(conv(x1, p, pre + "cv1"))), 1)
    return bn(zb, N_batch, mask, p[pre + "bn1.weight"], p[pre + "bn1.bias"], st[pre + "bn1"], training)


def _lg_edge(p, pre, XL, X_like, WL, Pm, Pd, E_batch, mask_lg, st, training, fast=False):
    go, pm = _ops(fast)
    xd = torch.cat((go(WL, XL), pm(Pm.transpose(2, 1), X_like), pm(Pd.transpose(2, 1), X_like)), 1)
    zd = torch.cat((conv(xd, p, pre + "cv4"), F.relu(conv(xd, p, pre + "cv3"))), 1)
    return bn(zd, E_batch, mask_lg, p[pre + "bn2.weight"], p[pre + "bn2.bias"], st[pre + "bn2"], training)


def bn_states(n_layers, c, kind="lg", dtype=torch.float32):
    st = {}
    for l in range(n_layers - 1):
        for nm in (("bn1", "bn2") if kind == "lg" else ("bn1",)):
            st[f"layer{l}.{nm}"] = {"running_mean": torch.zeros(c, dtype=dtype), "running_std": torch.zeros(c, dtype=dtype)}
    return st


def gnn_lg(p, state, N_batch, mask, E_batch, mask_lg, n_layers, order, st, training=True, fast=False):
    """GNN_lg.forward (model_mnb.py:124-129, order switch 102-119) on a parameter dict with
    state_dict names.  fast=True: batched contractions instead of the per-graph loops."""
    X, XL, W, WL, Pm, Pd = state
    for l in range(n_layers - 1):
        pre = f"layer{l}."
        if order == 1:
            Z = _lg_node(p, pre, X, XL, W, Pm, Pd, N_batch, mask, st, training, fast)
            ZL = _lg_edge(p, pre, XL, Z, WL, Pm, Pd, E_batch, mask_lg, st, training, fast)
        elif order == 2:
            ZL = _lg_edge(p, pre, XL, X, WL, Pm, Pd, E_batch, mask_lg, st, training, fast)
            Z = _lg_node(p, pre, X, ZL, W, Pm, Pd, N_batch, mask, st, training, fast)
        else:
            Z = _lg_node(p, pre, X, XL, W, Pm, Pd, N_batch, mask, st, training, fast)
            ZL = _lg_edge(p, pre, XL, X, WL, Pm, Pd, E_batch, mask_lg, st, training, fast)
        X, XL = Z, ZL
    go, pm = _ops(fast)
    x1 = torch.cat((go(W, X), pm(Pm, XL), pm(Pd, XL)), 1)
    y = torch.sum(conv(x1, p, "layerlast.fc"), dim=2)
    return y.view(y.shape[0], -1)


def gnn_simple(p, state, N_batch, mask, n_layers, st, training=True, fast=False):
    """GNN_simple.forward (model_mnb.py:58-66)."""
    X, W = state
    go, _ = _ops(fast)
    for l in range(n_layers - 1):
        pre = f"layer{l}."
        x1 = go(W, X)
        zb = torch.cat((F.relu(conv(x1, p, pre + "cv2")), F.relu(conv(x1, p, pre + "cv1"))), 1)
        X = bn(zb, N_batch, mask, p[pre + "bn1.weight"], p[pre + "bn1.bias"], st[pre + "bn1"], training)
    y = torch.sum(conv(go(W, X), p, "layerlast.fc"), dim=2)
    return y.view(y.shape[0], -1)
