"""Helpers shared by the golden-fixture generator and the parity tests.

Test infrastructure only.  Nothing here imports the reference or the product;
the fixture script (run once, in the survey container) and the tests both use
the same deterministic weight assignment so the fixtures need not store
weights.
"""

import zlib

import numpy as np
import torch


def det_init(model, seed, scale=0.1):
    """Overwrite every parameter with N(0, scale^2) from a per-name generator.

    Independent of construction order and of the global RNG, so the reference
    model and the drop-in model receive bit-identical weights from a seed.
    """
    with torch.no_grad():
        for name, p in sorted(model.named_parameters()):
            g = torch.Generator().manual_seed((seed * 1000003 + zlib.crc32(name.encode())) % (2 ** 62))
            p.copy_(torch.randn(p.shape, generator=g, dtype=torch.float64).to(p.dtype) * scale)


def pack_graphs(graphs):
    """Flatten a list of (X, A, t) into a few arrays for an npz file."""
    ns = np.array([g[0].shape[0] for g in graphs], dtype=np.int64)
    X = np.concatenate([g[0].numpy().astype(np.float32).reshape(-1) for g in graphs])
    A = np.concatenate([g[1].numpy().astype(np.float32).reshape(-1) for g in graphs])
    t = np.stack([g[2].numpy().astype(np.float32) for g in graphs])
    f = graphs[0][0].shape[1]
    return {"g_n": ns, "g_X": X, "g_A": A, "g_t": t, "g_f": np.array(f)}


def unpack_graphs(z, prefix=""):
    ns = z[prefix + "g_n"]
    f = int(z[prefix + "g_f"])
    X = z[prefix + "g_X"]
    A = z[prefix + "g_A"]
    t = z[prefix + "g_t"]
    out = []
    xo = ao = 0
    for i, n in enumerate(ns):
        n = int(n)
        Xi = torch.from_numpy(X[xo:xo + n * f].reshape(n, f).copy())
        Ai = torch.from_numpy(A[ao:ao + n * n].reshape(n, n).copy())
        xo += n * f
        ao += n * n
        out.append((Xi, Ai, torch.from_numpy(t[i].copy())))
    return out


def chi_position_maps(adj):
    """Reference CCN receptive fields as int position maps.

    nbr_i = ascending nonzero(adj[i]) (`functions/utils_ccn.py:195-199`);
    p[i][a][x] = index of nbr_i[x] within nbr_{j_a}, or -1
    (`functions/utils_ccn.py:66-106`), j_a = a-th neighbour of i.
    Returns flat arrays (deg, nbr_flat, pos_flat) in a canonical order.
    """
    A = np.asarray(adj)
    n = A.shape[0]
    nbrs = [np.nonzero(A[i] > 0)[0] for i in range(n)]
    deg = np.array([len(v) for v in nbrs], dtype=np.int64)
    pos = []
    for i in range(n):
        for j in nbrs[i]:
            where = {int(v): k for k, v in enumerate(nbrs[j])}
            pos.extend(where.get(int(v), -1) for v in nbrs[i])
    return deg, np.concatenate(nbrs).astype(np.int64) if n else np.zeros(0, np.int64), np.array(pos, dtype=np.int64)
