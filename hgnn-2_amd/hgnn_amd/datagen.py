"""Seeded synthetic graph generators for the benchmark configurations.

The reference ships no SBM generator and its QM9 pipeline needs rdkit
(SURVEY.md §2, §8 d), so the build defines both generators here, with the
statistics SURVEY.md §8 d fixes:

* QM9-shape: N ~ U{9..29}, a random recursive tree with bond orders drawn from
  {1, 1, 1, 1.5, 2, 3}, round(0.25 N) extra unit bonds, one-hot atom type over 5
  types, 13 regression targets (task 0 is used).
* SBM: two equal blocks (z = i mod 2), p_in / p_out, symmetric, no self loops,
  one-hot(min(deg, 4)) node features (5 features).

Each generator returns a list of ``(X (N, f), A (N, N), t (13,))`` float32
tensors -- the first three members of the reference's 7-tuple instances
(`functions/data_generator.py:85`, `preprocessing/preprocessing.py:95-97`).
The operator members are produced by ``functions.operators.graph_operators``.

This module imports nothing but torch/random so the golden-fixture script can
load it next to the reference without a package-name clash.
"""

import random

import torch

BOND_ORDERS = (1.0, 1.0, 1.0, 1.5, 2.0, 3.0)


def qm9_shape_graph(rng, gen, n_types=5, n_targets=13, n_min=9, n_max=29):
    """One QM9-shaped molecule graph (SURVEY.md §8 d, 'QM9-shape generator')."""
    n = rng.randint(n_min, n_max)
    A = torch.zeros(n, n)
    for v in range(1, n):
        p = rng.randrange(v)
        w = rng.choice(BOND_ORDERS)
        A[p, v] = w
        A[v, p] = w
    extra = int(round(0.25 * n))
    added = 0
    tries = 0
    while added < extra and tries < 100:
        tries += 1
        i = rng.randrange(n)
        j = rng.randrange(n)
        if i == j or A[i, j] != 0:
            continue
        A[i, j] = 1.0
        A[j, i] = 1.0
        added += 1
    X = torch.zeros(n, n_types)
    for v in range(n):
        X[v, rng.randrange(n_types)] = 1.0
    t = torch.randn(n_targets, generator=gen)
    return X, A, t


def qm9_shape_dataset(n_graphs, seed=0, **kw):
    rng = random.Random(seed)
    gen = torch.Generator().manual_seed(seed)
    return [qm9_shape_graph(rng, gen, **kw) for _ in range(n_graphs)]


def sbm_graph(gen, n=50, p_in=0.3, p_out=0.05, n_feat=5, n_targets=13):
    """Two-block stochastic block model graph (SURVEY.md §8 d, 'SBM generator')."""
    z = torch.arange(n) % 2
    same = z.view(-1, 1) == z.view(1, -1)
    prob = torch.where(same, torch.tensor(p_in), torch.tensor(p_out))
    u = torch.rand(n, n, generator=gen) < prob
    upper = torch.triu(u, diagonal=1).float()
    A = upper + upper.t()
    deg = A.sum(dim=1).long()
    X = torch.zeros(n, n_feat)
    X[torch.arange(n), torch.clamp(deg, max=n_feat - 1)] = 1.0
    t = torch.randn(n_targets, generator=gen)
    return X, A, t


def sbm_dataset(n_graphs, n=50, seed=0, **kw):
    gen = torch.Generator().manual_seed(seed)
    return [sbm_graph(gen, n=n, **kw) for _ in range(n_graphs)]
