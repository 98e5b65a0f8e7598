"""World-size-2 data-parallel gradient all-reduce over gloo (CPU).

Each rank computes the oracle's gradients for its own shard of graphs (the
model math is the reference's, oracle/ref_mnb.py), the shared GradAllReduce
(hgnn_amd/dp.py, the exact code bench.py runs over RCCL) averages them, and
rank 0 checks the result against the average of both shards' gradients
computed in one process: "2 reference batches, gradients averaged"
(SURVEY.md §8 e semantics caveat).
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_grads(rank, d=8, L=3):
    import sys
    for p in (REPO, os.path.join(REPO, "hgnn-2_amd"), os.path.join(REPO, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import fixture_util as fu
    import hgnn_amd.datagen as dg
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    from models.gnns.model_mnb import GNN_lg
    from oracle import ref_mnb as R
    graphs = dg.qm9_shape_dataset(6, seed=500 + rank)
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = prepare_batch(data, 0, 1)
    m = GNN_lg(0, d, L, 5, 1, 1, 2)
    fu.det_init(m, 42)
    p = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    st = R.bn_states(L, 2 * d)
    out = R.gnn_lg(p, [X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg, L, 2, st, True)
    torch.nn.MSELoss()(out, T).backward()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(REPO, "hgnn-2_amd"))
    from hgnn_amd.dp import GradAllReduce
    p = _shard_grads(rank)
    params = [p[k] for k in sorted(p)]
    GradAllReduce(params)()
    if rank == 0:  # numpy copies: pickled by value, no shared-memory handle outliving the worker
        q.put({k: p[k].grad.detach().numpy().copy() for k in sorted(p)})
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_grad_allreduce_matches_shard_average():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    g0 = _shard_grads(0)
    g1 = _shard_grads(1)
    for k, v in got.items():
        v = torch.from_numpy(v)
        ref = (g0[k].grad + g1[k].grad) / 2
        assert torch.allclose(v, ref, rtol=1e-6, atol=1e-7), k


def test_shard_graphs_balanced_partition():
    """Σ(N+M)-balanced LPT sharding: a partition, loads within one graph's cost of each other."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "hgnn-2_amd"))
    import hgnn_amd.datagen as dg
    from hgnn_amd.dp import graph_cost, shard_graphs
    graphs = dg.qm9_shape_dataset(4096, seed=3)
    costs = [graph_cost(X, A) for X, A, _ in graphs]
    for world in (1, 2, 4, 8):
        sh = shard_graphs(costs, world)
        assert sorted(i for s in sh for i in s) == list(range(len(costs)))
        assert all(s == sorted(s) for s in sh)
        loads = [sum(costs[i] for i in s) for s in sh]
        assert max(loads) - min(loads) <= max(costs)
        counts = [len(s) for s in sh]
        assert max(counts) - min(counts) <= max(1, len(costs) // (world * 20)), counts
    assert shard_graphs([3, 1, 2], 2) == [[0], [1, 2]]


def _bucket_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(REPO, "hgnn-2_amd"))
    from hgnn_amd.dp import LayerBucketAllReduce, running_stats
    from models.gnns.model_mnb import GNN_lg
    torch.manual_seed(0)
    m = GNN_lg(0, 8, 3, 5, 1, 1, 2)
    ar = LayerBucketAllReduce(m)
    g = torch.Generator().manual_seed(100 + rank)
    for p in m.parameters():
        p.grad = torch.randn(p.shape, generator=g)
    for t in running_stats(m):
        t.copy_(torch.randn(t.shape, generator=g))
    ar.grad_targets()  # p.grad present: the one-collective (fresh) path, as after accumulated backwards
    ar()
    if rank == 0:
        q.put(({k: p.grad.numpy().copy() for k, p in m.named_parameters()},
               [t.numpy().copy() for t in running_stats(m)], ar.buckets[-1], ar.n_grad, ar.n_run))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world3_layer_buckets_carry_running_stats():
    """LayerBucketAllReduce's CPU path (the fresh-gradient form, one collective): gradients and the BN
    running statistics -- carried in the tail of the last layer's bucket, no second collective --
    come out as the average over three ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    grads, run, last_bucket, n_grad, n_run = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    import sys
    sys.path.insert(0, os.path.join(REPO, "hgnn-2_amd"))
    from hgnn_amd.dp import running_stats
    from models.gnns.model_mnb import GNN_lg
    torch.manual_seed(0)
    m = GNN_lg(0, 8, 3, 5, 1, 1, 2)
    names = [k for k, _ in m.named_parameters()]
    want_g = {k: torch.zeros(p.shape) for k, p in m.named_parameters()}
    want_r = [torch.zeros(t.shape) for t in running_stats(m)]
    for r in range(world):
        g = torch.Generator().manual_seed(100 + r)
        for k in names:
            want_g[k] += torch.randn(want_g[k].shape, generator=g) / world
        for w in want_r:
            w += torch.randn(w.shape, generator=g) / world
    for k in names:
        assert torch.allclose(torch.from_numpy(grads[k]), want_g[k], rtol=1e-6, atol=1e-7), k
    for got_t, w in zip(run, want_r):
        assert torch.allclose(torch.from_numpy(got_t), w, rtol=1e-6, atol=1e-7)
    off, n = last_bucket
    assert off + n == n_grad + n_run and n_run == sum(w.numel() for w in want_r)
