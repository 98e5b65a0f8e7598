"""World-size-2 and -8 data parallelism with the real HIP executor (SURVEY.md §8 e).

Two (or eight: config 4's 4096-graph global batch) ranks (gloo on GPU tensors, all on cuda:0) take Σ(N+M)-balanced shards of one global batch
(hgnn_amd.dp.shard_graphs), run GNN_lg forward + backward through the executor with the per-layer
bucketed all-reduce (hgnn_amd.dp.LayerBucketAllReduce: the executor writes the gradients into the
flat buffer and records per-layer events that the communication stream waits on) and average
their BN running statistics (carried in the last layer's bucket).  Checked against the fp64 oracle run on each shard (oracle/ref_mnb.py):
"2 reference batches, gradients averaged" -- the semantics of gradient-only DP (the reference itself
has one batch: models/layers/batch_normalization.py:80-93).
"""

import os
import socket

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

D, L, ORDER, NG, WSEED = 16, 4, 2, 40, 71


def _paths():
    import sys
    for p in (REPO, os.path.join(REPO, "hgnn-2_amd"), os.path.join(REPO, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shards(world, ng=NG):
    _paths()
    import hgnn_amd.datagen as dg
    from hgnn_amd.dp import graph_cost, shard_graphs
    graphs = dg.qm9_shape_dataset(ng, seed=909)
    return graphs, shard_graphs([graph_cost(X, A) for X, A, _ in graphs], world)


def _batch(graphs):
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    return list(prepare_batch(data, 0, 1))


def _worker(rank, world, port, q, mode="none", shape=(D, L, NG, 2)):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HGNN_STRICT", "1")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _paths()
        import fixture_util as fu
        from hgnn_amd.dp import LayerBucketAllReduce, running_stats
        from models.gnns.model_mnb import GNN_lg
        d, nl, ng, steps = shape
        torch.cuda.set_device(0)
        graphs, shards = _shards(world, ng)
        b = [t.cuda() for t in _batch([graphs[i] for i in shards[rank]])]
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = b
        model = GNN_lg(0, d, nl, 5, 1, 1, ORDER).cuda()
        fu.det_init(model, WSEED)
        dp = LayerBucketAllReduce(model)
        for step in range(steps):  # twice: the flat buffer and the events are reused across steps
            if mode == "none":
                model.zero_grad(set_to_none=True)
            elif mode == "zero":
                model.zero_grad(set_to_none=False)  # p.grad kept (the flat buffer's views), zeroed
            elif step == 0:  # "accum": the second backward adds to the first step's averaged grads
                model.zero_grad(set_to_none=True)
            out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
            torch.nn.MSELoss()(out, T).backward()
            dp()
        torch.cuda.synchronize()
        res = {"grad." + k: p.grad.detach().cpu().numpy().copy() for k, p in model.named_parameters()}
        res["flat_is_grad"] = all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(dp.params, dp.views))
        res["running"] = [t.detach().cpu().numpy().copy() for t in running_stats(model)]
        q.put((rank, res))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _oracle_shard(graphs, idx, d=D, nl=L, steps=2):
    _paths()
    import fixture_util as fu
    from models.gnns.model_mnb import GNN_lg
    from oracle import ref_mnb as R
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = _batch([graphs[i] for i in idx])
    m = GNN_lg(0, d, nl, 5, 1, 1, ORDER)
    fu.det_init(m, WSEED)
    dt = torch.float64
    p = {k: v.detach().to(dt).requires_grad_(True) for k, v in m.state_dict().items()}
    st = R.bn_states(nl, 2 * d, dtype=dt)
    runs = []
    for _ in range(steps):  # the ranks ran `steps` steps: running stats advanced that often
        for v in p.values():
            v.grad = None
        out = R.gnn_lg(p, [X.to(dt), XL.to(dt), W.to(dt), WL.to(dt), Pm.to(dt), Pd.to(dt)], Nb, mask.to(dt), Eb,
                       mask_lg.to(dt), nl, ORDER, st, True, fast=True)
        torch.nn.MSELoss()(out, T.to(dt)).backward()
        runs.append({k: v.grad.clone() for k, v in p.items()})
    return runs[-1], st


@pytest.mark.parametrize("mode", ["none", "zero", "accum"])
def test_world2_bucketed_allreduce_matches_shard_average(mode):
    """mode: p.grad None before each backward (the overlapped per-layer buckets), zeroed but kept
    (zero_grad(set_to_none=False)) and accumulated over two backwards (expected: twice the
    average) -- the last two take the fresh-gradient path, one collective after the backward."""
    import multiprocessing as mp
    ctx = mp.get_context("forkserver")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=240) for _ in range(2))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    graphs, shards = _shards(2)
    # balanced shards: every graph in exactly one, loads within one graph's cost
    assert sorted(shards[0] + shards[1]) == list(range(NG))
    (g0, s0), (g1, s1) = _oracle_shard(graphs, shards[0]), _oracle_shard(graphs, shards[1])
    ref = {k: (g0[k] + g1[k]) / 2 * (2 if mode == "accum" else 1) for k in g0}
    gmax = max(v.abs().max().item() for v in ref.values())
    for r in (0, 1):
        res = got[r]
        assert res["flat_is_grad"]
        for k, v in ref.items():
            g = torch.from_numpy(res["grad." + k]).double()
            assert torch.all((g - v).abs() <= 1e-4 * gmax + 1e-5 * v.abs()), (r, k)
        # BN running statistics averaged across the ranks
        i = 0
        for l in range(L - 1):
            for nm in ("bn1", "bn2"):
                for key in ("running_mean", "running_std"):
                    want = ((s0[f"layer{l}.{nm}"][key] + s1[f"layer{l}.{nm}"][key]) / 2).numpy()
                    np.testing.assert_allclose(res["running"][i], want, rtol=1e-4, atol=1e-5)
                    i += 1
    # both ranks hold identical averaged gradients
    for k in ref:
        assert np.array_equal(got[0]["grad." + k], got[1]["grad." + k]), k


def _run_world(world, d, nl, ng, timeout=300):
    """Start `world` ranks of _worker on cuda:0 (one step, p.grad None), compute the fp64 oracle of every
    shard in this process while they run, then collect the ranks' gradients and running statistics."""
    import multiprocessing as mp
    ctx = mp.get_context("forkserver")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "none", (d, nl, ng, 1))) for r in range(world)]
    for pr in procs:
        pr.start()
    graphs, shards = _shards(world, ng)
    oracle = [_oracle_shard(graphs, shards[r], d, nl, 1) for r in range(world)]
    got = dict(q.get(timeout=timeout) for _ in range(world))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    return graphs, shards, oracle, got


def _check_world(world, nl, shards, oracle, got, ng):
    """Every rank's gradients against the fp64 oracle's shard average (SURVEY.md §8 c gradient bound),
    running statistics against the average of the shards' running statistics, all ranks identical."""
    assert sorted(i for s in shards for i in s) == list(range(ng))
    ref = {k: sum(g[k] for g, _ in oracle) / world for k in oracle[0][0]}
    gmax = max(v.abs().max().item() for v in ref.values())
    for r in range(world):
        res = got[r]
        assert res["flat_is_grad"]
        for k, v in ref.items():
            g = torch.from_numpy(res["grad." + k]).double()
            assert torch.all((g - v).abs() <= 1e-4 * gmax + 1e-5 * v.abs()), (r, k)
        i = 0
        for l in range(nl - 1):
            for nm in ("bn1", "bn2"):
                for key in ("running_mean", "running_std"):
                    want = (sum(s[f"layer{l}.{nm}"][key] for _, s in oracle) / world).numpy()
                    np.testing.assert_allclose(res["running"][i], want, rtol=1e-4, atol=1e-5)
                    i += 1
    for k in ref:
        for r in range(1, world):
            assert np.array_equal(got[0]["grad." + k], got[r]["grad." + k]), (r, k)


def test_world2_config4_rank_shape_d128():
    """Config 4's per-rank shape: GNN_lg d=128, 5 layers, 512 graphs per rank (a global batch of
    1024 split in two Σ(N+M)-balanced shards), one step with the overlapped per-layer buckets;
    the averaged gradients and running statistics against the fp64 oracle's two-shard average."""
    d, nl, ng = 128, 5, 1024
    graphs, shards, oracle, got = _run_world(2, d, nl, ng)
    assert abs(len(shards[0]) - len(shards[1])) <= 16
    _check_world(2, nl, shards, oracle, got, ng)


def test_world8_config4_global_batch_4096_d128():
    """Config 4 itself on one device: 8 ranks (gloo over device tensors), GNN_lg d=128, 5 layers, one
    global batch of 4096 QM9-shape graphs in 8 Σ(N+M)-balanced shards of ~512, one step with the
    per-layer buckets and the running statistics in the same collectives.  Gradients and running
    statistics against the fp64 oracle's 8-shard average ("8 reference batches, gradients averaged",
    models/layers/batch_normalization.py:80-93), all 8 ranks bitwise identical."""
    d, nl, ng, world = 128, 5, 4096, 8
    graphs, shards, oracle, got = _run_world(world, d, nl, ng, timeout=600)
    assert max(len(s) for s in shards) - min(len(s) for s in shards) <= 16
    _check_world(world, nl, shards, oracle, got, ng)


def _nccl_world1_worker(port, q):
    """One rank in an RCCL ("nccl") process group of world size 1: the plain step's gradients, then the same
    step with LayerBucketAllReduce forced on (communication stream, per-layer executor events, the RCCL
    all-reduce kernels) -- a sum over one rank and a division by 1 leave every gradient bit unchanged."""
    os.environ.setdefault("HGNN_STRICT", "1")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        _paths()
        import fixture_util as fu
        from hgnn_amd.dp import LayerBucketAllReduce, running_stats
        from models.gnns.model_mnb import GNN_lg
        graphs, _ = _shards(1, 64)
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cuda() for t in _batch(graphs)]
        model = GNN_lg(0, D, L, 5, 1, 1, ORDER).cuda()
        fu.det_init(model, WSEED)
        out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        torch.nn.MSELoss()(out, T).backward()
        plain = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
        run_plain = [t.clone() for t in running_stats(model)]
        dp = LayerBucketAllReduce(model, force=True)
        res = {"backend": dist.get_backend()}
        for step in range(2):
            model.zero_grad(set_to_none=True)
            out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
            torch.nn.MSELoss()(out, T).backward()
            dp.timing = step == 1
            dp()
        torch.cuda.synchronize()
        res["comm"] = dp.timing_summary()
        res["flat_is_grad"] = all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(dp.params, dp.views))
        res["bitwise"] = {k: bool(torch.equal(p.grad, plain[k])) for k, p in model.named_parameters()}
        # the running statistics went through the collective too (after two more training forwards)
        res["running_finite"] = all(bool(torch.isfinite(t).all()) for t in running_stats(model))
        res["running_moved"] = any(not torch.equal(a, b) for a, b in zip(running_stats(model), run_plain))
        q.put(res)
    finally:
        dist.destroy_process_group()


def test_rccl_world1_bucketed_allreduce_bitwise():
    """The RCCL branch executed on hardware (review r05 #7): an "nccl" process group of world size 1 with the
    per-layer buckets forced on; every gradient bitwise equal to the step without DP."""
    import multiprocessing as mp
    ctx = mp.get_context("forkserver")
    q = ctx.Queue()
    pr = ctx.Process(target=_nccl_world1_worker, args=(_free_port(), q))
    pr.start()
    res = q.get(timeout=240)
    pr.join(timeout=120)
    assert pr.exitcode == 0
    assert res["backend"] == "nccl"
    assert res["flat_is_grad"]
    assert all(res["bitwise"].values()), [k for k, v in res["bitwise"].items() if not v]
    assert res["running_finite"] and res["running_moved"]
    assert res["comm"] is not None and res["comm"]["buckets"] == L - 1
