#!/usr/bin/env python3
"""Benchmark: graphs/s forward+backward, QM9-shape batch=512, LG-GNN 5-layer d=64 (BASELINE.json).

One step = one training pass of the drop-in GNN_lg (order 2, the reference's
`--update 2`) over a batch of 512 synthetic QM9-shape graphs already resident
in HBM: dense padded inputs as prepare_batch returns them, forward, MSE loss,
backward (X and W require grad as in scripts/train_mnb.py:56-57), and with N>1
GPUs the RCCL all-reduce of the gradients (batch-axis data parallelism, weak
scaling: each rank takes its Σ(N+M)-balanced shard of a global batch of 512·N
graphs, hgnn_amd.dp.shard_graphs; per-layer gradient buckets are all-reduced on a
communication stream while the earlier layers' backward still runs, and the BN
running statistics are averaged, hgnn_amd.dp.LayerBucketAllReduce).

Run:  python bench.py [--gpus N --steps K --warmup W]   (N > 1: starts the N ranks itself)
      python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
      (--gpus must equal the launcher's WORLD_SIZE)
Prints ONE JSON line (rank 0) with the BASELINE metric, a live roofline of the
dominant kernel class and HBM rooflines of the two aggregation classes (HIP
events around their launches in a second and a third timed region of the same steps), a
forward-only line (roofline_fwd), and the oracle's CPU time on a bounded sample
with the parity check of the GPU step against it (rank 0, N=1 only).
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "hgnn-2_amd"))
sys.path.insert(0, REPO)


def _dp_hw_queues():
    """With a process group (N > 1, or --force-dp 1), at least 8 hardware queues per process (set before HIP starts).
    The HIP runtime maps a process's streams round-robin onto GPU_MAX_HW_QUEUES queues (4 by default); the streams of
    an RCCL process group then push the executor's weight-gradient side stream onto the main stream's queue, which
    serialises the two: 1.31-1.33 vs 1.06-1.09 ms per step with an idle group at 4 vs 8 queues (tools/dp_ab.py,
    DESIGN.md §8 round 6).  The N = 1 run keeps the box's setting."""
    argv = " ".join(sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    gpus = 1
    for i, a in enumerate(sys.argv):
        if a == "--gpus" and i + 1 < len(sys.argv):
            gpus = int(sys.argv[i + 1])
        elif a.startswith("--gpus="):
            gpus = int(a.split("=", 1)[1])
    force = "--force-dp 1" in argv or "--force-dp=1" in argv
    if world > 1 or gpus > 1 or force:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
        if cur < 8:
            os.environ["GPU_MAX_HW_QUEUES"] = "8"


_dp_hw_queues()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "graphs/sec forward+backward, QM9-shape batch=512, LG-GNN 5-layer d=64"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bs", type=int, default=512, help="graphs per GPU")
    ap.add_argument("--d", "--dim", dest="d", type=int, default=64)
    ap.add_argument("--layers", type=int, default=5)
    ap.add_argument("--order", type=int, default=2)
    ap.add_argument("--settle-s", type=float, default=1.5,
                    help="untimed steps for this many seconds (after 40 warm-up / sampling steps) before the "
                         "warmup steps (clock ramp)")
    ap.add_argument("--force-dp", type=int, default=0,
                    help="at --gpus 1: form an RCCL (nccl) process group of world size 1 and run the per-layer "
                         "bucketed all-reduce anyway (exercises the N > 1 communication path on one GPU)")
    ap.add_argument("--dp-single", type=int, default=0,
                    help="N > 1: one all-reduce of the whole gradient buffer after the backward instead of per-layer "
                         "buckets overlapped with it")
    ap.add_argument("--attribution", type=int, default=1,
                    help="host-enqueue and GPU-busy time per step, each over a region of its own")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-bs", type=int, default=128,
                    help="graphs per step of the CPU baseline's timed protocol (bounded sample)")
    ap.add_argument("--cpu-warmup", type=int, default=3)
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--roofline", type=int, default=1)
    ap.add_argument("--fwd-line", type=int, default=1, help="also time the forward alone (cfg2f)")
    ap.add_argument("--graph", type=int, default=0,
                    help="capture the step (forward + backward) in a HIP graph and replay it (off by default: "
                         "the eager step is GPU-bound, DESIGN.md §8)")
    return ap.parse_args()


def make_batch(bs, seed, world=1, rank=0):
    """This rank's share of a global batch of bs * world QM9-shape graphs: Σ(N+M)-balanced shards
    (hgnn_amd.dp.shard_graphs, SURVEY.md §8 e); the reference's dense padded 11-tuple."""
    import hgnn_amd.datagen as dg
    from functions.batching import prepare_batch
    from functions.operators import graph_operators
    from hgnn_amd.dp import graph_cost, shard_graphs
    graphs = dg.qm9_shape_dataset(bs * world, seed=seed)
    if world > 1:
        mine = shard_graphs([graph_cost(X, A) for X, A, _ in graphs], world)[rank]
        graphs = [graphs[i] for i in mine]
    data = [[X, A, t, *graph_operators([X, A], 1, True)] for X, A, t in graphs]
    return list(prepare_batch(data, 0, 1))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, batch_cpu, model, gpu_res):
    """Oracle (CPU restatement of the reference, oracle/ref_mnb.py) with the same weights, timed to
    BASELINE.md §3's protocol on a bounded sample: --cpu-warmup (3) warm-up steps, then the median
    of --cpu-steps (5) fwd+bwd steps of --cpu-bs (128) graphs of the same generator and seed, forward
    and backward timed apart.  Then one fwd+bwd step of the full bench batch (also timed, reported
    beside it: the reference's per-slice CopySlices backward grows faster than the batch), whose
    outputs are the parity check of the GPU step (SURVEY.md §8 c policy, oracle/parity.py): fp32
    oracle (the reference's op order) for outputs, loss and every gradient, plus an fp64 forward
    (batched leg) as the second output leg."""
    from oracle import parity as PP
    from oracle import ref_mnb as R
    b = [t.clone() for t in batch_cpu]
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = b
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}  # leaves of their own
    threads = torch.get_num_threads()

    def run(bb, dtype=torch.float32, fast=False, grads=True):
        X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = bb
        p = {k: v.to(dtype).detach().clone().requires_grad_(grads) for k, v in sd.items()}
        st = R.bn_states(args.layers, 2 * args.d, dtype=dtype)
        Xr = X.to(dtype).detach().clone().requires_grad_(grads)
        Wr = W.to(dtype).detach().clone().requires_grad_(grads)
        t0 = time.perf_counter()
        with torch.set_grad_enabled(grads):
            out = R.gnn_lg(p, [Xr, XL.to(dtype), Wr, WL.to(dtype), Pm.to(dtype), Pd.to(dtype)], Nb, mask.to(dtype),
                           Eb, mask_lg.to(dtype), args.layers, args.order, st, True, fast=fast)
            loss = torch.nn.MSELoss()(out, T.to(dtype))
        t1 = time.perf_counter()
        if grads:
            loss.backward()
        t2 = time.perf_counter()
        g = {k: v.grad for k, v in p.items()} if grads else None
        return out.detach(), loss.item(), g, (Xr.grad, Wr.grad), t1 - t0, t2 - t1

    import statistics
    small = make_batch(args.cpu_bs, 1000)
    for _ in range(args.cpu_warmup):
        run(small)
    tf, tb = [], []
    for _ in range(max(1, args.cpu_steps)):
        r = run(small)
        tf.append(r[4])
        tb.append(r[5])
    tt = [f + b_ for f, b_ in zip(tf, tb)]
    med = statistics.median(tt)
    out32, loss32, g32, (dx32, dw32), t_f, t_b = run(b)
    out64 = run(b, torch.float64, fast=True, grads=False)[0]
    n = X.shape[0]
    res = {"value": round(args.cpu_bs / med, 3), "unit": "graphs/s", "cores": threads, "kind": "port",
           "cpu_model": _cpu_model(), "forward_s_median": round(statistics.median(tf), 4),
           "backward_s_median": round(statistics.median(tb), 4), "step_s_all": [round(x, 4) for x in tt],
           "full_batch_step": {"graphs": n, "value": round(n / (t_f + t_b), 3), "forward_s": round(t_f, 3),
                               "backward_s": round(t_b, 3)},
           "sample": f"BASELINE.md §3 protocol on a bounded sample: {args.cpu_warmup} warm-up steps, then the "
                     f"median of {len(tt)} fwd+bwd steps of {args.cpu_bs} QM9-shape graphs (same generator and "
                     f"seed), d={args.d}, L={args.layers}, order {args.order}, on oracle/ref_mnb.py (the reference's "
                     f"dense per-graph loops; torch CPU, {threads} threads); full_batch_step: one step of the "
                     f"{n}-graph bench batch, {t_f + t_b:.1f} s"}
    outp = PP.outputs_two_leg(gpu_res["out"], out32, out64)
    gr = PP.grads_global(gpu_res["grads"], g32)
    gx = PP.grads_global({"dX": gpu_res["dX"], "dW": gpu_res["dW"]}, {"dX": dx32, "dW": dw32})
    dloss = abs(gpu_res["loss"] - loss32)
    par = {"vs": "oracle fp32 (reference op order) on the bench batch and weights; outputs also vs fp64",
           "max_abs_out_vs_ref32": outp["max_abs_vs_ref32"], "bound_out_ref32": outp["bound_ref32"],
           "max_abs_out_vs_ref64": outp["max_abs_vs_ref64"], "bound_out_ref64": outp["bound_ref64"],
           "abs_loss_diff": dloss,
           "max_grad_err_over_bound": round(gr["worst_err_over_bound"], 4), "worst_grad": gr["worst_tensor"],
           "max_input_grad_err_over_bound": round(gx["worst_err_over_bound"], 4),
           "n_param_grads": len(g32)}
    par["pass"] = bool(outp["pass"] and gr["pass"] and gx["pass"] and dloss <= 1e-5 * max(1.0, abs(loss32)))
    return res, par


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`python bench.py --gpus N` without a launcher: start the N ranks as fresh child processes of
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) before this process touches
    the GPU, relay their output (rank 0's JSON line) and exit with their status.  A child, not an
    exec: this process must never replace itself once anything could have initialised HIP."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + ["--dim" if a == "--d" else a for a in sys.argv[1:]]
    # (torch.distributed.run's own parser takes "--d" for an ambiguous abbreviation of its options)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    proc = subprocess.run(cmd, env=env)
    if proc.returncode != 0:
        sys.stderr.write(f"bench: the {n}-rank run failed (exit {proc.returncode})\n")
    sys.exit(proc.returncode)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            launch_ranks(args.gpus)  # does not return
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench: --gpus {args.gpus} does not match WORLD_SIZE={os.environ['WORLD_SIZE']} "
                 "from the launcher")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HGNN_BENCH_BACKEND=gloo: rehearsal of the N > 1 path on a box with fewer GPUs than ranks (the
    # ranks share devices round-robin; gloo reduces device tensors through the host) -- timings of
    # such a run are not the RCCL numbers
    backend = os.environ.get("HGNN_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    force_dp = world == 1 and bool(args.force_dp)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    elif force_dp:
        torch.cuda.set_device(local)
        dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                **({"device_id": torch.device("cuda", local)} if backend == "nccl" else {}))
    dev = torch.device("cuda", local)

    from hgnn_amd import roofline as RF
    from hgnn_amd.net import KernelTimer
    from models.gnns.model_mnb import GNN_lg

    torch.manual_seed(0)
    model = GNN_lg(0, args.d, args.layers, 5, 1, 1, args.order).to(dev)
    params = list(model.parameters())
    batch_cpu = make_batch(args.bs, 1000, world, rank)
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.to(dev) for t in batch_cpu]
    X.requires_grad_(True)
    W.requires_grad_(True)
    crit = torch.nn.MSELoss()
    from hgnn_amd.dp import GradAllReduce, LayerBucketAllReduce
    # N > 1: per-layer gradient buckets reduced on a communication stream while the executor's
    # backward is still running (its per-layer events), BN running statistics averaged
    allreduce = (LayerBucketAllReduce(model, force=force_dp, single=bool(args.dp_single))
                 if (world > 1 or force_dp) and not args.graph
                 else GradAllReduce(params))
    last_out = [None]

    def compute():
        for p in params:
            p.grad = None
        X.grad = None
        W.grad = None  # the reference rebuilds W every batch: no accumulation into an old W.grad
        out = model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        loss = crit(out, T)
        loss.backward()
        # values only: keeping `out` itself would keep this step's autograd nodes alive, among them the
        # parameters' AccumulateGrad nodes with the stream they were created on -- a HIP-graph capture
        # on another stream then meets a cross-stream sync with that stream and capture_end fails
        # (tools/graph_diag.py)
        last_out[0] = out.detach()
        return loss.detach()

    def step():
        loss = compute()
        allreduce()  # no-op at N = 1
        return loss

    # warm-up, then settle by wall time (review r05 #1): WARM untimed steps first (one-time costs: module
    # loads, the caching allocator, the executor's program cache -- on a fresh box the first steps take
    # ~25 ms each, so a step time sampled over them sized the settle far too short), then the step time
    # sampled over SAMPLE more steps sizes a count of untimed steps covering --settle-s seconds, so a fresh
    # box's clocks have ramped before anything is timed.  A step count, not a deadline: every rank must
    # run the same number of steps (their all-reduces pair up), so the count is maxed over the ranks.
    WARM, SAMPLE = 20, 20
    settle_steps = 0
    settle_sample_ms = None
    if args.settle_s > 0:
        for _ in range(WARM):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(SAMPLE):
            step()
        torch.cuda.synchronize()
        per = max((time.perf_counter() - t0) / SAMPLE, 1e-5)
        settle_sample_ms = round(per * 1e3, 4)
        n = int(args.settle_s / per) + 1
        if world > 1:
            t = torch.tensor([n], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            n = int(t.item())
        for _ in range(n):
            step()
        settle_steps = WARM + SAMPLE + n
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    dominant = None
    if args.roofline:
        # two passes of prof_steps steps, per class the faster pass: one stalled launch (seen once:
        # 0.59 ms of agg_fwd in a 2-step pass) must not pick the class
        prof_steps = 3
        per = None
        for _ in range(2):
            with KernelTimer(8192, range(RF.N_CLASSES)) as tm:
                for _ in range(prof_steps):
                    step()
                torch.cuda.synchronize()
                cur = {k: tm.elapsed(k) for k in range(RF.N_CLASSES)}
            tm.close()
            per = cur if per is None else {k: min(per[k], cur[k]) for k in per}
        dominant = max(per, key=lambda k: per[k][0])

    # the dominant class, plus the two aggregation classes (the north_star's HBM-roofline target is on
    # the aggregation): each class gets a timed region of its own -- a HIP event recorded between two
    # kernels of the main stream also times the next dispatch's start-up and changes what the side
    # stream's blocks share the CUs with, so events around one class only keep its per-launch time
    # comparable with the rocprofv3 trace of the same command
    hbm_classes = [RF.K_AGG_FWD, RF.K_AGG_BWD]
    timed = ([dominant] + [k for k in hbm_classes if k != dominant]) if dominant is not None else []
    # in-kernel stamps (HGNN_TIMER_STAMPS): each wave of a timed launch writes its entry / exit time, nothing
    # is added to the stream -- event pairs around a dispatch make that dispatch itself slower (the
    # aggregation backward 19 -> 30 us per launch inside rocprofv3's own trace of a round-5 bench run)
    from hgnn_amd.net import TIMER_STAMPS
    wave_bound = 2 * (X.shape[0] * (X.shape[2] + XL.shape[2])) + 16384  # waves of the largest timed launch

    def stamp_timer(k, steps_):
        n = max(1, per[k][1] // prof_steps * steps_ + 8)
        return KernelTimer(n, [k], mode=TIMER_STAMPS, stamp_words=2 * n * wave_bound)
    timers = {k: stamp_timer(k, args.steps) for k in timed}
    graph = None
    if args.graph:
        # The step (~90 kernel launches + Python autograd) is captured once and replayed; every
        # kernel of the step runs on each replay.
        # The RCCL all-reduce of the gradients stays outside the graph (eager, after each replay).
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                compute()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            compute()
        graph.replay()
        allreduce()
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph is not None:
        for _ in range(args.steps):
            graph.replay()
            allreduce()  # no-op at N = 1
    else:
        for _ in range(args.steps):
            step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rank_ms = None
    comm = None
    if world > 1:
        # every rank's own time (a slow rank shows here), then the max over ranks for `value`
        e = torch.zeros(world, device=dev, dtype=torch.float64)
        e[rank] = elapsed
        dist.all_reduce(e)
        rank_ms = [round(float(v) * 1e3 / args.steps, 4) for v in e.cpu()]
        elapsed = float(e.max().item())
    if world > 1 or force_dp:
        if isinstance(allreduce, LayerBucketAllReduce):
            # the per-step gradient all-reduce (HIP events on the communication stream) over a
            # separate region of the same steps, so `value` carries no event records
            allreduce.timing = True
            for _ in range(args.steps):
                step()
            allreduce.timing = False
            comm = allreduce.timing_summary()
            if comm is not None:
                c = torch.tensor([comm["allreduce_span_ms"], comm["allreduce_exposed_ms"]], device=dev,
                                 dtype=torch.float64)
                dist.all_reduce(c, op=dist.ReduceOp.MAX)
                comm["allreduce_span_ms_max_rank"] = round(float(c[0]), 4)
                comm["allreduce_exposed_ms_max_rank"] = round(float(c[1]), 4)

    # attribution (review r05 #1), each over a region of its own after the `value` region: the host's
    # enqueue time per step (perf_counter around the steps, no synchronisation inside: the executor never
    # waits on the GPU, so this is the host's cost while the GPU still runs), and the GPU's busy time per
    # step: the union of every stamped executor launch span (all streams; in-kernel s_memrealtime stamps,
    # nothing added to the streams; torch's loss kernels and memsets are not stamped and count as idle)
    attribution = None
    if args.attribution and graph is None:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tw = time.perf_counter() - t0
        nb = 5
        tmb = KernelTimer(400 * nb, range(RF.N_CLASSES), mode=TIMER_STAMPS, stamp_words=(1 << 22) * nb)
        with tmb:
            for _ in range(nb):
                step()
            torch.cuda.synchronize()
        lau = tmb.launches(400 * nb)
        tmb.close()
        busy, span = [], []
        per_step = len(lau) // nb if lau else 0
        for i in range(nb if per_step else 0):
            iv = sorted((e0, e1) for _, e0, e1, _ in lau[i * per_step:(i + 1) * per_step])
            tot, cs, ce = 0.0, iv[0][0], iv[0][1]
            for e0, e1 in iv[1:]:
                if e0 > ce:
                    tot += ce - cs
                    cs, ce = e0, e1
                else:
                    ce = max(ce, e1)
            tot += ce - cs
            busy.append(tot)
            span.append(iv[-1][1] - iv[0][0] if iv else 0.0)
        import statistics as _st
        attribution = {
            "host_enqueue_ms_per_step": round(th * 1e3 / args.steps, 4),
            "wall_ms_per_step": round(tw * 1e3 / args.steps, 4),
            "gpu_busy_ms_per_step": round(_st.median(busy) / 1e3, 4) if busy else None,
            "gpu_span_ms_per_step": round(_st.median(span) / 1e3, 4) if span else None,
            "stamped_launches_per_step": per_step,
            "settle_sample_ms_per_step": settle_sample_ms,
            "note": ("host_enqueue: perf_counter over the enqueue of --steps steps without synchronisation; "
                     "gpu_busy: union of the stamped executor launch spans of one step (median of 5 steps, "
                     "all streams), gpu_span: first entry to last exit of the step's stamped launches"),
        }

    # every timed class over its own region of args.steps eager steps, after the `value` region (event
    # records cost ~10 us each: 1.90 vs 1.72 ms per step measured on one box; events captured into a
    # HIP graph give no elapsed times either)
    timer_ms = {}
    for k in timed:
        torch.cuda.synchronize()
        with timers[k]:
            for _ in range(args.steps):
                step()
        torch.cuda.synchronize()
        timer_ms[k] = timers[k].elapsed(k)
        timers[k].close()
    roof = None
    roof_hbm = None
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    ktr = os.path.join(REPO, "profiles", "kernel_trace.json")
    trace_note = ("committed profile (profiles/kernel_trace.json: rocprofv3 --kernel-trace of an earlier run of this "
                  "step, tools/trace_step.py), not measured in this run; frac_trace = the same work over that launch time")
    traffic_note = ("committed profile (profiles/pmc_traffic.json: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE of an earlier "
                    "run of this step), not measured in this run")
    if timed:
        counts = RF.batch_counts(W.detach(), WL, Pm, Pd, Nb, Eb)
        ms, n = timer_ms[dominant]
        roof = RF.roofline_entry(dominant, ms, n, counts, args.order, 5, args.d, args.layers, args.steps, pmc_path=pmc,
                                 trace_path=ktr)
        roof["traffic_source"] = traffic_note
        if "frac_trace" in roof:
            roof["trace_source"] = trace_note
        roof["timed_in"] = (f"a region of its own: {args.steps} eager steps, every wave of this class's launches "
                            "stamping s_memrealtime at entry and exit (a launch = last exit - first entry; no "
                            "events in the stream); each aggregation class in another such region")
        roof["class_ms_per_step_profile"] = {RF.NAMES[k]: round(v[0] / prof_steps, 4) for k, v in per.items()}
        roof_hbm = {}
        for k in hbm_classes:
            kms, kn = timer_ms[k]
            e = RF.roofline_entry(k, kms, kn, counts, args.order, 5, args.d, args.layers, args.steps, pmc_path=pmc,
                                  trace_path=ktr)
            roof_hbm[RF.NAMES[k]] = {x: e[x] for x in (
                "bound", "achieved", "peak", "unit", "frac", "traffic", "algorithmic_bytes_per_launch",
                "launches_per_step", "avg_launch_us", "requested_bytes_per_launch", "requested_gbs",
                "requested_frac", "traffic_gbs", "traffic_frac", "trace_avg_launch_us", "frac_trace") if x in e}
            roof_hbm[RF.NAMES[k]]["traffic_source"] = traffic_note

    # forward-only line (config "cfg2f"): the north star's HBM target is stated on the batched
    # LG-GNN forward.  Train-mode BN (batch statistics), no autograd graph kept.
    roof_fwd = None
    if args.fwd_line:
        from hgnn_amd.net import KernelTimer as KT

        def fwd():
            with torch.no_grad():
                model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg)
        for _ in range(3):
            fwd()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fwd()
        torch.cuda.synchronize()
        fms = (time.perf_counter() - t0) * 1e3 / args.steps
        nl = (args.layers * 2) * args.steps + 8  # aggregation launches of the forwards, with room
        with KT(nl, [RF.K_AGG_FWD], mode=TIMER_STAMPS, stamp_words=2 * nl * wave_bound) as tf:
            for _ in range(args.steps):
                fwd()
            torch.cuda.synchronize()
            ams, an = tf.elapsed(RF.K_AGG_FWD)
        tf.close()
        counts_f = RF.batch_counts(W.detach(), WL, Pm, Pd, Nb, Eb)
        ffl, fby = RF.forward_work(counts_f, args.order, 5, args.d, args.layers)
        agg = RF.roofline_entry(RF.K_AGG_FWD, ams, an, counts_f, args.order, 5, args.d, args.layers, args.steps)
        roof_fwd = {"workload": f"forward only (train-mode BN), {args.bs} graphs", "ms_per_forward": round(fms, 4),
                    "graphs_per_s": round(args.bs / fms * 1e3, 1),
                    "algorithmic_flops": ffl, "algorithmic_bytes": fby,
                    "achieved_tflops": round(ffl / fms / 1e9, 3),
                    "frac_mfma": round(ffl / fms / 1e9 / RF.PEAK_FP32_MFMA_TFS, 4),
                    "achieved_gbs": round(fby / fms / 1e6, 2),
                    "frac_hbm": round(fby / fms / 1e6 / RF.PEAK_HBM_GBS, 4),
                    "agg_fwd": {x: agg[x] for x in ("achieved", "unit", "frac", "launches_per_step", "avg_launch_us",
                                                    "requested_gbs", "requested_frac")}}

    value = args.bs * world * args.steps / elapsed
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "graphs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_steps": settle_steps,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic: seeded QM9-shape graphs (SURVEY.md §8 d generator), random-init weights",
        "launch": "hip_graph_replay" if graph is not None else "eager",
        "config": {
            "workload": f"GNN_lg order {args.order}, {args.layers} layers, d={args.d}, fwd+bwd, "
                        f"{args.bs} QM9-shape graphs per GPU",
            "graphs_per_gpu": args.bs,
            "global_batch": args.bs * world,
            "parallelism": f"dp{world}",
            "collective": ("rccl" if backend == "nccl" else backend) if (world > 1 or force_dp) else None,
        },
        "rank_ms_per_step": rank_ms,
        "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
        "comm": comm,
        "attribution": attribution,
        "roofline": roof,
        "roofline_hbm": roof_hbm,
        "roofline_fwd": roof_fwd,
        "cpu_baseline": None,
        "parity": None,
    }
    if rank == 0 and world == 1 and args.cpu_baseline:
        # one more GPU step on the same batch: its outputs / grads are checked against the oracle
        loss = compute()
        gpu_res = {"loss": loss.item(), "out": last_out[0].detach().cpu(),
                   "grads": {k: p.grad.detach().cpu() for k, p in model.named_parameters()},
                   "dX": X.grad.detach().cpu(), "dW": W.grad.detach().cpu()}
        res["cpu_baseline"], res["parity"] = cpu_baseline(args, batch_cpu, model, gpu_res)
    # every rank's last step must have produced a finite loss; any rank failing fails the run
    ok = 1 if bool(torch.isfinite(last_out[0].detach()).all()) else 0
    if world > 1:
        f = torch.tensor([ok], device=dev, dtype=torch.int32)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = int(f.item())
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1 or force_dp:
        dist.destroy_process_group()
    if not ok:
        sys.exit("bench: a rank produced non-finite outputs")
    if res.get("parity") is not None and not res["parity"]["pass"]:
        sys.exit("bench: GPU step breaches the SURVEY.md §8 c parity policy (see the 'parity' object)")


def _main_checked():
    """A rank that raises exits non-zero (torch.distributed.run then stops the others and fails)."""
    try:
        main()
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        sys.stderr.write(f"bench: rank {os.environ.get('RANK', '0')} failed: {e!r}\n")
        sys.stderr.flush()
        os._exit(1)


if __name__ == "__main__":
    _main_checked()
