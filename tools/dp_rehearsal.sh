#!/bin/bash
# Rehearsal of bench.py's N = 2 path on a one-GPU box: two ranks on cuda:0 over gloo (the
# RCCL run is the driver's 8-GPU scaling bench).  Checks the launcher, sharding, layer buckets,
# BN statistics averaging, max-over-ranks timing and the JSON line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
HGNN_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-baseline 0 \
    > gpurun_out/dp2.json 2> gpurun_out/dp2.err || { tail -20 gpurun_out/dp2.err; exit 1; }
tail -1 gpurun_out/dp2.json | cut -c1-700
