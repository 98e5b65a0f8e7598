#!/bin/bash
# Round 3: dW split-K with device-derived chunks -- parity tests, then A/B of the block target and
# the HIP-graph replay with / without packet capture.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py tests/test_gpu_fullsize.py tests/test_gpu_ops.py \
    tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
AB="HGNN_DW_BLOCKS=256|HGNN_DW_BLOCKS=512|HGNN_DW_BLOCKS=1024" REPS="1 2" bash tools/ab_env.sh || exit 1
AB="|DEBUG_CLR_GRAPH_PACKET_CAPTURE=0|DEBUG_HIP_FORCE_GRAPH_QUEUES=4" REPS="1" BENCH_ARGS="--graph 1" bash tools/ab_env.sh || exit 1
timeout -k 10 300 python bench.py --cpu-baseline 0 --fwd-line 0 > gpurun_out/b1.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/b1.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['class_ms_per_step_profile'], d['roofline']['frac'], d['roofline']['avg_launch_us'])"
timeout -k 10 200 python -u -m pytest tests/test_gpu_ccn.py tests/test_gpu_graph.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; tail -3 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/bench_configs.py --only cfg3_pergraph,cfg3,cfg3g,cfg1,cfg1g > gpurun_out/cfgs.jsonl 2>&1 || { tail -5 gpurun_out/cfgs.jsonl; exit 1; }
cut -c1-200 gpurun_out/cfgs.jsonl
