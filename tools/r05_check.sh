#!/bin/bash
# Round-5 GPU check: GPU tests, default bench, rocprofv3 kernel trace of the bench command (the timer's
# per-launch times reconciled against it), the marker-event timer for comparison, and the 8-rank gloo
# rehearsal of config 4 (d = 128, 512 graphs per rank).  Each step has its own limit; the first failure
# ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05a}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
    -- python3 bench.py --cpu-baseline 0 > $O/prof_bench.json 2> $O/prof_bench.err || { tail -5 $O/prof_bench.err; exit 1; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/reconcile.py $T $O/prof_bench.json | tee $O/reconcile.txt
python3 tools/trace_step.py $T 20 > $O/trace_step.txt || true
python3 tools/kstats.py $O/prof 40 > $O/kstats.txt || true
HGNN_TIMER_MARKERS=1 timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/bench_markers.json 2> $O/bench_markers.err || { tail -5 $O/bench_markers.err; exit 1; }
python3 tools/reconcile.py $T $O/bench_markers.json > $O/reconcile_markers.txt
cat $O/reconcile_markers.txt
if [ "${SKIP_GLOO8:-0}" != "1" ]; then
  HGNN_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 8 --d 128 --steps 5 --roofline 0 --fwd-line 0 \
      > $O/bench_gloo8_d128.json 2> $O/bench_gloo8_d128.err || { tail -5 $O/bench_gloo8_d128.err; exit 1; }
  tail -1 $O/bench_gloo8_d128.json | cut -c1-600
fi
