#!/usr/bin/env python3
"""Per-step view of a rocprofv3 kernel trace of bench.py: per-kernel time per step, and the
busy / idle split of the GPU timeline (union of kernel intervals over the last steps).

usage: python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv [steps_in_trace] [out.json]
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 13
k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "")) for r in rows]
k.sort()
# the last `steps` steps: find the last k_plan / k_readout anchors -> use the final 40% of the trace
t_end = k[-1][1]
anchors = [s for s, e, n, q in k if "k_plan" in n or "k_repack" in n]
t0 = anchors[-min(len(anchors), max(1, steps // 2))]
win = [x for x in k if x[0] >= t0]
nstep = sum(1 for x in win if "k_plan" in x[2]) or 1
tot = defaultdict(float)
cnt = defaultdict(int)
for s, e, n, q in win:
    short = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("hgnn::", "").split("(")[0]
    tot[short] += (e - s) / 1e3
    cnt[short] += 1
span = (win[-1][1] - win[0][0]) / 1e3
# union of intervals
busy = 0.0
cs, ce = win[0][0], win[0][1]
for s, e, n, q in win[1:]:
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"steps in window: {nstep}; span {span / nstep:.1f} us/step; GPU busy (any kernel) {busy / 1e3 / nstep:.1f} us/step; "
      f"sum of kernel time {sum(tot.values()) / nstep:.1f} us/step")
for sid in sorted({q for _, _, _, q in win}):
    iv = [(s, e) for s, e, n, q in win if q == sid]
    b = 0
    cs, ce = iv[0]
    for s, e in iv[1:]:
        if s > ce:
            b += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    b += ce - cs
    print(f"  stream {sid}: {len(iv) / nstep:.0f} launches/step, busy {b / 1e3 / nstep:.1f} us/step")
for n, t in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{t / nstep:9.1f} us/step {cnt[n] / nstep:5.1f} launches  {t / cnt[n]:7.1f} us avg  {n[:90]}")
if len(sys.argv) > 3:  # JSON: per kernel, its average launch and launches per step (bench.py's roofline cross-check)
    import json
    with open(sys.argv[3], "w") as fh:
        json.dump({n: {"avg_us": round(t / cnt[n], 3), "launches_per_step": round(cnt[n] / nstep, 3)}
                   for n, t in tot.items()}, fh, indent=1)
