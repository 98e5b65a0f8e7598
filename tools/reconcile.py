#!/usr/bin/env python3
"""Per-launch times of bench.py's roofline classes against a rocprofv3 kernel trace of the same command.

usage: python tools/reconcile.py <run_kernel_trace.csv> <bench JSON line file>
For each class bench.py times (the dominant class and the two aggregation classes), prints the bench's
avg_launch_us next to the trace's mean dispatch duration over every launch of the class's kernels in the
whole run (hgnn_amd.roofline.CLASS_KERNELS), and their ratio.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hgnn-2_amd"))
from hgnn_amd import roofline as RF  # noqa: E402

rows = list(csv.DictReader(open(sys.argv[1])))
line = [x for x in open(sys.argv[2]).read().splitlines() if x.startswith("{")][-1]
b = json.loads(line)
ent = {}
if b.get("roofline"):
    ent[b["roofline"]["kernel"]] = b["roofline"]["avg_launch_us"]
for k, v in (b.get("roofline_hbm") or {}).items():
    ent[k] = v["avg_launch_us"]
print(f"{'class':10s} {'bench us':>9s} {'trace us':>9s} {'n trace':>8s} {'bench/trace':>11s}")
for name, us in ent.items():
    kc = RF.NAMES.index(name)
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if RF._in_class(kc, r["Kernel_Name"])]
    m = sum(d) / len(d) if d else float("nan")
    print(f"{name:10s} {us:9.2f} {m:9.2f} {len(d):8d} {us / m:11.3f}")
