#!/usr/bin/env python3
"""HBM bytes per step: the per-kernel PMC traffic (profiles/pmc_traffic.json, tools/pmc.sh) weighted by
the launches per step of the step trace (tools/trace_step.py output).
usage: pmc_step_sum.py profiles/pmc_traffic.json profiles/rXX_trace_step.txt"""
import json
import re
import sys

t = json.load(open(sys.argv[1]))
per = {}
for line in open(sys.argv[2]):
    m = re.match(r"\s*([\d.]+) us/step\s+([\d.]+) launches\s+([\d.]+) us avg\s+(.*)$", line)
    if m:
        per[m.group(4).strip()] = float(m.group(2))
tot = 0.0
rows = []
for name, v in t.items():
    short = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("hgnn::", "").split("(")[0]
    n = next((c for k, c in per.items() if k.startswith(short[:60]) or short.startswith(k[:60])), 0.0)
    b = v["traffic_bytes"] * n
    tot += b
    rows.append((b, n, short))
for b, n, s in sorted(rows, reverse=True)[:15]:
    print(f"{b / 1e6:9.1f} MB/step  {n:4.1f} launches  {s[:80]}")
print(f"total {tot / 1e9:.3f} GB per step")
