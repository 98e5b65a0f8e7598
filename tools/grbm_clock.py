#!/usr/bin/env python3
"""Effective clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md,
DVFS give-back: clock ~= GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time; reads high on dispatches
shorter than ~0.3 ms).  Usage: grbm_clock.py <pmc_dir> [name-substring ...]"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    want = sys.argv[2:]
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != "GRBM_GUI_ACTIVE":
                continue
            k = r["Kernel_Name"]
            if want and not any(w in k for w in want):
                continue
            t0, t1 = r.get("Start_Timestamp"), r.get("End_Timestamp")
            if not t0 or not t1:
                continue
            dur_ns = float(t1) - float(t0)
            if dur_ns > 0:
                acc[k].append((float(r["Counter_Value"]) / 8.0 / dur_ns * 1e3, dur_ns / 1e3))
    for k, v in sorted(acc.items(), key=lambda kv: -sum(x[1] for x in kv[1])):
        print(f"{statistics.median(x[0] for x in v):8.1f} MHz  {statistics.median(x[1] for x in v):8.2f} us  "
              f"n={len(v):4d}  {k[:110]}")


if __name__ == "__main__":
    main()
