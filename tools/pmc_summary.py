"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE on gfx950 counts
128-B requests as 64 B for wide (16 B/lane) coalesced reads, so it is doubled;
WRITE_SIZE is taken as is.  rocprofv3 reports both in KiB.
Usage: pmc_summary.py <fetch_dir> <write_dir> [out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    fetch = per_kernel(fd, "FETCH_SIZE")
    write = per_kernel(wd, "WRITE_SIZE")
    rows = []
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * 1024.0 * (sum(f) / len(f)) if f else None
        wb = 1024.0 * (sum(w) / len(w)) if w else None
        tot = (fb or 0.0) + (wb or 0.0)
        rows.append((tot, k, fb, wb, len(f)))
    rows.sort(reverse=True)
    res = {}
    for tot, k, fb, wb, n in rows:
        print(f"{tot / 1e6:10.3f} MB/launch  fetch(x2) {0 if fb is None else fb / 1e6:9.3f}  "
              f"write {0 if wb is None else wb / 1e6:9.3f}  n={n:4d}  {k[:90]}")
        res[k] = {"fetch_bytes_x2": fb, "write_bytes": wb, "traffic_bytes": tot, "launches": n}
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
