#!/usr/bin/env python3
"""Where a dW GEMM launch (k_gemm3_tn, side stream) spends its span inside the config-2 step: run with the
diagnostic build (make -C hgnn-2_amd BUILD=build_clk OUT=hgnn_amd/libhgnn_amd_clk.so EXTRA=-DHGNN_CLOCK_DIAG)
loaded through HGNN_LIB_PATH.  Thread 0 of every dW block stamps s_memrealtime (100 MHz, chip-wide) at
entry, loop start, loop end and exit with the CU it ran on; after >= 2 s of back-to-back steps the stamps of
the next steps are grouped into launches (time gaps) and summarised per launch shape:

  span            first entry -> last exit of the launch (us)
  pre / loop / post   per-block medians: entry -> loop start (index math, first loads), main loop, epilogue
  late_blocks     blocks whose entry is later than the first entry + 0.5 x the median block time (a
                  second round of blocks, or blocks that waited for CUs held by main-stream kernels)
  entry_p50/p90/max   entry offsets from the first entry
  cus             distinct CUs (XCC, SE, SH, CU) the launch ran on

  HGNN_LIB_PATH=hgnn-2_amd/hgnn_amd/libhgnn_amd_clk.so python tools/dw_phases.py [--settle-s 2 --steps 3]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "hgnn-2_amd"), REPO]

import torch  # noqa: E402


class Stamp(ctypes.Structure):
    _fields_ = [("t", ctypes.c_uint64 * 4), ("hw", ctypes.c_uint32), ("xcc", ctypes.c_uint32),
                ("blk", ctypes.c_uint32), ("rows", ctypes.c_uint32)]


def q(v, f):
    v = sorted(v)
    return v[min(len(v) - 1, int(f * len(v)))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settle-s", type=float, default=2.0)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from bench import make_batch
    from hgnn_amd import _lib as L
    from models.gnns.model_mnb import GNN_lg
    lib = L.lib()
    if not hasattr(lib, "hgnn_diag_phase_read"):
        sys.exit("dw_phases: load the HGNN_CLOCK_DIAG build through HGNN_LIB_PATH")
    rd = lib.hgnn_diag_phase_read
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    rd.restype = ctypes.c_int
    torch.manual_seed(0)
    model = GNN_lg(0, 64, 5, 5, 1, 1, 2).cuda()
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = [t.cuda() for t in make_batch(512, 1000)]
    X.requires_grad_(True)
    W.requires_grad_(True)

    def step():
        model.zero_grad(set_to_none=True)
        X.grad = W.grad = None
        torch.nn.MSELoss()(model([X, XL, W, WL, Pm, Pd], Nb, mask, Eb, mask_lg), T).backward()

    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < a.settle_s:
        step()
        n += 1
        if n % 20 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    cap = 1 << 17
    buf = (Stamp * cap)()
    rd(ctypes.byref(buf), 0, 1)  # reset
    t1 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t1) * 1e3 / a.steps
    k = rd(ctypes.byref(buf), cap, 1)
    st = sorted((buf[i] for i in range(k)), key=lambda s: s.t[0])
    # launches: the side stream runs them one after the other, so a block entering after every block of
    # the current group has exited starts the next launch
    launches, cur, last_exit = [], [], 0
    for s in st:
        if cur and s.t[0] > last_exit:
            launches.append(cur)
            cur = []
        cur.append(s)
        last_exit = max(last_exit, s.t[3]) if len(cur) > 1 else s.t[3]
    if cur:
        launches.append(cur)
    shapes = {}
    for ln in launches:
        live = [s for s in ln if s.rows > 0]
        if not live:
            continue
        t_first = min(s.t[0] for s in ln)
        span = (max(s.t[3] for s in ln) - t_first) / 100.0
        tot = [(s.t[3] - s.t[0]) / 100.0 for s in live]
        med_tot = statistics.median(tot)
        ent = [(s.t[0] - t_first) / 100.0 for s in ln]
        late = sum(1 for e in ent if e > 0.5 * med_tot)
        cus = {(s.xcc & 0xF, (s.hw >> 13) & 7, (s.hw >> 12) & 1, (s.hw >> 8) & 0xF) for s in ln}
        key = f"{len(ln)} blocks, {max(s.rows for s in live)} rows per chunk"
        shapes.setdefault(key, []).append({
            "span_us": span, "pre_us": statistics.median((s.t[1] - s.t[0]) / 100.0 for s in live),
            "loop_us": statistics.median((s.t[2] - s.t[1]) / 100.0 for s in live),
            "post_us": statistics.median((s.t[3] - s.t[2]) / 100.0 for s in live),
            "block_us": med_tot, "late_blocks": late, "blocks": len(ln), "empty_blocks": len(ln) - len(live),
            "entry_p50_us": q(ent, 0.5), "entry_p90_us": q(ent, 0.9), "entry_max_us": max(ent),
            "exit_spread_us": (max(s.t[3] for s in ln) - min(s.t[3] for s in ln)) / 100.0, "cus": len(cus)})
    out = {"settle_steps": n, "stamped_steps": a.steps, "ms_per_step_diag_build": round(ms, 4), "stamps": k,
           "launches": len(launches), "shapes": {}}
    for key, v in shapes.items():
        out["shapes"][key] = {f: round(statistics.median(x[f] for x in v), 2) for f in v[0]}
        out["shapes"][key]["launches"] = len(v)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
