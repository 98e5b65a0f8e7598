#!/usr/bin/env python3
"""In-kernel clock of the fp32 MFMA GEMMs during the config-2 step (MI355X_MICROARCH.md, DVFS
give-back item 6): run with the diagnostic build (make -C hgnn-2_amd BUILD=build_clk
OUT=hgnn_amd/libhgnn_amd_clk.so EXTRA=-DHGNN_CLOCK_DIAG) loaded through HGNN_LIB_PATH.  Wave 0
of every GEMM block stamps s_memtime / s_memrealtime around its main loop; after >= 2 s of
back-to-back steps the stamps of the next steps are read back and, per kernel, the median clock
(d memtime / d memrealtime x 100 MHz) and the median loop duration are printed as JSON.

  HGNN_LIB_PATH=hgnn-2_amd/hgnn_amd/libhgnn_amd_clk.so python tools/clock_diag.py [--settle-s 2]
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

KIDS = {0: "k_gemm3 (forward, 32x32x2)", 1: "k_gemm3 (dA / store)", 2: "k_gemm3_tn (dW)",
        3: "k_gemm5 (forward, 16x16x4)", 4: "k_gemm5 (dA, 16x16x4 LDS-DMA)"}


class Stamp(ctypes.Structure):
    _fields_ = [("dt", ctypes.c_uint64), ("dr", ctypes.c_uint64), ("kid", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--settle-s", type=float, default=2.0)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from bench import make_batch
    from hgnn_amd import _lib as L
    from models.gnns.model_mnb import GNN_lg
    lib = L.lib()
    if not hasattr(lib, "hgnn_diag_clock_read"):
        sys.exit("clock_diag: load the HGNN_CLOCK_DIAG build through HGNN_LIB_PATH")
    rd = lib.hgnn_diag_clock_read
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
    buf = (Stamp * 65536)()
    rd(ctypes.byref(buf), 0, 1)  # reset
    t1 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t1) * 1e3 / a.steps
    k = rd(ctypes.byref(buf), 65536, 1)
    per = {}
    for i in range(k):
        s = buf[i]
        if s.dr > 0:
            per.setdefault(int(s.kid), []).append((s.dt / s.dr * 100.0, s.dt))
    out = {"settle_steps": n, "settle_s": a.settle_s, "stamped_steps": a.steps, "ms_per_step_diag_build": round(ms, 4),
           "kernels": {}}
    for kid, v in sorted(per.items()):
        clk = sorted(x[0] for x in v)
        cyc = sorted(x[1] for x in v)
        out["kernels"][KIDS.get(kid, str(kid))] = {
            "blocks": len(v), "clock_mhz_median": round(statistics.median(clk), 1),
            "clock_mhz_p10": round(clk[len(clk) // 10], 1), "clock_mhz_p90": round(clk[(9 * len(clk)) // 10], 1),
            "loop_cycles_median": int(statistics.median(cyc)),
            "loop_us_median_at_clock": round(statistics.median(cyc) / statistics.median(clk), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
