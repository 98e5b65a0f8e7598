"""Algorithmic work (FLOPs / compulsory HBM bytes) of each kernel class of the executor.

Used by bench.py to turn a measured kernel-class duration into a roofline
fraction.  Counts follow SURVEY.md §8 d: sizes from the actual batch (real,
unpadded rows; nnz of the extracted operator lists including the phantom edge
slots), fp32 = 4 B, index = 4 B; every input row read once, every output row
written once (gather re-reads served on chip are not algorithmic traffic).
"""

import torch

from .net import expected_k

PEAK_HBM_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_FP32_MFMA_TFS = 157.3   # v_mfma_f32_32x32x2_f32 dense peak
PEAK_BF16_MFMA_TFS = 16 * PEAK_FP32_MFMA_TFS  # dense bf16 MFMA: 16x the fp32 rate per clock (MI355X_MICROARCH.md)
# the split-bf16 GEMMs (k_gemm_bf3_fwd, k_gemm_bf3_da, k_gemm_bf3_tn) run six bf16 products per fp32 product: their fp32
# algorithmic FLOPs are priced against a sixth of the bf16 peak
PEAK_SPLIT_BF16_TFS = PEAK_BF16_MFMA_TFS / 6

(K_STRUCT, K_AGG_FWD, K_GEMM_FWD, K_BN_FWD, K_READOUT, K_BN_BWD, K_GEMM_DW, K_GEMM_DA, K_AGG_BWD, K_DW_DENSE,
 K_DW_REDUCE) = range(11)
NAMES = ["struct", "agg_fwd", "gemm_fwd", "bn_fwd", "readout", "bn_bwd", "gemm_dw", "gemm_da", "agg_bwd", "dw_dense",
         "dw_reduce"]
N_CLASSES = len(NAMES)


def batch_counts(W, WL, Pm, Pd, N_batch, E_batch):
    """Real rows and union-pattern nnz of the operator lists (host, from the dense batch)."""
    nW = int((W != 0).any(dim=3).sum())
    nWL = int((WL != 0).any(dim=3).sum())
    nP = int(((Pm != 0) | (Pd != 0)).sum())
    return dict(nodes=int(N_batch.sum()), edges=int(E_batch.sum()), nnz_w=nW, nnz_wl=nWL, nnz_p=nP)


def lg_halves(order, f_in, d, n_layers, jt):
    """(edge?, rows key, K, Cg, Cp) per half in program order, mirroring net.hip build_program."""
    ks, k_last = expected_k(1, order, f_in, d, n_layers, jt)
    out = []
    cn, ce = f_in, 1
    for kn, ke in ks:
        if order == 1:
            hs = [(False, kn, cn, ce), (True, ke, ce, 2 * d)]
        elif order == 2:
            hs = [(True, ke, ce, cn), (False, kn, cn, 2 * d)]
        else:
            hs = [(False, kn, cn, ce), (True, ke, ce, cn)]
        out += hs
        cn, ce = 2 * d, 2 * d
    return out, k_last


def diag_id(cg, cp, d):
    """Whether the executor builds a half's I / D operand columns in its GEMMs instead of aggregating them (net.hip
    diag_id_on: HGNN_DIAG_ID=1 (off by default), the split-bf16 forward and dW GEMMs, 2d % 64 == 0, 2d <= 256; halves whose G input
    is a layer output of 2d channels)."""
    import os
    c2 = 2 * d
    on = (os.environ.get("HGNN_DIAG_ID", "0") == "1" and split_bf16(K_GEMM_FWD, d) and split_bf16(K_GEMM_DW, d)
          and c2 <= 256)
    return on and cg == c2 and cp in (0, c2)


def class_work(kcls, counts, order, f_in, d, n_layers, jt=3):
    """(flops, bytes) of one training step for kernel class kcls (sum over its launches).  With the diagonal I / D
    columns (diag_id) the aggregate a half stores is k - 2 cg wide and its GEMMs read the half's input (cg wide)
    for the other 2 cg operand columns."""
    halves, k_last = lg_halves(order, f_in, d, n_layers, jt)
    c2 = 2 * d
    rows = lambda edge: counts["edges"] if edge else counts["nodes"]  # noqa: E731
    nnz_g = lambda edge: counts["nnz_wl"] if edge else counts["nnz_w"]  # noqa: E731
    opnd = lambda k, cg, cp: (k - cg) if diag_id(cg, cp, d) else k  # noqa: E731  (operand columns read per row)
    fl = by = 0.0
    if kcls == K_GEMM_FWD:
        for edge, k, cg, cp in halves:
            r = rows(edge)
            fl += 2.0 * r * k * c2
            by += 4.0 * (r * opnd(k, cg, cp) + r * c2 + c2 * (k + 1))
    elif kcls == K_GEMM_DA:
        for edge, k, cg, cp in halves:
            r = rows(edge)
            fl += 2.0 * r * c2 * k
            by += 4.0 * (r * c2 + r * k + c2 * k)
    elif kcls == K_GEMM_DW:
        for edge, k, cg, cp in halves:
            r = rows(edge)
            fl += 2.0 * r * c2 * k
            by += 4.0 * (r * c2 + r * opnd(k, cg, cp) + c2 * k)
    elif kcls in (K_AGG_FWD, K_AGG_BWD):
        # the last layer's forward aggregation is a k_agg_fwd launch; its backward is the readout class
        # (k_readout_agg_bwd: the readout gradient R_b broadcast per graph, no [rows][K] dA read)
        items = [(e, k, cg, cp) for e, k, cg, cp in halves] + ([(False, k_last, c2, c2)] if kcls == K_AGG_FWD else [])
        for i, (edge, k, cg, cp) in enumerate(items):
            r, ro = rows(edge), rows(not edge)
            cut = kcls == K_AGG_FWD and i < len(halves) and diag_id(cg, cp, d)
            s_bytes = 8.0 * (r + r) + 16.0 * (nnz_g(edge) + counts["nnz_p"])
            by += 4.0 * (r * (k - 2 * cg if cut else k) + r * cg + ro * cp) + s_bytes
            fl += 2.0 * (nnz_g(edge) * (jt - 2 if cut else jt) * cg + 2 * counts["nnz_p"] * cp)
    elif kcls == K_BN_FWD:
        for edge, k, cg, cp in halves:
            by += 4.0 * 2 * rows(edge) * c2
    elif kcls == K_BN_BWD:
        # statistics pass (dz, y read) and apply pass (dz, y read, dY written)
        for edge, k, cg, cp in halves:
            by += 4.0 * 5 * rows(edge) * c2
    return fl, by


def agg_requested_bytes(kcls, counts, order, f_in, d, n_layers, jt=3):
    """Bytes the aggregation kernels of one step request from the memory system, on-chip reuse
    not subtracted: one source row per list entry (forward: the row feeds all J+2 coefficients;
    backward: one row slice per nonzero coefficient -- the diagonal entry's I and D slices, one
    A slice per other entry), every output row written once, the row lists read once.  The
    gap to class_work's compulsory bytes is what the L2 / MALL serve."""
    halves, k_last = lg_halves(order, f_in, d, n_layers, jt)
    c2 = 2 * d
    rows = lambda edge: counts["edges"] if edge else counts["nodes"]  # noqa: E731
    nnz_g = lambda edge: counts["nnz_wl"] if edge else counts["nnz_w"]  # noqa: E731
    by = 0.0
    if kcls == K_AGG_FWD:
        for i, (edge, k, cg, cp) in enumerate(halves + [(False, k_last, c2, c2)]):
            r = rows(edge)
            kw = k - 2 * cg if i < len(halves) and diag_id(cg, cp, d) else k
            by += 4.0 * (nnz_g(edge) * cg + counts["nnz_p"] * cp + r * kw) + 8.0 * 2 * r + 16.0 * (
                nnz_g(edge) + counts["nnz_p"])
    elif kcls == K_AGG_BWD:
        for edge, k, cg, cp in halves:
            r, ro = rows(edge), rows(not edge)
            by += 4.0 * ((nnz_g(edge) + r) * cg + 2 * counts["nnz_p"] * cp + r * cg + ro * cp) + 8.0 * (r + ro) + 16.0 * (
                nnz_g(edge) + counts["nnz_p"])
    return by


def forward_work(counts, order, f_in, d, n_layers, jt=3):
    """(flops, compulsory bytes) of one LG-GNN forward (SURVEY.md §8 d 'LG-GNN forward bytes / FLOPs'):
    every layer reads its input features once and writes its pre-BN output once; the structure
    (CSR of W, WL, Pm, Pd: 4 (rows + 1) + 8 nnz) is read by every layer; weights once."""
    halves, k_last = lg_halves(order, f_in, d, n_layers, jt)
    c2 = 2 * d
    N, M = counts["nodes"], counts["edges"]
    by = 0.0
    cn, ce = f_in, 1
    for _ in range(n_layers - 1):
        by += 4.0 * (cn * N + ce * M + c2 * (N + M))
        cn, ce = c2, c2
    by += 4.0 * (c2 * (N + M)) + 4.0
    S = (4.0 * (N + 1) + 8.0 * counts["nnz_w"] + 4.0 * (M + 1) + 8.0 * counts["nnz_wl"] +
         2 * (4.0 * (N + 1) + 8.0 * counts["nnz_p"]))
    by += n_layers * S
    params = sum(c2 * (k + 1) for _, k, _, _ in halves) + k_last + 1
    by += 4.0 * params
    fl = sum(class_work(k, counts, order, f_in, d, n_layers, jt)[0] for k in (K_GEMM_FWD, K_AGG_FWD))
    fl += 2.0 * N * k_last
    return fl, by


# kernel-name predicates of each class (rocprofv3 names of csrc/*.hip), for the PMC traffic join
CLASS_KERNELS = {
    K_STRUCT: ("k_plan", "k_extract", "k_pack_nodes", "k_pack_edges", "k_repack", "k_unpack_nodes"),
    K_AGG_FWD: ("k_agg_fwd",),
    K_GEMM_FWD: ("k_gemm3<", "k_gemm_fwd", "k_gemm_bf3_fwd", "k_gemm5<"),
    K_BN_FWD: ("k_bn_finalize", "k_bn_apply"),
    K_READOUT: ("k_readout",),  # incl. k_readout_agg_bwd (net.hip times it in this class)
    K_BN_BWD: ("k_bn_bwd",),
    K_GEMM_DW: ("k_gemm3_tn", "k_gemm_dw", "k_gemm_bf3_tn"),
    K_GEMM_DA: ("k_gemm3<", "k_gemm_da", "k_gemm5<", "k_gemm_bf3_da"),
    K_AGG_BWD: ("k_agg_bwd",),
    K_DW_DENSE: ("k_dw_dense",),
    K_DW_REDUCE: ("k_dw_reduce",),
}


def _in_class(kcls, name):
    if not any(t in name for t in CLASS_KERNELS[kcls]):
        return False
    if "k_gemm3<" in name:  # k_gemm3<BM, BN, BK, WGM, WGN, EPI>: EPI 0 = forward, 1 = dA
        epi = name.split(">")[0].rsplit(",", 1)[-1].strip()
        return (kcls == K_GEMM_FWD) == (epi == "0")
    if "k_gemm5<" in name:  # k_gemm5<BM, BN, WGM, WGN, FWD>: the forward epilogue or dA
        fwd = name.split(">")[0].rsplit(",", 1)[-1].strip()
        return (kcls == K_GEMM_FWD) == (fwd == "true")
    return True


def split_bf16(kcls, d):
    """Whether the executor runs class kcls on the split-bf16 GEMMs at width d (net.hip fwd_bf3 / da_bf3,
    gemm3.hip launch_gemm3_dw; their switches HGNN_FWD_BF3 / HGNN_DA_BF3 / HGNN_DW_BF3)."""
    import os
    if kcls == K_GEMM_FWD:
        return (2 * d) % 64 == 0 and os.environ.get("HGNN_FWD_BF3", "1") != "0"
    if kcls == K_GEMM_DA:
        return (2 * d + 3) // 4 * 4 <= 128 and os.environ.get("HGNN_DA_BF3", "1") != "0"
    if kcls == K_GEMM_DW:
        return os.environ.get("HGNN_DW_BF3", "1") != "0"
    return False


def pmc_traffic(kcls, path):
    """HBM bytes per launch of class kcls from a tools/pmc_summary.py JSON (FETCH_SIZE x2 + WRITE_SIZE,
    MI355X_MICROARCH.md HBM section), launch-weighted over the class's kernels; None if absent."""
    import json
    import os
    if not path or not os.path.exists(path):
        return None
    with open(path) as fh:
        rows = json.load(fh)
    tot = n = 0.0
    for name, r in rows.items():
        if _in_class(kcls, name) and r.get("traffic_bytes") is not None:
            tot += r["traffic_bytes"] * r["launches"]
            n += r["launches"]
    return tot / n if n else None


def trace_avg_us(kcls, path):
    """Average launch duration (us) of class kcls in a committed rocprofv3 kernel trace of the bench step
    (tools/trace_step.py --json: per kernel avg_us and launches per step), launch-weighted; None if absent."""
    import json
    import os
    if not path or not os.path.exists(path):
        return None
    with open(path) as fh:
        rows = json.load(fh)
    tot = n = 0.0
    for name, r in rows.items():
        if _in_class(kcls, name):
            tot += r["avg_us"] * r["launches_per_step"]
            n += r["launches_per_step"]
    return tot / n if n else None


def roofline_entry(kcls, ms_total, launches, counts, order, f_in, d, n_layers, steps, jt=3, pmc_path=None,
                   trace_path=None):
    """bench.py 'roofline' object for a kernel class measured over `steps` steps."""
    fl, by = class_work(kcls, counts, order, f_in, d, n_layers, jt)
    sec = max(ms_total / 1e3, 1e-12)
    extra = {}
    if kcls in (K_GEMM_FWD, K_GEMM_DA, K_GEMM_DW):
        achieved = fl * steps / sec / 1e12
        peak, unit, bound = PEAK_FP32_MFMA_TFS, "TFLOP/s", "mfma"
        if split_bf16(kcls, d):
            peak = round(PEAK_SPLIT_BF16_TFS, 1)
            extra["peak_note"] = ("fp32 algorithmic FLOPs against the split-bf16 rate: dense bf16 MFMA peak "
                                  f"{PEAK_BF16_MFMA_TFS:.1f} TFLOP/s / 6 products per fp32 product")
    else:
        achieved = by * steps / sec / 1e9
        peak, unit, bound = PEAK_HBM_GBS, "GB/s", "hbm"
    per_launch = launches / max(steps, 1)
    traffic = pmc_traffic(kcls, pmc_path)
    avg_s = ms_total / 1e3 / max(launches, 1)
    if traffic is not None and bound == "hbm":
        # the HBM bytes the PMC counters saw per launch, over the same per-launch time
        extra["traffic_gbs"] = round(traffic / avg_s / 1e9, 1)
        extra["traffic_frac"] = round(traffic / avg_s / 1e9 / PEAK_HBM_GBS, 4)
    tr = trace_avg_us(kcls, trace_path)
    if tr is not None:
        # the same algorithmic work over the kernel trace's launch time (rocprofv3's dispatch end includes the
        # end-of-kernel write-back that the in-kernel stamps leave out)
        extra["trace_avg_launch_us"] = round(tr, 3)
        extra["frac_trace"] = round(achieved / peak * (avg_s * 1e6) / tr, 4)
    if kcls in (K_AGG_FWD, K_AGG_BWD):
        rq = agg_requested_bytes(kcls, counts, order, f_in, d, n_layers, jt)
        rq_gbs = rq * steps / sec / 1e9
        extra.update({"requested_bytes_per_launch": rq / max(per_launch, 1e-9), "requested_gbs": round(rq_gbs, 1),
                      "requested_frac": round(rq_gbs / PEAK_HBM_GBS, 4)})
    return {**extra, **{
        "kernel": NAMES[kcls],
        "bound": bound,
        "achieved": round(achieved, 3),
        "peak": peak,
        "unit": unit,
        "frac": round(achieved / peak, 4),
        "traffic": traffic,
        "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_traffic.json)",
        "algorithmic_bytes_per_launch": by / max(per_launch, 1e-9),
        "launches_per_step": per_launch,
        "avg_launch_us": round(ms_total * 1e3 / max(launches, 1), 3),
        "algorithmic_per_step": {"flops": fl, "bytes": by},
    }}


def to_device_counts(batch):
    X, W, T, XL, WL, Pm, Pd, mask, mask_lg, Nb, Eb = batch
    with torch.no_grad():
        return batch_counts(W, WL, Pm, Pd, Nb, Eb)
