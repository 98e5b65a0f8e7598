"""ORACLE -- test infrastructure only.  The parity policy of SURVEY.md §8 c as functions.

Used by tests/ and by bench.py's cpu_baseline leg (which compares the GPU step against the
oracle run it times on the same batch).  Nothing in the product path imports it.

  outputs   |gpu - ref32| <= 1e-5 * max(1, max|ref32|)            (the reference's fp32 op order)
            |gpu - ref64| <= 2 * max|ref32 - ref64| + 1e-6         (fp64 anchor)
  gradients |gpu - ref|   <= 1e-4 * max_global|g| + 1e-5 * |g|     per element, global floor
            (cv2 / cv4 bias grads are analytically zero: their fp32 values are noise)
"""

import torch


def _t(x):
    return x.detach().to("cpu", torch.float64)


def outputs_two_leg(gpu, ref32, ref64=None, factor=2.0):
    g, r32 = _t(gpu), _t(ref32)
    scale = max(1.0, r32.abs().max().item())
    e32 = (g - r32).abs().max().item() if g.numel() else 0.0
    res = {"max_abs_vs_ref32": e32, "bound_ref32": 1e-5 * scale}
    ok = e32 <= 1e-5 * scale
    if ref64 is not None:
        r64 = _t(ref64)
        e64 = (g - r64).abs().max().item() if g.numel() else 0.0
        b64 = factor * ((r32 - r64).abs().max().item() if g.numel() else 0.0) + 1e-6
        res.update({"max_abs_vs_ref64": e64, "bound_ref64": b64})
        ok = ok and e64 <= b64
    res["pass"] = bool(ok)
    return res


def grads_global(gpu, ref):
    """gpu, ref: dicts name -> tensor (same keys).  Returns the worst element's error as a
    fraction of its bound (<= 1 passes) and the tensor it is in."""
    gmax = max(_t(v).abs().max().item() for v in ref.values())
    worst, where = 0.0, None
    for k, r in ref.items():
        assert gpu[k] is not None, k
        g, r = _t(gpu[k]), _t(r)
        bound = 1e-4 * gmax + 1e-5 * r.abs()
        frac = ((g - r).abs() / bound).max().item() if r.numel() else 0.0
        if frac > worst:
            worst, where = frac, k
    return {"gmax": gmax, "worst_err_over_bound": worst, "worst_tensor": where, "pass": bool(worst <= 1.0)}
