"""ctypes binding of include/hgnn_amd.h (the C ABI of the gfx950 hot path).

The shared library is built in-tree (``make -C hgnn-2_amd`` or
``__graft_entry__.build()``) next to this file.  torch is imported first so
that the HIP runtime torch already loaded (same soname, libamdhip64.so.7) is
the one the library binds to: one runtime per process.

There is no fallback: if the library is missing, every product entry point
raises.
"""

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before ours)

LIB_PATH = os.environ.get("HGNN_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                            "libhgnn_amd.so")

HGNN_OK = 0
STATUS = {0: "ok", 1: "invalid argument", 2: "unsupported configuration", 3: "HIP runtime error",
          4: "index out of range"}
DEVERR = {
    0x1: "operator entry outside a graph's real block (padding must be zero)",
    0x2: "mask[:, :, 0] disagrees with N_batch / E_batch",
    0x4: "N_batch > Nmax, E_batch > Emax or a negative count",
    0x8: "CCN adjacency without a self loop (chi_ii undefined, functions/utils_ccn.py:137-140)",
    0x10: "CCN vertex degree above the compiled bound (1024 for CCN-1D, 256 for CCN-2D)",
    0x20: "CCN adjacency pattern is not symmetric (the batched CCN backward needs A_ij > 0 <=> A_ji > 0)",
    0x40: ("operator slice 0 or 1 (graph_operators' I and D, functions/operators.py:19-23) holds an off-diagonal "
           "entry, which the opt-in HGNN_DIAG_ID=1 form (these two slices taken as diagonal) cannot take -- unset "
           "HGNN_DIAG_ID (the default aggregates them as general slices)"),
}


class NetConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "kind", "order", "bs", "nmax", "emax", "f_in", "d", "n_layers", "j_tot", "dim_out",
        "training", "need_dx", "need_dw", "reserved")]


class NetInputs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "d_X", "d_XL", "d_W", "d_WL", "d_Pm", "d_Pd", "d_N_batch", "d_E_batch", "d_mask", "d_mask_lg")]


class CsrLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("bs", "nmax", "emax", "f_in", "j_tot", "dual", "stride_w",
                                               "reserved")] + \
               [("nodes", ctypes.c_int64), ("edges", ctypes.c_int64), ("rows", ctypes.c_int64 * 6),
                ("nnz", ctypes.c_int64 * 6)] + \
               [(n, ctypes.c_int64) for n in ("off_node_off", "off_edge_off", "off_totals", "off_n_batch",
                                               "off_e_batch", "off_x", "off_xl")] + \
               [("off_rows", ctypes.c_int64 * 6), ("off_entries", ctypes.c_int64 * 6), ("bytes", ctypes.c_int64)]


class CsrBatch(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("d_node_off", "d_edge_off", "d_totals", "d_n_batch", "d_e_batch",
                                                "d_x", "d_xl")] + \
               [("d_rows", ctypes.c_void_p * 6), ("d_entries", ctypes.c_void_p * 6),
                ("stride_w", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("nodes", ctypes.c_int64), ("edges", ctypes.c_int64)]


class CcnConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("order", "bs", "nmax", "f_in", "hidden", "layers", "n_out", "reserved")]


_lib = None

_VP = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long

SIGNATURES = {
    "hgnn_abi_version": ([], _I),
    "hgnn_status_string": ([_I], ctypes.c_char_p),
    "hgnn_net_param_count": ([ctypes.POINTER(NetConfig)], _I),
    "hgnn_net_bn_count": ([ctypes.POINTER(NetConfig)], _I),
    "hgnn_net_workspace_bytes": ([ctypes.POINTER(NetConfig)], ctypes.c_size_t),
    "hgnn_net_error_word": ([ctypes.POINTER(NetConfig), _VP], _VP),
    "hgnn_net_forward": ([ctypes.POINTER(NetConfig), ctypes.POINTER(NetInputs), _VP, _VP, _VP, _VP, _VP], _I),
    "hgnn_net_backward": ([ctypes.POINTER(NetConfig), ctypes.POINTER(NetInputs), _VP, _VP, _VP, _VP, _VP, _VP,
                           _VP], _I),
    "hgnn_graph_oper_forward": ([_VP, _VP, _VP, _I, _I, _I, _I, _VP], _I),
    "hgnn_graph_oper_backward": ([_VP, _VP, _VP, _VP, _VP, _I, _I, _I, _I, _VP], _I),
    "hgnn_p_multi_forward": ([_VP, _L, _L, _L, _VP, _VP, _I, _I, _I, _I, _VP], _I),
    "hgnn_p_multi_backward": ([_VP, _L, _L, _L, _VP, _VP, _VP, _VP, _I, _I, _I, _I, _VP], _I),
    "hgnn_bn_forward": ([_VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _I, _I, _I, _I, _VP], _I),
    "hgnn_bn_backward": ([_VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _I, _I, _I, _I, _VP], _I),
    "hgnn_timer_create": ([_I, ctypes.c_uint], _VP),
    "hgnn_timer_create_ex": ([_I, ctypes.c_uint, _I, ctypes.c_longlong], _VP),
    "hgnn_timer_reset": ([_VP], None),
    "hgnn_timer_elapsed": ([_VP, _I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I)], _I),
    "hgnn_timer_destroy": ([_VP], None),
    "hgnn_timer_launches": ([_VP, _I, ctypes.POINTER(_I), ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I)], _I),
    "hgnn_timer_waves": ([_VP, _I, ctypes.c_longlong, ctypes.POINTER(ctypes.c_double),
                          ctypes.POINTER(ctypes.c_double)], ctypes.c_longlong),
    "hgnn_net_forward_timed": ([ctypes.POINTER(NetConfig), ctypes.POINTER(NetInputs), _VP, _VP, _VP, _VP, _VP,
                                _VP], _I),
    "hgnn_net_backward_timed": ([ctypes.POINTER(NetConfig), ctypes.POINTER(NetInputs), _VP, _VP, _VP, _VP, _VP,
                                 _VP, _VP, _VP], _I),
    "hgnn_ccn_plan_bytes": ([ctypes.POINTER(CcnConfig), ctypes.c_longlong], ctypes.c_size_t),
    "hgnn_ccn_plan": ([ctypes.POINTER(CcnConfig), _VP, _VP, _VP, ctypes.c_longlong,
                       ctypes.POINTER(ctypes.c_longlong), _VP], _I),
    "hgnn_ccn_plan_async": ([ctypes.POINTER(CcnConfig), _VP, _VP, _VP, ctypes.c_longlong,
                             ctypes.POINTER(ctypes.c_longlong), _VP], _I),
    "hgnn_ccn_error_word": ([ctypes.POINTER(CcnConfig), _VP, ctypes.c_longlong], _VP),
    "hgnn_ccn_workspace_bytes": ([ctypes.POINTER(CcnConfig), ctypes.POINTER(ctypes.c_longlong)], ctypes.c_size_t),
    "hgnn_ccn_forward": ([ctypes.POINTER(CcnConfig), ctypes.POINTER(ctypes.c_longlong), _VP, _VP, _VP,
                          ctypes.c_longlong, _VP, _VP, _VP], _I),
    "hgnn_ccn_backward": ([ctypes.POINTER(CcnConfig), ctypes.POINTER(ctypes.c_longlong), _VP, _VP,
                           ctypes.c_longlong, _VP, _VP, _VP, _VP, _VP], _I),
    "hgnn_ccn_small_supported": ([ctypes.POINTER(CcnConfig)], _I),
    "hgnn_host_word_alloc": ([ctypes.POINTER(_VP), ctypes.POINTER(_VP)], _I),
    "hgnn_ccn_small_workspace_bytes": ([ctypes.POINTER(CcnConfig)], ctypes.c_size_t),
    "hgnn_ccn_small_forward": ([ctypes.POINTER(CcnConfig), _VP, _VP, _VP, _VP, _VP, _VP, _I, _VP, _VP], _I),
    "hgnn_ccn_small_backward": ([ctypes.POINTER(CcnConfig), _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP], _I),
    "hgnn_collapse6to3": ([_VP, _VP, _I, _I, _VP], _I),
    "hgnn_collapse6to3_backward": ([_VP, _VP, _I, _I, _VP], _I),
    "hgnn_ccn_plan_offsets": ([ctypes.POINTER(CcnConfig), ctypes.c_longlong, ctypes.POINTER(ctypes.c_size_t)], _I),
    "hgnn_graph_edge_slots": ([_I, _VP], _I),
    "hgnn_graph_operators": ([_I, _VP, _I, _I, _VP, _I, _VP, _VP, _VP], _I),
    "hgnn_csr_batch_plan": ([_I, _VP, _VP, _I, _I, _I, ctypes.POINTER(CsrLayout)], _I),
    "hgnn_csr_batch_build": ([_I, _VP, _VP, _VP, _I, _I, _I, ctypes.POINTER(CsrLayout), _VP], _I),
    "hgnn_csr_batch_view": ([ctypes.POINTER(CsrLayout), _VP, ctypes.POINTER(CsrBatch)], _I),
    "hgnn_net_backward_ex": ([ctypes.POINTER(NetConfig), ctypes.POINTER(NetInputs), ctypes.POINTER(CsrBatch), _VP, _VP,
                              _VP, _VP, _VP, _VP, _VP, _VP, _VP, _I], _I),
    "hgnn_net_forward_csr": ([ctypes.POINTER(NetConfig), ctypes.POINTER(CsrBatch), _VP, _VP, _VP, _VP, _VP], _I),
    "hgnn_net_backward_csr": ([ctypes.POINTER(NetConfig), ctypes.POINTER(CsrBatch), _VP, _VP, _VP, _VP, _VP,
                               _VP], _I),
    "hgnn_mse_loss": ([_VP, _VP, _I, ctypes.c_float, ctypes.c_float, _VP, _VP, _VP], _I),
    "hgnn_xent_loss": ([_VP, _VP, _I, _I, _VP, _VP, _VP, _VP], _I),
    "hgnn_adamax_step": ([_I, _VP, _VP, _VP, _VP, _VP, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                          ctypes.c_double, ctypes.c_double, ctypes.c_longlong, _VP], _I),
    "hgnn_conv1x1_workspace_bytes": ([_I, _I, _I, _I], ctypes.c_size_t),
    "hgnn_conv1x1_forward": ([_VP, _VP, _VP, _VP, _I, _I, _I, _I, _I, _VP, _VP], _I),
    "hgnn_conv1x1_backward": ([_VP, _VP, _VP, _VP, _VP, _VP, _I, _I, _I, _I, _VP, _VP], _I),
}


def lib():
    """Load (once) and return the shared library; raise if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"hgnn_amd: native library not found at {LIB_PATH}; build it with "
                "`make -C hgnn-2_amd` (or __graft_entry__.build()). There is no CPU fallback.")
        h = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = res
        _lib = h
    return _lib


def check(status, what):
    if status != HGNN_OK:
        raise RuntimeError(f"hgnn_amd: {what} failed: {STATUS.get(status, status)}")


def deverr_message(bits):
    msgs = [m for b, m in DEVERR.items() if bits & b]
    return "; ".join(msgs) if msgs else f"device error bits {bits:#x}"


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def ptr_array(tensors):
    arr = (ctypes.c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = None if t is None else t.data_ptr()
    return arr


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle(device):
    """The current HIP stream of `device` as a void* (torch's raw accessor: ~10 us less host time per call
    than building a torch.cuda.Stream object; the per-graph CCN step makes two such calls)."""
    if _raw_stream is not None:
        return ctypes.c_void_p(_raw_stream(device.index if device.index is not None else torch.cuda.current_device()))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
