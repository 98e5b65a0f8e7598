"""hgnn_amd -- MI355X (gfx950) runtime behind the drop-in HGNN modules.

Layout of the drop-in tree (put this directory on sys.path, as the reference's
drivers put their repo root, scripts/main_gnn_qm9.py:22):

    functions/   operators.py, batching.py, utils.py, contraction.py, utils_ccn.py
    models/      layers/{layers_mnb, batch_normalization, gru_update}.py,
                 gnns/model_mnb.py, compnets/model_ccn.py
    hgnn_amd/    this package: ctypes binding of include/hgnn_amd.h, autograd
                 wrappers, synthetic data generators
    csrc/        HIP kernels for gfx950 and the C ABI implementation
"""

from ._lib import LIB_PATH, lib  # noqa: F401
from .net import check_errors  # noqa: F401

__all__ = ["lib", "LIB_PATH", "check_errors"]
