"""Drop-in for functions/contraction.py of the reference.

collapse6to3(F) (reference lines 106-121) maps F (C, n, n, n, n, n) to
(n, n, 18 C) with contraction q in channels [q C, (q+1) C): five plain
collapses (_c6to2_111, lines 44-61), ten "contract two indices, sum one"
(_c6to2_12, 64-85) and three triple diagonals (_c6to2_3, 88-103).  It runs as
one gfx950 kernel per direction (hgnn_collapse6to3 / _backward); the CCN
models never call it -- their executor uses the closed form for T (x) I
 -- it is kept for code that contracts general 6-D tensors.

collapse_cube / filter_diag_cube are the reference's small tensor helpers
(lines 21-41), restated with torch ops.
"""

import torch

from hgnn_amd.ccn import collapse6to3  # noqa: F401


def collapse_cube(F):
    """Sum the 2nd..4th of the last five axes (reference lines 21-26)."""
    d = F.dim()
    return F.sum(dim=(d - 4, d - 3, d - 2))


def filter_diag_cube(F, planar_diag=True, cudaflag=False):
    """Zero all but the diagonal of the last two (planar) or three spatial axes (reference lines 29-41)."""
    n = F.shape[1]
    eye = torch.eye(n, dtype=F.dtype, device=F.device)
    if not planar_diag:
        eye = (eye.unsqueeze(2) * eye).unsqueeze(3)
    else:
        eye = eye.unsqueeze(2)
    return F * eye
