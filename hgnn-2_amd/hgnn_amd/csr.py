"""Sparse ("CSR") batches: prepare_batch straight into the executor's layout.

The reference pads every graph's dense operators into (bs, Nmax, Nmax, J+2),
(bs, Emax, Emax, J+2) and (bs, Nmax, Emax) tensors (functions/batching.py:77-185),
which the executor then re-extracts into row lists on the device.  A CsrBatch
is built by the native batcher (csrc/builder.cpp, hgnn_csr_batch_plan/_build)
from the graphs themselves: the packed operator row lists, packed X / XL and the
batch offsets in one host image (~11 KB per QM9-shape graph instead of ~85 KB of
dense operators), copied to the device once.  The executor runs on it with no
plan / extraction pass (hgnn_net_forward_csr / _backward_csr).

Same numbers as the dense path: the lists hold exactly the entries the device
extraction finds, in the same (ascending column) order.
"""

import ctypes

import numpy as np
import torch

from . import _lib as L


class CsrBatch:
    """A batch of graphs in the executor's packed sparse layout, resident on one device.

    Attributes: bs, nmax, emax, f_in, j_tot, dual, nodes, edges, T (bs, 1) targets
    (or None), x (nodes, f_in) packed node features (a view into the image),
    N_batch / E_batch (bs,) int64 (views), layout (hgnn_csr_layout).
    """

    def __init__(self, graphs, J=1, dual=True, targets=None, device="cuda", pin=True):
        """graphs: list of (X (n, f), A (n, n)) CPU tensors (the first members of the
        reference's instances); targets: optional (bs,) or (bs, 1) tensor."""
        lib = L.lib()
        bs = len(graphs)
        if bs == 0:
            raise RuntimeError("hgnn_amd: empty batch")
        f_in = graphs[0][0].shape[1]
        xs, As = [], []
        for X, A in graphs:
            n = X.shape[0]
            if X.dim() != 2 or X.shape[1] != f_in or tuple(A.shape) != (n, n):
                raise RuntimeError(f"hgnn_amd: CsrBatch: graph shapes X {tuple(X.shape)}, A {tuple(A.shape)}")
            xs.append(X.detach().to("cpu", torch.float32).contiguous())
            As.append(A.detach().to("cpu", torch.float32).contiguous())
        n_nodes = (ctypes.c_int * bs)(*[x.shape[0] for x in xs])
        a_ptrs = (ctypes.c_void_p * bs)(*[a.data_ptr() for a in As])
        x_ptrs = (ctypes.c_void_p * bs)(*[x.data_ptr() for x in xs])
        lay = L.CsrLayout()
        st = lib.hgnn_csr_batch_plan(bs, n_nodes, a_ptrs, f_in, J, 1 if dual else 0, ctypes.byref(lay))
        if st == 4:
            raise IndexError("hgnn_amd: a graph's edge-slot construction writes past nnz(A) "
                             "(the reference's graph_operators raises IndexError)")
        L.check(st, "csr batch plan")
        host = torch.empty(int(lay.bytes), dtype=torch.uint8, pin_memory=pin and torch.cuda.is_available())
        L.check(lib.hgnn_csr_batch_build(bs, n_nodes, a_ptrs, x_ptrs, f_in, J, 1 if dual else 0, ctypes.byref(lay),
                                         ctypes.c_void_p(host.data_ptr())), "csr batch build")
        self.layout = lay
        self.host = host
        self.image = host.to(device, non_blocking=True) if str(device) != "cpu" else host
        self.bs, self.nmax, self.emax = bs, int(lay.nmax), int(lay.emax)
        self.f_in, self.j_tot, self.dual = f_in, int(lay.j_tot), bool(dual)
        self.nodes, self.edges = int(lay.nodes), int(lay.edges)
        self.view = L.CsrBatch()
        L.check(lib.hgnn_csr_batch_view(ctypes.byref(lay), ctypes.c_void_p(self.image.data_ptr()),
                                        ctypes.byref(self.view)), "csr batch view")
        self.x = self._f32(lay.off_x, self.nodes * f_in).view(self.nodes, f_in)
        self.N_batch = self._i64(lay.off_n_batch, bs)
        self.E_batch = self._i64(lay.off_e_batch, bs)
        self.T = None
        if targets is not None:
            self.T = torch.as_tensor(targets, dtype=torch.float32).reshape(bs, 1).to(self.image.device)

    def _f32(self, off, n):
        return self.image[off:off + 4 * n].view(torch.float32)

    def _i64(self, off, n):
        return self.image[off:off + 8 * n].view(torch.int64)

    @property
    def device(self):
        return self.image.device

    def lists(self):
        """Host copies of the six row-list kinds (W, WT, WL, WLT, PN, PE) as
        (rows (R, 2) int32 [start, count], entries (nnz, stride) float32), for tests."""
        out = []
        h = self.host.numpy()
        lay = self.layout
        for k in range(6):
            r = int(lay.rows[k])
            stride = 4 if k >= 4 else int(lay.stride_w)
            rows = np.frombuffer(h, dtype=np.int32, count=2 * r, offset=int(lay.off_rows[k])).reshape(r, 2)
            nz = int(lay.nnz[k])
            ent = np.frombuffer(h, dtype=np.float32, count=nz * stride, offset=int(lay.off_entries[k]))
            out.append((rows, ent.reshape(nz, stride)))
        return out


def prepare_batch_csr(batch, task, J=1, device="cuda"):
    """Native counterpart of prepare_batch (functions/batching.py:77-185) for the executor:
    batch = reference instances [x, A, t, ...] (only x, A, t are read); targets t[task]."""
    graphs = [(inst[0], inst[1]) for inst in batch]
    T = torch.tensor([float(inst[2][task]) for inst in batch], dtype=torch.float32)
    return CsrBatch(graphs, J=J, dual=True, targets=T, device=device)
