"""Drop-in for functions/utils_ccn.py of the reference (CompnetUtils).

The CCN models of this package do not go through these per-node lists: their
forward runs the batched device executor (hgnn_amd.ccn).  CompnetUtils keeps
the reference's method surface (lines 28-324) for code that builds its own
compnet from the pieces, restated with tensor ops on the input's device:
receptive fields are index vectors, chi matrices are built from position maps
and promotions are gathers instead of chi @ F @ chi^T products.  outer_contract
is the gfx950 collapse6to3 (so, like every product path here, it needs the GPU).

Semantics kept from the reference: deg_i counts A[i] > 0 (line 159), the
receptive field is nonzero(A[i]) in ascending order (161-163), chi_ij[k, p] = 1
iff nbr_i[k] == nbr_j[p] (66-84), F0 tiles X[i] (167-172, 212-216), and the
2-D update is relu(W(collapse6to3(T_i (x) chi_ii))) (281-300).
"""

import torch
import torch.nn.functional as Func

from functions.contraction import collapse6to3


class CompnetUtils():

    def __init__(self, cudaflag=False):
        self.cudaflag = cudaflag

        def python_contract(T, adj):
            # T (n, n, n, C), adj (n, n) -> collapse6to3(T (x) adj) (reference lines 37-45)
            return collapse6to3(self.tensorprod(T.permute(3, 0, 1, 2), adj).contiguous())

        self.outer_contract = python_contract

    def tensorprod(self, T, A):
        d1 = T.dim()
        for i in range(A.dim()):
            T = torch.unsqueeze(T, d1 + i)
        return T * A

    # ---------------------------------------------------------------- receptive fields
    def _fields(self, A):
        self.A = A
        self.deg = torch.sum(A > 0.0, dim=1)
        self.neighbors = [torch.nonzero(A[i, :]).flatten()[:int(self.deg[i])] for i in range(A.shape[0])]

    def _position(self, i, j):
        """p[k] = index of nbr_i[k] in nbr_j, or -1."""
        ni, nj = self.neighbors[i], self.neighbors[j]
        eq = ni.unsqueeze(1) == nj.unsqueeze(0)
        return torch.where(eq.any(1), eq.int().argmax(1), torch.full_like(ni, -1))

    def _get_chi(self, i, j):
        ni, nj = self.neighbors[i], self.neighbors[j]
        return (ni.unsqueeze(1) == nj.unsqueeze(0)).to(torch.float32)

    def _get_chi_root(self, i):
        n = self.A.shape[0]
        chi = torch.zeros(n, int(self.deg[i]), dtype=torch.float32, device=self.A.device)
        chi[self.neighbors[i], torch.arange(int(self.deg[i]), device=self.A.device)] = 1
        return chi

    def _register_chis(self, A):
        n = A.shape[0]
        self.chis = []
        for i in range(n):
            row = [self._get_chi(i, j) if A[i][j] > 0 else None for j in range(n)]
            row.append(self._get_chi_root(i))
            self.chis.append(row)
        return self.chis

    def get_F0(self, X, A):
        self._fields(A)
        self._register_chis(A)
        return [X[i].view(1, 1, -1).expand(int(d), int(d), X.shape[1]).contiguous() for i, d in enumerate(self.deg)]

    def get_F0_1D(self, X, A):
        self._fields(A)
        self._register_chis(A)
        return [X[i].view(1, -1).expand(int(d), X.shape[1]).contiguous() for i, d in enumerate(self.deg)]

    # ---------------------------------------------------------------- promotions
    def _promote(self, F_prev, i, j):
        p = self._position(i, j)
        ok = (p >= 0).to(F_prev[j].dtype)
        q = p.clamp(min=0)
        G = F_prev[j][q][:, q]
        return G * (ok.view(-1, 1, 1) * ok.view(1, -1, 1))

    def _promote_1D(self, F_prev, i, j):
        p = self._position(i, j)
        ok = (p >= 0).to(F_prev[j].dtype)
        return F_prev[j][p.clamp(min=0)] * ok.view(-1, 1)

    def get_nbr_promotions(self, F_prev, i):
        return torch.stack([self._promote(F_prev, i, int(j)) for j in self.neighbors[i]], 0)

    def get_nbr_promotions_1D(self, F_prev, i):
        return torch.stack([self._promote_1D(F_prev, i, int(j)) for j in self.neighbors[i]], 0)

    # ---------------------------------------------------------------- updates
    def update_F(self, F_prev, W):
        assert len(F_prev) == self.A.shape[0]
        return [Func.relu(W(self.outer_contract(self.get_nbr_promotions(F_prev, i), self.chis[i][i])))
                for i in range(len(F_prev))]

    def update_F_1D(self, F_prev, W):
        out = []
        for i in range(len(F_prev)):
            T = self.get_nbr_promotions_1D(F_prev, i)
            out.append(Func.relu(W(torch.cat([T.sum(0), T.sum(1)], 1))))
        return out
