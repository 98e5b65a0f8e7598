"""Drop-in for models/layers/batch_normalization.py of the reference.

BN keeps the reference's semantics (batch_normalization.py:23-108): SCALAR
affine parameters, masked statistics over the real positions of the whole
batch (sum over (b, n) / sum(N_batch)), var = 1e-5 + masked mean of squared
deviations, std = sqrt(var), running statistics with the reversed momentum
(running = 0.9 * batch + 0.1 * running) held as plain attributes (not
buffers, not in the state_dict).  Compute runs in the HIP kernels of
hgnn-2_amd/csrc/dense_ops.hip; inside GNN_lg / GNN_simple the same math is
fused into the network executor instead.
"""

import torch
import torch.nn as nn

from hgnn_amd import ops

if torch.cuda.is_available():
    dtype = torch.cuda.FloatTensor
else:
    dtype = torch.FloatTensor


def _default_device():
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


class BN(nn.Module):
    def __init__(self, n_features, scale=0.1):
        super(BN, self).__init__()
        # 0-dim parameters, same construction and RNG order as the reference (lines 26-29)
        self.weight = nn.Parameter(torch.tensor(n_features).type(torch.FloatTensor))
        self.bias = nn.Parameter(torch.tensor(n_features).type(torch.FloatTensor))
        torch.nn.init.normal_(self.weight, 0, scale)
        torch.nn.init.normal_(self.bias, 0, scale)
        self.running_mean = torch.zeros(n_features, device=_default_device())
        self.running_std = torch.zeros(n_features, device=_default_device())
        self.momentum = 0.1

    def __setstate__(self, state):
        # whole-module checkpoints of the reference (torch.save(model), functions/logs.py:99-111)
        # pickle the running statistics with their autograd history attached: keep the values only
        super(BN, self).__setstate__(state)
        for n in ("running_mean", "running_std"):
            v = self.__dict__.get(n)
            if torch.is_tensor(v):
                self.__dict__[n] = v.detach()

    def _apply(self, fn, *args, **kwargs):
        super(BN, self)._apply(fn, *args, **kwargs)
        self.running_mean = fn(self.running_mean)
        self.running_std = fn(self.running_std)
        return self

    def running_on(self, device):
        """Running statistics as contiguous float32 tensors on `device` (rebinding if needed)."""
        if self.running_mean.device != device or self.running_mean.dtype != torch.float32:
            self.running_mean = self.running_mean.to(device=device, dtype=torch.float32).contiguous()
        if self.running_std.device != device or self.running_std.dtype != torch.float32:
            self.running_std = self.running_std.to(device=device, dtype=torch.float32).contiguous()
        return self.running_mean, self.running_std

    def forward(self, X, N_batch, mask):
        if self.training:
            out, mean, std = ops.bn(X, N_batch, mask, self.weight, self.bias, None, None)
            rm, rs = self.running_on(X.device)
            m = self.momentum
            self.running_mean = (1 - m) * mean + m * rm
            self.running_std = (1 - m) * std + m * rs
            return out
        rm, rs = self.running_on(X.device)
        out, _, _ = ops.bn(X, N_batch, mask, self.weight, self.bias, rm, rs)
        return out


class spatial_batch_norm(nn.Module):
    """Unused by the reference's models (batch_normalization.py:45-62); kept for import parity."""

    def __init__(self, n_feat):
        super(spatial_batch_norm, self).__init__()
        self.n_feat = n_feat
        self.layer = torch.nn.Conv1d(n_feat, n_feat, 1)

    def forward(self, X, N_batch, mask, mean=None, std=None):
        X_norm, _, _ = sb_normalization(X, N_batch, mask, mean, std)
        return ops.conv1x1(X_norm, self.layer.weight, self.layer.bias)


def sb_normalization(H, N_batch, mask, mean=None, std=None):
    """(H - mean) / std over masked positions; batch statistics unless mean/std given (lines 65-77)."""
    one = torch.ones((), device=H.device, dtype=torch.float32)
    zero = torch.zeros((), device=H.device, dtype=torch.float32)
    if not torch.is_tensor(mean) or not torch.is_tensor(std):
        out, mean, std = ops.bn(H, N_batch, mask, one, zero, None, None)
    else:
        out, mean, std = ops.bn(H, N_batch, mask, one, zero, mean, std)
    return out, mean, std


def mean_with_padding(tensor, N_batch, mask):
    """sum over (b, n) of the masked tensor / sum(N_batch) -> (n_features,) (lines 80-93)."""
    return ops.masked_mean(tensor, N_batch, mask)


def mask_embedding(H, mask):
    """H * mask[:, :, 0] broadcast over features (lines 96-108)."""
    return ops.mask_rows(H, mask)
