"""Drop-in for functions/utils.py of the reference.

graph_op / Pmul (reference lines 24-81) are exact duplicates of graph_oper /
P_multi and run on the same HIP kernels; the rest (target normalisation,
MAE, meters) is host-side bookkeeping of the training loop, restated with the
reference's semantics (lines 84-146), e.g. normalize_data only subtracts the
mean when std < 1e-5 (Q14).
"""

import torch

from hgnn_amd import ops

cuda = True
if torch.cuda.is_available() and cuda:
    dtype = torch.cuda.FloatTensor
else:
    dtype = torch.FloatTensor


def graph_op(A, X):
    """(bs, N, N, J) x (bs, F, N) -> (bs, J*F, N)."""
    return ops.graph_oper(A, X)


def Pmul(P, X):
    """(bs, N, M) x (bs, F, M) -> (bs, F, N)."""
    return ops.p_multi(P, X)


def normalize_data(data, mean=None, std=None):
    if mean is None or std is None:
        _, _, mean, std = data_stats(data)
    if std < 10 ** -5:
        return data - mean
    return (data - mean) / std


def evaluation(pred, target):
    return torch.mean(torch.abs(pred - target))


def data_stats(data):
    minimum = torch.min(data)
    maximum = torch.max(data)
    mean = torch.mean(data)
    std = 10 ** -5 + torch.std(data)
    return minimum.item(), maximum.item(), mean.item(), std.item()


class AverageMeter():
    """Computes and stores the average and current value."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


class RunningAverage():
    """Running average with momentum: val <- (1 - m) * new + m * val, first value taken as is."""

    def __init__(self, momentum=0.1):
        self.momentum = momentum
        self.val = 0.0

    def update(self, val):
        if self.val == 0.0:
            self.val = val
        else:
            self.val = (1 - self.momentum) * val + self.momentum * self.val
