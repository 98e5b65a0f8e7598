"""Drop-in for models/gnns/model_mnb.py of the reference.

GNN_simple (reference lines 19-66) and GNN_lg (69-129) keep the reference's
constructor signatures, attributes (.dual, .J, .n_features, .n_layers,
.n_outputs, .order), submodule names (layer0, layer1.., layerlast) and
parameter shapes, so `scripts/main_gnn_qm9.py` / `scripts/train_mnb.py`
(which read model.dual and model.J, scripts/train_mnb.py:29-30) and saved
state_dicts work unchanged.

forward() runs the whole network -- every layer, BN and the readout -- as one
enqueue of gfx950 kernels (hgnn_amd.net -> hgnn_net_forward) and backward as
another (hgnn_net_backward).  Running BN statistics are updated in place in
training mode exactly as the reference rebinds them.
"""

import torch
import torch.nn as nn

import os

from hgnn_amd.dp import attached
from hgnn_amd.library import run_net_ops
from hgnn_amd.net import NetSpec, run_net, run_net_csr


def use_torch_ops():
    """The registered torch.library operators (hgnn_amd.library) while torch.compile traces the
    module, or always with HGNN_TORCH_OPS=1; the autograd.Function path otherwise."""
    return os.environ.get("HGNN_TORCH_OPS") == "1" or torch.compiler.is_compiling()
from models.layers import layers_mnb


# The parameters in ABI order, read through the modules' _modules / _parameters dicts: the attribute path
# (nn.Module.__getattr__, two per parameter) cost ~130 us of host time per forward at config 2; a name that
# is not a registered submodule / parameter falls back to it
def _sub(mod, name):
    m = mod._modules.get(name)
    return m if m is not None else getattr(mod, name)


def _param(mod, name):
    p = mod._parameters.get(name)
    return p if p is not None else getattr(mod, name)


def _pair(mod, name):
    m = _sub(mod, name)
    return [_param(m, "weight"), _param(m, "bias")]


def _lg_params(layer):
    return (_pair(layer, "cv1") + _pair(layer, "cv2") + _pair(layer, "bn1") + _pair(layer, "cv3") + _pair(layer, "cv4") +
            _pair(layer, "bn2"))


def _simple_params(layer):
    return _pair(layer, "cv1") + _pair(layer, "cv2") + _pair(layer, "bn1")


class GNN_simple(nn.Module):
    """Power GNN (Community Detection with Hierarchical GNN); reference lines 19-66."""

    def __init__(self, task, n_features, n_layers, dim_input, dim_output=1, J=1, gru=False):
        super(GNN_simple, self).__init__()
        self.dual = False
        self.J = J
        self.gru = False
        self.n_features = n_features
        self.n_layers = n_layers
        self.n_outputs = dim_output
        self.featuremap_in = [dim_input, n_features]
        self.featuremap_mi = [2 * n_features, n_features]
        self.featuremap_end = [2 * n_features, dim_output]
        self.layer0 = layers_mnb.layer_simple(self.featuremap_in, J + 2, gru)
        for i in range(n_layers - 2):
            module = layers_mnb.layer_simple(self.featuremap_mi, J + 2, gru)
            self.add_module('layer{}'.format(i + 1), module)
        self.layerlast = layers_mnb.layer_last(self.featuremap_end, J + 2)

    def _layers(self):
        return [self.layer0] + [self._modules['layer{}'.format(i + 1)] for i in range(self.n_layers - 2)]

    def _spec(self, device):
        params, running = [], []
        for layer in self._layers():
            params += _simple_params(layer)
            running += list(layer.bn1.running_on(device))
        params += [self.layerlast.fc.weight, self.layerlast.fc.bias]
        return NetSpec(kind=0, order=0, d=self.n_features, n_layers=self.n_layers, dim_out=self.n_outputs,
                       params=params, running=running, training=self.training, dp=attached(self))

    def forward(self, state, N_batch, mask):
        X, W = state
        if use_torch_ops():
            return run_net_ops(self._spec(X.device), X, W, N_batch, mask)
        return run_net(self._spec(X.device), X, W, N_batch, mask)

    def forward_csr(self, batch):
        """Same network on a hgnn_amd.csr.CsrBatch (native batcher, no dense operators)."""
        return run_net_csr(self._spec(batch.device), batch)


class GNN_lg(nn.Module):
    """GNN on the line graph with non-backtracking operator; reference lines 69-129."""

    def __init__(self, task, n_features, n_layers, dim_input, dim_output=1, J=1, order=1):
        super(GNN_lg, self).__init__()
        self.dual = True
        self.J = J
        self.n_features = n_features
        self.n_layers = n_layers
        self.n_outputs = dim_output
        self.order = order
        self.featuremap_in = [dim_input, 1, n_features]
        self.featuremap_mi = [2 * n_features, 2 * n_features, n_features]
        self.featuremap_end = [2 * n_features, dim_output]
        if order == 1:
            cls = layers_mnb.layer_with_lg_1
        elif order == 2:
            cls = layers_mnb.layer_with_lg_2
        else:
            cls = layers_mnb.layer_with_lg_3
        self.layer0 = cls(self.featuremap_in, J + 2)
        for i in range(n_layers - 2):
            module = cls(self.featuremap_mi, J + 2)
            self.add_module('layer{}'.format(i + 1), module)
        self.layerlast = layers_mnb.layer_last_lg(self.featuremap_end, J + 2)

    def _layers(self):
        return [self.layer0] + [self._modules['layer{}'.format(i + 1)] for i in range(self.n_layers - 2)]

    def _spec(self, device):
        params, running = [], []
        for layer in self._layers():
            params += _lg_params(layer)
            running += list(layer.bn1.running_on(device)) + list(layer.bn2.running_on(device))
        params += [self.layerlast.fc.weight, self.layerlast.fc.bias]
        order = self.order if self.order in (1, 2) else 3
        return NetSpec(kind=1, order=order, d=self.n_features, n_layers=self.n_layers, dim_out=self.n_outputs,
                       params=params, running=running, training=self.training, dp=attached(self))

    def forward(self, state, N_batch, mask, E_batch, mask_lg):
        X, XL, W, WL, Pm, Pd = state
        if use_torch_ops():
            return run_net_ops(self._spec(X.device), X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg)
        return run_net(self._spec(X.device), X, W, N_batch, mask, XL, WL, Pm, Pd, E_batch, mask_lg)

    def forward_csr(self, batch):
        """Same network on a hgnn_amd.csr.CsrBatch (native batcher, no dense operators)."""
        return run_net_csr(self._spec(batch.device), batch)
