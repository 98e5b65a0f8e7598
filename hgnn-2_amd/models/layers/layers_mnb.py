"""Drop-in for models/layers/layers_mnb.py of the reference.

Same classes, constructor signatures, submodule names, parameter shapes and
init (normal(0, 0.1) on every Conv1d weight and bias) as the reference, so
state_dicts and seeded initialisations carry over.  The layers used one at a
time run on the layer-level HIP ops (hgnn_amd.ops); GNN_lg / GNN_simple run
all layers through the fused network executor instead (models/gnns/model_mnb.py).

Reference line map: graph_oper 391-411, P_multi 414-434, layer_simple 25-69,
layer_last 72-95, layer_with_lg_1 157-225, layer_with_lg_2 228-290,
layer_with_lg_3 293-358, layer_last_lg 361-388.
"""

import torch
import torch.nn as nn

from hgnn_amd import ops
from models.layers.batch_normalization import BN
from models.layers.gru_update import GRUUpdate, Identity

if torch.cuda.is_available():
    dtype = torch.cuda.FloatTensor
else:
    dtype = torch.FloatTensor


def _mix(x1, lin, relu_conv, relu_lin=False):
    """cat(lin(x1) [ReLU if relu_lin], relu(relu_conv(x1))) -- the reference's two-Conv1d block."""
    a = ops.conv1x1(x1, lin.weight, lin.bias, relu=relu_lin)
    b = ops.conv1x1(x1, relu_conv.weight, relu_conv.bias, relu=True)
    return torch.cat((a, b), 1)


class layer_simple(nn.Module):
    """Layer of the simple GNN with ReLU non-linearity (reference lines 25-69)."""

    def __init__(self, feature_maps, J, gru):
        super(layer_simple, self).__init__()
        self.n_inputs = feature_maps[0]
        self.n_outputs = feature_maps[1]
        self.gop = graph_oper()
        self.cv1 = torch.nn.Conv1d(J * self.n_inputs, self.n_outputs, 1)
        self.cv2 = torch.nn.Conv1d(J * self.n_inputs, self.n_outputs, 1)
        if gru is True:
            self.update = GRUUpdate(self.n_inputs, 2 * self.n_outputs)
        else:
            self.update = Identity()
        self.bn1 = BN(2 * self.n_outputs)
        self._init_weights()

    def _init_weights(self, scale=0.1):
        for layer in [self.cv1, self.cv2]:
            layer.weight.data.normal_(0, scale)
            layer.bias.data.normal_(0, scale)

    def forward(self, state, N_batch, mask):
        X, W = state
        x1 = self.gop(W, X)
        zb1 = _mix(x1, self.cv2, self.cv1, relu_lin=True)  # both halves ReLU (reference 59-65)
        zbn1 = self.bn1(zb1, N_batch, mask)
        return (zbn1, W)


class layer_last(nn.Module):
    """Readout of the simple GNN (reference lines 72-95)."""

    def __init__(self, feature_maps, J):
        super(layer_last, self).__init__()
        self.n_inputs = feature_maps[0]
        self.n_outputs = feature_maps[1]
        self.gop = graph_oper()
        self.fc = torch.nn.Conv1d(J * self.n_inputs, self.n_outputs, 1)
        self._init_weights()

    def _init_weights(self, scale=0.1):
        self.fc.weight.data.normal_(0, scale)
        self.fc.bias.data.normal_(0, scale)

    def forward(self, state, N_batch, mask):
        X, W = state
        x1 = self.gop(W, X)
        y1 = ops.conv1x1(x1, self.fc.weight, self.fc.bias)
        y = torch.sum(y1, dim=2)
        return y.view(y.shape[0], self.n_outputs)


class _LgBase(nn.Module):
    def _init_weights(self, scale=0.1):
        for layer in [self.cv1, self.cv2, self.cv3, self.cv4]:
            layer.weight.data.normal_(0, scale)
            layer.bias.data.normal_(0, scale)

    def _node(self, X, XL_like, W, Pm, Pd, N_batch, mask):
        x1 = torch.cat((self.gop(W, X), self.pmul(Pm, XL_like), self.pmul(Pd, XL_like)), 1)
        return self.bn1(_mix(x1, self.cv2, self.cv1), N_batch, mask)

    def _edge(self, XL, X_like, WL, Pm, Pd, E_batch, mask_lg):
        xd1 = torch.cat((self.gop(WL, XL), self.pmul(Pm.transpose(2, 1), X_like),
                         self.pmul(Pd.transpose(2, 1), X_like)), 1)
        return self.bn2(_mix(xd1, self.cv4, self.cv3), E_batch, mask_lg)


class layer_with_lg_1(_LgBase):
    """Node half first; the edge half reads the normalised node output (reference 157-225)."""

    def __init__(self, feature_maps, J):
        super(layer_with_lg_1, self).__init__()
        self.n_inputs = feature_maps[0]
        self.n_edges = feature_maps[1]
        self.n_outputs = feature_maps[2]
        self.gop = graph_oper()
        self.pmul = P_multi()
        self.cv1 = torch.nn.Conv1d(J * self.n_inputs + 2 * self.n_edges, self.n_outputs, 1)
        self.cv2 = torch.nn.Conv1d(J * self.n_inputs + 2 * self.n_edges, self.n_outputs, 1)
        self.bn1 = BN(2 * self.n_outputs)
        self.cv3 = torch.nn.Conv1d(J * self.n_edges + 4 * self.n_outputs, self.n_outputs, 1)
        self.cv4 = torch.nn.Conv1d(J * self.n_edges + 4 * self.n_outputs, self.n_outputs, 1)
        self.bn2 = BN(2 * self.n_outputs)
        self._init_weights()

    def forward(self, state, N_batch, mask, E_batch, mask_lg):
        X, XL, W, WL, Pm, Pd = state
        zbn1 = self._node(X, XL, W, Pm, Pd, N_batch, mask)
        zdbn1 = self._edge(XL, zbn1, WL, Pm, Pd, E_batch, mask_lg)
        return (zbn1, zdbn1, W, WL, Pm, Pd)


class layer_with_lg_2(_LgBase):
    """Edge half first; the node half reads the normalised edge output (reference 228-290)."""

    def __init__(self, feature_maps, J):
        super(layer_with_lg_2, self).__init__()
        self.n_inputs = feature_maps[0]
        self.n_edges = feature_maps[1]
        self.n_outputs = feature_maps[2]
        self.gop = graph_oper()
        self.pmul = P_multi()
        self.cv1 = torch.nn.Conv1d(J * self.n_inputs + 4 * self.n_outputs, self.n_outputs, 1)
        self.cv2 = torch.nn.Conv1d(J * self.n_inputs + 4 * self.n_outputs, self.n_outputs, 1)
        self.bn1 = BN(2 * self.n_outputs)
        self.cv3 = torch.nn.Conv1d(J * self.n_edges + 2 * self.n_inputs, self.n_outputs, 1)
        self.cv4 = torch.nn.Conv1d(J * self.n_edges + 2 * self.n_inputs, self.n_outputs, 1)
        self.bn2 = BN(2 * self.n_outputs)
        self._init_weights()

    def forward(self, state, N_batch, mask, E_batch, mask_lg):
        X, XL, W, WL, Pm, Pd = state
        zdbn1 = self._edge(XL, X, WL, Pm, Pd, E_batch, mask_lg)
        zbn1 = self._node(X, zdbn1, W, Pm, Pd, N_batch, mask)
        return (zbn1, zdbn1, W, WL, Pm, Pd)


class layer_with_lg_3(_LgBase):
    """Independent node and edge halves (reference 293-358)."""

    def __init__(self, feature_maps, J):
        super(layer_with_lg_3, self).__init__()
        self.n_inputs = feature_maps[0]
        self.n_edges = feature_maps[1]
        self.n_outputs = feature_maps[2]
        self.gop = graph_oper()
        self.pmul = P_multi()
        self.cv1 = torch.nn.Conv1d(J * self.n_inputs + 2 * self.n_edges, self.n_outputs, 1)
        self.cv2 = torch.nn.Conv1d(J * self.n_inputs + 2 * self.n_edges, self.n_outputs, 1)
        self.bn1 = BN(2 * self.n_outputs)
        self.cv3 = torch.nn.Conv1d(J * self.n_edges + 2 * self.n_inputs, self.n_outputs, 1)
        self.cv4 = torch.nn.Conv1d(J * self.n_edges + 2 * self.n_inputs, self.n_outputs, 1)
        self.bn2 = BN(2 * self.n_outputs)
        self._init_weights()

    def forward(self, state, N_batch, mask, E_batch, mask_lg):
        X, XL, W, WL, Pm, Pd = state
        zbn1 = self._node(X, XL, W, Pm, Pd, N_batch, mask)
        zdbn1 = self._edge(XL, X, WL, Pm, Pd, E_batch, mask_lg)
        return (zbn1, zdbn1, W, WL, Pm, Pd)


class layer_last_lg(nn.Module):
    """Readout of the line-graph GNN (reference 361-388)."""

    def __init__(self, feature_maps, J):
        super(layer_last_lg, self).__init__()
        self.n_inputs = feature_maps[0]
        self.n_outputs = feature_maps[1]
        self.gop = graph_oper()
        self.pmul = P_multi()
        self.fc = torch.nn.Conv1d((J + 2) * self.n_inputs, self.n_outputs, 1)
        self._init_weights()

    def _init_weights(self, scale=0.1):
        self.fc.weight.data.normal_(0, scale)
        self.fc.bias.data.normal_(0, scale)

    def forward(self, state, N_batch, mask):
        X, XL, W, WL, Pm, Pd = state
        x1 = torch.cat((self.gop(W, X), self.pmul(Pm, XL), self.pmul(Pd, XL)), 1)
        y1 = ops.conv1x1(x1, self.fc.weight, self.fc.bias)
        y = torch.sum(y1, dim=2)
        return y.view(y.shape[0], self.n_outputs)


class graph_oper(nn.Module):
    """out[b, j*F + f, n] = sum_m A[b, n, m, j] X[b, f, m] (reference 391-411)."""

    def forward(self, A, X):
        return ops.graph_oper(A, X)


class P_multi(nn.Module):
    """out[b, f, n] = sum_m P[b, n, m] X[b, f, m] (reference 414-434)."""

    def forward(self, P, X):
        return ops.p_multi(P, X)
