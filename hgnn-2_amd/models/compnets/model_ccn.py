"""Drop-in for models/compnets/model_ccn.py of the reference.

CCN_1D (reference lines 18-64) and CCN_2D (67-105) keep the constructor
signatures, attributes (.input_feats, .n_outputs, .hidden_size,
.num_contractions, .layers, .utils), submodule names (w1..wL, fc), parameter
shapes and the reference's initialisation (1D: normal(0, 0.1) weights and
biases, lines 35-39; 2D: normal(0, 0.1) w weights with default-init biases
and fc.weight drawn twice, finally normal(0, 0.5), lines 86-91), in the same
RNG order, so seeded runs and saved state_dicts carry over.

forward(X (n, f), adj (n, n) with self loops) -> (n_outputs,) as in the
reference; forward_batch(X (bs, nmax, f), adj (bs, nmax, nmax), n_batch)
-> (bs, n_outputs) runs a padded batch of graphs in one executor call
(hgnn_amd.ccn -> hgnn_ccn_forward / hgnn_ccn_backward).
"""

import torch.nn as nn

from functions.utils_ccn import CompnetUtils
from hgnn_amd.ccn import CcnPlan, CcnSpec, run_ccn


class _CCN(nn.Module):
    order = 1

    def _params(self):
        ps = []
        for i in range(self.layers):
            w = self._modules['w{}'.format(i + 1)]
            ps += [w.weight, w.bias]
        return ps + [self.fc.weight, self.fc.bias]

    def _spec(self):
        key = (self.order, self.input_feats, self.w1.out_features, self.layers, self.n_outputs)
        sp = self.__dict__.get("_spec_cache")
        if sp is None or sp[0] != key:  # kept: it caches the batch configurations of the native calls
            sp = (key, CcnSpec(*key))
            self.__dict__["_spec_cache"] = sp
        return sp[1]

    def plan(self, adj, n_batch):
        """Index construction of a padded batch, reusable across forward_batch calls on it
        (hgnn_amd.ccn.CcnPlan; lets the step be captured in a HIP graph)."""
        return CcnPlan(self._spec(), adj, n_batch)

    def forward_batch(self, X, adj, n_batch, plan=None):
        return run_ccn(self._spec(), self._params(), X, adj, n_batch, plan)

    def forward(self, X, adj):
        if X.dim() != 2 or adj.dim() != 2:
            raise RuntimeError(f"hgnn_amd: CCN forward expects X (n, f) and adj (n, n), got {tuple(X.shape)}, "
                               f"{tuple(adj.shape)}")
        # one graph of n = nmax nodes: no n_batch tensor (run_ccn makes one only for the general path)
        return self.forward_batch(X.unsqueeze(0), adj.unsqueeze(0), None).view(self.n_outputs)


class CCN_1D(_CCN):
    order = 1

    def __init__(self, input_feats, n_outputs=1, hidden_size=2, layers=2, cudaflag=False):
        super(CCN_1D, self).__init__()
        self.input_feats = input_feats
        self.n_outputs = n_outputs
        self.hidden_size = hidden_size
        self.num_contractions = 2
        self.layers = layers
        self.utils = CompnetUtils(cudaflag)
        self.w1 = nn.Linear(input_feats * self.num_contractions, hidden_size)
        for i in range(layers - 1):
            self.add_module('w{}'.format(i + 2), nn.Linear(hidden_size * self.num_contractions, hidden_size))
        self.fc = nn.Linear(self.layers * hidden_size + input_feats, self.n_outputs)
        self._init_weights()

    def _init_weights(self, scale=0.1):
        for l in [self._modules['w{}'.format(i + 1)] for i in range(self.layers)] + [self.fc]:
            l.weight.data.normal_(0, scale)
            l.bias.data.normal_(0, scale)


class CCN_2D(_CCN):
    order = 2

    def __init__(self, input_feats=2, n_outputs=1, hidden_size=2, layers=2, cudaflag=True):
        super(CCN_2D, self).__init__()
        self.input_feats = input_feats
        self.n_outputs = n_outputs
        self.hidden_size = 2  # the reference pins the attribute (line 73); the Linears use the argument
        self.num_contractions = 18
        self.layers = layers
        self.cudaflag = cudaflag
        self.utils = CompnetUtils(cudaflag)
        self.w1 = nn.Linear(input_feats * self.num_contractions, hidden_size)
        for i in range(layers - 1):
            self.add_module('w{}'.format(i + 2), nn.Linear(hidden_size * self.num_contractions, hidden_size))
        self.fc = nn.Linear(self.layers * hidden_size + input_feats, self.n_outputs)
        self._init_weights()

    def _init_weights(self, scale=0.1):
        for l in [self._modules['w{}'.format(i + 1)] for i in range(self.layers)]:
            l.weight.data.normal_(0, scale)
        self.fc.weight.data.normal_(0, scale)
        self.fc.weight.data.normal_(0, scale * 5)
