"""Drop-in for models/layers/gru_update.py of the reference.

GRUUpdate is constructed by layer_simple when gru=True (layers_mnb.py:38-41)
but never called in any forward (out of the hot path).  It is
kept as a parameter container so state_dicts and seeded initialisation order
match the reference.
"""

import torch
import torch.nn as nn


class GRUUpdate(nn.Module):
    def __init__(self, fmap_in, fmap_out):
        super(GRUUpdate, self).__init__()
        self.ih = nn.Linear(fmap_in, 3 * fmap_out)
        self.hh = nn.Linear(fmap_out, 3 * fmap_out)

    def forward(self, i, h):
        r_i, z_i, n_i = self.ih(i).chunk(3, -1)
        r_h, z_h, n_h = self.hh(h).chunk(3, -1)
        r = torch.sigmoid(r_i + r_h)
        z = torch.sigmoid(z_i + z_h)
        n = torch.tanh(n_i + r * n_h)
        return (1 - z) * n + z * h


class Identity(nn.Module):
    def forward(self, emb_in, emb_update):
        return emb_update
