"""CPU oracle: restatement of the reference ``code/models/MDMIL.py`` (MDMIL :60-114).

TEST INFRASTRUCTURE ONLY.  Only ``tests/`` may import this module.

MDMIL is TransMIL with ``_fc1 = Linear(1024, 512) + GELU`` (:66), the head named
``_fc2`` (:73) and ``forward(x) -> (logits, attn2)`` (:114).  Its TransLayer and PPEG
(:19-57) equal TransMIL's, so the oracle's are reused.  Differences from the reference
source, none of which change arithmetic: the class token is moved to the input's device
instead of ``.cuda()`` (:91).  Pinned by ``tests/golden/mdmil_n300.npz``
(``tests/golden/make_golden_branches.py`` imports ``code/models/MDMIL.py``).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .transmil_ref import PPEG, TransLayer


class MDMIL(nn.Module):
    def __init__(self, n_classes):
        super().__init__()
        in_features, out_features = 1024, 512                            # :63-64
        self.pos_layer = PPEG(dim=out_features)                           # :65
        self._fc1 = nn.Sequential(nn.Linear(in_features, out_features), nn.GELU())   # :66
        self.cls_token = nn.Parameter(torch.randn(1, 1, out_features))   # :68
        self.n_classes = n_classes
        self.layer1 = TransLayer(dim=out_features)                       # :70-71
        self.layer2 = TransLayer(dim=out_features)
        self.norm = nn.LayerNorm(out_features)                           # :72
        self._fc2 = nn.Linear(out_features, n_classes)                   # :73

    def forward(self, x):
        h = self._fc1(x.float())                                          # :78-79
        n = h.shape[1]
        side = int(math.ceil(math.sqrt(n)))                               # :83-86
        h = torch.cat([h, h[:, :side * side - n, :]], dim=1)
        cls = self.cls_token.expand(h.shape[0], -1, -1).to(h.device)     # :90-92
        h = torch.cat((cls, h), dim=1)
        h, _ = self.layer1(h)                                             # :96
        h = self.pos_layer(h, side, side)                                 # :101
        h, attn2 = self.layer2(h)                                         # :105
        logits = self._fc2(self.norm(h)[:, 0])                            # :110-113
        return logits, attn2                                              # :114
