"""Drop-in ``models/MDMIL.py`` (code/models/MDMIL.py) on the fused HIP TransMIL engine."""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .TransMIL import TransMIL, TransLayer, PPEG


class MDMIL(TransMIL):
    """``code/models/MDMIL.py:60-114``: TransMIL with ``_fc1 = Linear(1024, 512) + GELU``, the
    head named ``_fc2`` and ``forward(x) -> (logits, attn2)`` (attn2 = layer2's NystromAttention
    map, an ``AttentionMap`` here; row/col ``padding`` is the class token).  Same fused HIP engine."""

    _head = "_fc2"

    def __init__(self, n_classes):
        nn.Module.__init__(self)
        in_features, out_features = 1024, 512          # MDMIL.py:63-64
        self.pos_layer = PPEG(dim=out_features)
        self._fc1 = nn.Sequential(nn.Linear(in_features, out_features), nn.GELU())
        self.cls_token = nn.Parameter(torch.randn(1, 1, out_features))
        self.n_classes = n_classes
        self.in_features = in_features
        self.layer1 = TransLayer(norm_layer=ops.LayerNorm, dim=out_features)
        self.layer2 = TransLayer(norm_layer=ops.LayerNorm, dim=out_features)
        self.norm = ops.LayerNorm(out_features)
        self._fc2 = nn.Linear(out_features, self.n_classes)
        self.compute_dtype = torch.bfloat16
        self.register_buffer("_dropout_counter", torch.randint(0, 2 ** 62, (1,), dtype=torch.int64),
                             persistent=False)

    def forward_ce(self, x, label, class_stats=None):
        """No fused loss on this head: the task runs ``forward`` and its own CE launch."""
        return None

    def forward(self, x):
        logits, (attn2, _padding) = super().forward(x, return_attn=True)
        return logits, attn2
