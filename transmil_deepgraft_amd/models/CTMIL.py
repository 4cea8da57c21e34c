"""Drop-in ``models/CTMIL.py`` (code/models/CTMIL.py:74-163) on the MI355X kernels.

Same constructor, parameter names and ``forward(x) -> logits``.  The input is a feature grid
``[1, B, C, H, W]``: two conv blocks (Conv3x3 + BatchNorm + GELU + MaxPool(3,2,1); PyTorch-ROCm
convolutions, bf16 under the bf16 compute mode) give ``[B, 512, H', W']``, which the reference
REINTERPRETS with a raw ``view`` as ``[B, H'*H', 512]`` tokens (:137) -- reproduced exactly --
and the TransMIL body (grid pad, class token, TransLayer, PPEG ``pos_layer_0``, TransLayer,
LayerNorm, ``_fc2``) runs as the fused HIP engine in its pre-embedded-input mode, returning
dL/d(tokens) into the conv stack's autograd.  ``_fc1`` is constructed but unused, as there.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from ..engine import FC1_EMBED
from .TransMIL import PPEG, TransLayer, TransMIL


def conv_block(cin, cout):
    """Conv3x3 (no bias) + BatchNorm2d + GELU + MaxPool(3, 2, 1) (CTMIL.py:88-99)."""
    return nn.Sequential(nn.Conv2d(cin, cout, kernel_size=3, stride=1, padding=1, bias=False),
                         nn.BatchNorm2d(cout), nn.GELU(), nn.MaxPool2d(kernel_size=3, stride=2, padding=1))


class CTMIL(TransMIL):
    _head = "_fc2"

    def __init__(self, n_classes, in_features, out_features=512):
        nn.Module.__init__(self)
        self.pos_layer_0 = PPEG(dim=out_features)
        self.conv1 = conv_block(in_features, in_features // 2)
        self.conv2 = conv_block(in_features // 2, out_features)
        if in_features == 2048:                                     # :101-106
            self._fc1 = nn.Sequential(nn.Linear(in_features, in_features // 2),
                                      nn.Linear(in_features // 2, out_features), nn.GELU())
        elif in_features == 1024:                                   # :107-111
            self._fc1 = nn.Sequential(nn.Linear(in_features, out_features), nn.GELU(), nn.Dropout(p=0.6),
                                      ops.LayerNorm(out_features))
        elif in_features == 768:                                    # :112-113
            self._fc1 = nn.Sequential(nn.Linear(in_features, 512, bias=True), nn.ReLU())
        self.cls_token = nn.Parameter(torch.randn(1, 1, out_features))
        self.n_classes = n_classes
        self.in_features = in_features
        self.layer1 = TransLayer(dim=out_features)
        self.layer2 = TransLayer(dim=out_features)
        self.norm = ops.LayerNorm(out_features)
        self._fc2 = nn.Linear(out_features, self.n_classes)
        self.compute_dtype = torch.bfloat16
        self.register_buffer("_dropout_counter", torch.randint(0, 2 ** 62, (1,), dtype=torch.int64),
                             persistent=False)

    @property
    def pos_layer(self):
        return self.pos_layer_0

    def _fc1_layout(self):
        return FC1_EMBED

    def _pre_embed(self, x):
        return x

    def _engine_params(self, layout):
        named = [(n, p) for n, p in self.named_parameters() if not n.startswith(("conv1.", "conv2.", "_fc1."))]
        return (tuple(n.replace("pos_layer_0.", "pos_layer.", 1) for n, _ in named), tuple(p for _, p in named))

    def grad_bucket_parts(self, split_layer1=False):
        return [[p for _, p in self.named_parameters()]]

    def forward_ce(self, x, label, class_stats=None):
        """No fused loss on this head: the task runs ``forward`` and its own CE launch."""
        return None

    def forward(self, x):
        x = x.squeeze(0)                                            # :134
        if not x.is_cuda:
            raise RuntimeError("CTMIL (HIP) needs a GPU tensor: there is no CPU path")
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.compute_dtype == torch.bfloat16):
            h = self.conv2(self.conv1(x.float()))                   # :135-136
        h = h.float().contiguous()
        h = h.view(h.shape[0], h.shape[2] * h.shape[2], h.shape[1])    # :137, raw reinterpretation
        if not self.fused or self._hooked():
            return self._forward_modules(h, False)
        return self._fused(h.contiguous(), FC1_EMBED, False)
