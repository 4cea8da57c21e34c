"""Drop-in ``models/TransformerMIL.py`` (code/models/TransformerMIL.py:74-152, ViT blocks of
code/models/_transformer.py:6-58) on the MI355X kernels.

Same constructor, parameter names and ``forward(x) -> logits``: ``fc1``, class token,
Dropout(0.5), two 2-deep pre-norm transformers (full softmax attention, 8 heads x 64, MLP
512 -> 512), class token -> LayerNorm -> ``_fc2``.  The Linear layers and LayerNorms run on
the HIP GEMM / LayerNorm kernels; the softmax attention core is
``torch.nn.functional.scaled_dot_product_attention`` (the ROCm flash path in bf16 mode; this
sibling head is outside the NystromAttention hot path).  ``pos_layer_0``, ``conv1/2`` and
``layer1/2`` are constructed for state_dict compatibility and unused, as in the reference.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .CTMIL import conv_block
from .TransMIL import PPEG, TransLayer


class PreNorm(nn.Module):
    """``fn(LayerNorm(x))`` (_transformer.py:6-13), HIP LayerNorm."""

    def __init__(self, dim, fn):
        super().__init__()
        self.norm = ops.LayerNorm(dim)
        self.fn = fn

    def forward(self, x):
        return self.fn(self.norm(x))


class Attention(nn.Module):
    """_transformer.py:16-43: bias-free to_qkv, softmax(q k^T / sqrt(dh)) v, to_out + Dropout."""

    compute_dtype = torch.float32

    def __init__(self, dim=512, heads=8, dim_head=64, dropout=0.1):
        super().__init__()
        inner = dim_head * heads
        self.heads, self.scale = heads, dim_head ** -0.5
        self.to_qkv = nn.Linear(dim, inner * 3, bias=False)
        self.project_out = not (heads == 1 and dim_head == dim)
        self.to_out = nn.Sequential(nn.Linear(inner, dim), nn.Dropout(dropout)) if self.project_out else nn.Identity()

    def forward(self, x):
        b, n, _ = x.shape
        qkv = ops.linear(self.to_qkv, x)
        q, k, v = (t.reshape(b, n, self.heads, -1).transpose(1, 2) for t in qkv.chunk(3, dim=-1))
        dt = self.compute_dtype
        o = F.scaled_dot_product_attention(q.to(dt), k.to(dt), v.to(dt), scale=self.scale).float()
        o = o.transpose(1, 2).reshape(b, n, -1)
        if not self.project_out:
            return o
        return self.to_out[1](ops.linear(self.to_out[0], o))


class FeedForward(nn.Module):
    """Linear + GELU + Dropout + Linear + Dropout (_transformer.py:46-58), HIP GEMMs."""

    def __init__(self, dim=512, hidden_dim=1024, dropout=0.1):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(dim, hidden_dim), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(hidden_dim, dim), nn.Dropout(dropout))

    def forward(self, x):
        n = self.net
        return n[4](ops.linear(n[3], n[2](ops.linear_gelu(n[0], x))))


class Transformer(nn.Module):
    """TransformerMIL.py:18-32: ``depth`` x (x = Attn(LN x) + x; x = FF(LN x) + x)."""

    def __init__(self, dim, depth, heads, dim_head, mlp_dim, dropout=0.0):
        super().__init__()
        self.layers = nn.ModuleList([nn.ModuleList([
            PreNorm(dim, Attention(dim, heads=heads, dim_head=dim_head, dropout=dropout)),
            PreNorm(dim, FeedForward(dim, mlp_dim, dropout=dropout))]) for _ in range(depth)])

    def forward(self, x):
        for attn, ff in self.layers:
            x = attn(x) + x
            x = ff(x) + x
        return x


class TransformerMIL(nn.Module):
    def __init__(self, n_classes, in_features, out_features=512):
        super().__init__()
        self.pos_layer_0 = PPEG(dim=out_features)
        self.conv1 = conv_block(in_features, in_features // 2)
        self.conv2 = conv_block(in_features // 2, out_features)
        if in_features == 2048:                                      # :106-110
            self.fc1 = nn.Sequential(nn.Linear(in_features, in_features // 2), nn.GELU(), nn.Dropout(p=0.6),
                                     ops.LayerNorm(in_features // 2), nn.Linear(in_features // 2, out_features),
                                     nn.GELU())
        elif in_features == 1024:                                    # :111-115
            self.fc1 = nn.Sequential(nn.Linear(in_features, out_features), nn.GELU(), nn.Dropout(p=0.6),
                                     ops.LayerNorm(out_features))
        elif in_features in (768, 384):                              # :116-119
            self.fc1 = nn.Sequential(nn.Linear(in_features, 512, bias=True), nn.ReLU())
        self.cls_token = nn.Parameter(torch.randn(1, 1, out_features))
        self.n_classes = n_classes
        self.layer1 = TransLayer(dim=out_features)
        self.layer2 = TransLayer(dim=out_features)
        self.norm = ops.LayerNorm(out_features)
        self._fc2 = nn.Linear(out_features, self.n_classes)
        self.transformer1 = Transformer(dim=out_features, depth=2, dim_head=64, heads=8, mlp_dim=512, dropout=0.5)
        self.transformer2 = Transformer(dim=out_features, depth=2, dim_head=64, heads=8, mlp_dim=512, dropout=0.5)
        self.dropout = nn.Dropout(0.5)
        self.to_latent = nn.Identity()
        self.pool = "cls"

    def set_compute_dtype(self, dtype):
        """bf16: the attention core runs in bf16 (flash); fp32 otherwise."""
        for m in self.modules():
            if isinstance(m, Attention):
                m.compute_dtype = dtype
        return self

    def _fc1(self, x):
        f = self.fc1
        if len(f) == 2:                                              # Linear + ReLU
            return torch.relu(ops.linear(f[0], x))
        h = f[3](f[2](ops.linear_gelu(f[0], x)))
        return ops.linear_gelu(f[4], h) if len(f) == 6 else h

    def forward(self, x):
        x = x.squeeze(0)                                             # :139
        if not x.is_cuda:
            raise RuntimeError("TransformerMIL (HIP) needs a GPU tensor: there is no CPU path")
        b, _, _ = x.shape                                            # :141
        x = self._fc1(x.float())
        x = torch.cat((self.cls_token.expand(b, -1, -1), x), dim=1)
        x = self.transformer2(self.transformer1(self.dropout(x)))
        x = x.mean(dim=1) if self.pool == "mean" else x[:, 0]
        return ops.linear(self._fc2, self.norm(self.to_latent(x)[:, None])[:, 0])
