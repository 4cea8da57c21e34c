"""Drop-in ``nystrom_attention.NystromAttention`` on the HIP kernels.

The reference imports the class from the third-party package
(``code/models/TransMIL.py:5``; also CTMIL.py:5, TransformerMIL.py:5,
MDMIL.py:5) and builds it as ``NystromAttention(dim=512, dim_head=64, heads=8,
num_landmarks=256, pinv_iterations=6, residual=True, dropout=0.7)``
(``code/models/TransMIL.py:26-34``).  Constructor arguments, parameter names
(``to_qkv``, ``to_out.0``, ``res_conv``) and ``forward(x, mask=None,
return_attn=False)`` match the package, so state_dicts load unchanged.

Supported geometry on the HIP path: ``dim_head == 64``, ``num_landmarks ==
256``, ``residual=True`` with the 33-tap conv, ``mask=None`` (every reference
call site).  Anything else raises ``NotImplementedError`` -- there is no CPU
or eager-PyTorch fallback.

``return_attn=True`` materialises ``attn1 @ attn2_inv @ attn3`` ([B, h, n, n],
SURVEY.md App. A eq. 11) on the device from the saved factors; it is off the
training hot path (the reference computes it on every call, 301 GF per layer at
N = 8192, and never uses it for the loss).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .engine import NystromEngine, NL, DH


def _check_dtype(dtype):
    if dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("compute dtype must be torch.float32 or torch.bfloat16")
    return dtype


class _NystromFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, heads, drop_p, seed_dev, x, wqkv, wo, bo, wconv):
        out, c = engine.forward(x, wqkv, wo, bo, wconv, heads, drop_p, 0x51ED27, seed_dev)
        ctx.engine, ctx.c = engine, c
        return out

    @staticmethod
    def backward(ctx, dout):
        dx, dwqkv, dwo, dbo, dwconv = ctx.engine.backward(dout, ctx.c)
        return None, None, None, None, dx, dwqkv, dwo, dbo, dwconv


class NystromAttention(nn.Module):
    def __init__(self, dim, dim_head=64, heads=8, num_landmarks=256, pinv_iterations=6, residual=True,
                 residual_conv_kernel=33, eps=1e-8, dropout=0.0):
        super().__init__()
        self.eps = eps
        inner = heads * dim_head
        self.num_landmarks = num_landmarks
        self.pinv_iterations = pinv_iterations
        self.heads = heads
        self.dim_head = dim_head
        self.scale = dim_head ** -0.5
        self.to_qkv = nn.Linear(dim, inner * 3, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim), nn.Dropout(dropout))
        self.residual = residual
        self.residual_conv_kernel = residual_conv_kernel
        if residual:
            k = residual_conv_kernel
            self.res_conv = nn.Conv2d(heads, heads, (k, 1), padding=(k // 2, 0), groups=heads, bias=False)
        self.compute_dtype = torch.bfloat16
        self.register_buffer("_dropout_counter", torch.randint(0, 2 ** 62, (1,), dtype=torch.int64),
                             persistent=False)

    def _supported(self, mask):
        if mask is not None:
            raise NotImplementedError("HIP NystromAttention: mask is not supported (no reference call site uses it)")
        if (self.dim_head, self.num_landmarks, self.pinv_iterations) != (DH, NL, 6) or not self.residual \
                or self.residual_conv_kernel != 33:
            raise NotImplementedError(
                "HIP NystromAttention supports dim_head=64, num_landmarks=256, pinv_iterations=6, "
                "residual=True, residual_conv_kernel=33 (the TransMIL configuration)")

    def forward(self, x, mask=None, return_attn=False):
        self._supported(mask)
        if not x.is_cuda:
            raise RuntimeError("HIP NystromAttention needs a GPU tensor (no CPU path)")
        engine = NystromEngine(_check_dtype(self.compute_dtype))
        drop_p = self.to_out[1].p if self.training else 0.0
        seed_dev = None
        if drop_p > 0:
            self._dropout_counter.add_(1)
            seed_dev = self._dropout_counter.clone()
        out = _NystromFn.apply(engine, self.heads, drop_p, seed_dev, x.float(), self.to_qkv.weight,
                               self.to_out[0].weight, self.to_out[0].bias, self.res_conv.weight)
        if return_attn:
            return out, self._attn_matrix(x)
        return out

    @torch.no_grad()
    def _attn_matrix(self, x):
        engine = NystromEngine(torch.float32)
        _, c = engine.forward(x.float(), self.to_qkv.weight, self.to_out[0].weight, self.to_out[0].bias,
                              self.res_conv.weight, self.heads, 0.0, 0)
        return attention_matrix(c["qkv"], c["core"], self.heads)


@torch.no_grad()
def attention_matrix(qkv, core, heads):
    """attn1 @ Z @ attn3 ([B, h, n, n]) from the saved factors (App. A eq. 11)."""
    q, k = qkv[0].float(), qkv[1].float()
    a1 = torch.softmax(q @ core["kl"].transpose(-1, -2), dim=-1)
    a3 = torch.softmax(core["ql"] @ k.transpose(-1, -2), dim=-1)
    attn = (a1 @ core["z"]) @ a3
    n = attn.shape[-1]
    return attn.view(-1, heads, n, n)
