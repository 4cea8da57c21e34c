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

``return_attn=True`` returns an :class:`AttentionMap` -- ``attn1 @ attn2_inv @ attn3``
([B, h, n, n], SURVEY.md App. A eq. 11) held as the forward's factors.  Indexing one
row of it, ``attn[b, heads, r, cols]`` (the only access the reference's consumers
make, code/visualize_mil.py:580-581), runs the ``tm_nys_attn_row`` kernel:
O(h (m^2 + m n)) work and no n x n matrix.  Any other use materialises the full
product once (on the device).  The reference computes that product on every call
(301 GF per layer at N = 8192) and never uses it for the loss.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from ._lib import BF16, F32
from .engine import NystromEngine, NL, DH, _p, _stream


def _check_dtype(dtype):
    if dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("compute dtype must be torch.float32 or torch.bfloat16")
    return dtype


class _NystromFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, heads, drop_p, seed_dev, holder, x, wqkv, wo, bo, wconv):
        with torch.cuda.device(x.device):
            out, c = engine.forward(x, wqkv, wo, bo, wconv, heads, drop_p, 0x51ED27, seed_dev)
        ctx.engine, ctx.c = engine, c
        if holder is not None:
            holder["c"] = c
        return out

    @staticmethod
    def backward(ctx, dout):
        with torch.cuda.device(dout.device):
            dx, dwqkv, dwo, dbo, dwconv = ctx.engine.backward(dout, ctx.c)
        return None, None, None, None, None, dx, dwqkv, dwo, dbo, dwconv


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
        holder = {} if return_attn else None
        out = _NystromFn.apply(engine, self.heads, drop_p, seed_dev, holder, x.float(), self.to_qkv.weight,
                               self.to_out[0].weight, self.to_out[0].bias, self.res_conv.weight)
        if return_attn:   # the factors of THIS forward (the reference returns attn of the same call)
            return out, AttentionMap(holder["c"]["qkv"], holder["c"]["core"], self.heads)
        return out


@torch.no_grad()
def attention_matrix(qkv, core, heads):
    """attn1 @ Z @ attn3 ([B, h, n, n]) from the saved factors (App. A eq. 11)."""
    q, k = qkv[0].float(), qkv[1].float()
    a1 = torch.softmax(q @ core["kl"].transpose(-1, -2), dim=-1)
    a3 = torch.softmax(core["ql"] @ k.transpose(-1, -2), dim=-1)
    attn = (a1 @ core["z"]) @ a3
    n = attn.shape[-1]
    return attn.view(-1, heads, n, n)


@torch.no_grad()
def attention_row(qkv, core, heads, row):
    """Row `row` of attn1 @ Z @ attn3 for every bag and head: [B, h, n] fp32 (HIP kernel)."""
    q, k = qkv[0], qkv[1]
    nbh, n = q.shape[0], q.shape[1]
    if not -n <= row < n:
        raise IndexError(f"attention row {row} out of range for n = {n}")
    row %= n
    out = torch.empty(nbh, n, device=q.device, dtype=torch.float32)
    _lib.call("tm_nys_attn_row", BF16 if q.dtype == torch.bfloat16 else F32, _p(q), _p(k), _p(core["ql"]),
              _p(core["kl"]), _p(core["z"]), _p(core["lse3"]), nbh, n, row, _p(out), _stream())
    return out.view(-1, heads, n)


class AttentionMap:
    """The [B, h, n, n] ``return_attn`` product of one NystromAttention forward, kept as its
    factors (q, k, landmarks, Z = pinv(attn2), attn3's log-sum-exp rows).

    ``attn[b, heads, r, cols]`` with an integer row ``r`` computes that row only
    (``tm_nys_attn_row``); every other index, attribute or tensor use materialises the full
    product once (``attention_matrix``) and forwards to it.  That product is B·h·n'² fp32
    (35 GB per layer at N = 32768): above ``max_full_bytes`` (default 8 GiB, class attribute)
    it raises instead of allocating; raise the limit explicitly to materialise anyway."""

    max_full_bytes = 8 << 30

    def __init__(self, qkv, core, heads):
        self._qkv, self._core, self._heads = qkv, core, heads
        nbh, n = qkv.shape[1], qkv.shape[2]
        self.shape = torch.Size((nbh // heads, heads, n, n))
        self.dtype = torch.float32
        self.device = qkv.device
        self.ndim = 4
        self._full = None

    def __len__(self):
        return self.shape[0]

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim]

    def row(self, r):
        """[B, h, n] row r of every bag and head."""
        return attention_row(self._qkv, self._core, self._heads, int(r))

    def full(self):
        if self._full is None:
            nbytes = 4 * self.shape[0] * self.shape[1] * self.shape[2] * self.shape[3]
            if nbytes > AttentionMap.max_full_bytes:
                raise RuntimeError(
                    f"AttentionMap: materialising the full {tuple(self.shape)} return_attn product needs "
                    f"{nbytes / 2**30:.1f} GiB; index one row (attn[b, heads, r, cols]) instead, or raise "
                    "AttentionMap.max_full_bytes to allow it")
            self._full = attention_matrix(self._qkv, self._core, self._heads)
        return self._full

    def __getitem__(self, key):
        if isinstance(key, tuple) and len(key) == 4 and isinstance(key[2], int) and self._full is None:
            return self.row(key[2])[key[0], key[1], key[3]]
        return self.full()[key]

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.full(), name)

    def __array__(self, dtype=None):
        a = self.full().cpu().numpy()
        return a if dtype is None else a.astype(dtype)
