"""CPU oracle: restatement of the third-party ``nystrom_attention.NystromAttention``.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module; the product path
(``transmil_deepgraft_amd``) never does.

The reference calls ``from nystrom_attention import NystromAttention``
(``code/models/TransMIL.py:5``, ctor args ``code/models/TransMIL.py:26-34``,
call ``code/models/TransMIL.py:47``).  The package is the PyPI
``nystrom-attention`` project (lucidrains); the reference pins no version and
does not vendor it.  The variant is pinned by its consumers: a 4-D
``[B, h, n', n']`` attention return and FRONT padding to a multiple of the
landmark count (``code/visualize_mil.py:580-581``,
``code/models/TransMIL.py:190-193``) -- the 0.0.11-era API restated in
SURVEY.md section 8 Appendix A (eq. 1-11).  The package itself is absent (no
lock file, not installable offline), so no reference-held fixture pins this
class directly.  Its arithmetic is pinned against an independent
implementation of the same algorithm: ``tests/test_oracle.py::
test_nystrom_eq2_to_9_match_hf_nystromformer`` compares eq. 2-9 (segment-mean
landmarks, the three softmaxes, the Moore-Penrose iteration, the aggregation
and the 33-tap residual conv) with HF ``NystromformerSelfAttention.forward``
in fp64 to 1e-9 at n' in {512 (B=2), 1280, 8448}; the front pad and the
``out[:, -n:]`` slice (eq. 1, 10), which HF does not do, are pinned by the
fixtures generated from the reference's own ``code/models/TransMIL.py``
(tests/golden/make_golden*.py).

Everything is plain torch on the CPU, in the dtype of the input (fp32 or fp64).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


def moore_penrose_iter_pinv(x: torch.Tensor, iters: int = 6) -> torch.Tensor:
    """Iterative Moore-Penrose pseudo-inverse (SURVEY.md App. A eq. 7).

    ``Z0 = x^T / (max_all rowsum|x| * max_all colsum|x|)``; the two maxima are
    taken over the WHOLE tensor (all bags and heads), then 6 times
    ``XZ = x Z;  Z = (0.25 Z)(13I - XZ(15I - XZ(7I - XZ)))``.
    """
    abs_x = x.abs()
    col = abs_x.sum(dim=-1)          # row sums   ("col" in the package)
    row = abs_x.sum(dim=-2)          # column sums ("row" in the package)
    z = x.transpose(-1, -2) / (col.max() * row.max())
    eye = torch.eye(x.shape[-1], dtype=x.dtype, device=x.device).unsqueeze(0)
    for _ in range(iters):
        xz = x @ z
        z = (0.25 * z) @ (13 * eye - (xz @ (15 * eye - (xz @ (7 * eye - xz)))))
    return z


class NystromAttention(nn.Module):
    """Same ctor/forward contract and parameter names as the package class.

    Parameters: ``to_qkv`` Linear(dim, 3*heads*dim_head, bias=False);
    ``to_out`` = Sequential(Linear(inner, dim), Dropout(dropout));
    ``res_conv`` depthwise Conv2d(heads, heads, (k, 1), padding=(k//2, 0),
    groups=heads, bias=False)  (SURVEY.md section 8 a4).
    """

    def __init__(self, dim, dim_head=64, heads=8, num_landmarks=256,
                 pinv_iterations=6, residual=True, residual_conv_kernel=33,
                 eps=1e-8, dropout=0.0):
        super().__init__()
        self.eps = eps
        inner = heads * dim_head
        self.num_landmarks = num_landmarks
        self.pinv_iterations = pinv_iterations
        self.heads = heads
        self.scale = dim_head ** -0.5
        self.to_qkv = nn.Linear(dim, inner * 3, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim), nn.Dropout(dropout))
        self.residual = residual
        if residual:
            k = residual_conv_kernel
            self.res_conv = nn.Conv2d(heads, heads, (k, 1), padding=(k // 2, 0),
                                      groups=heads, bias=False)

    def forward(self, x, mask=None, return_attn=False):
        b, n, _ = x.shape
        h, m = self.heads, self.num_landmarks
        # eq. 1: zero rows at the FRONT up to a multiple of m
        if n % m:
            pad = m - n % m
            x = F.pad(x, (0, 0, pad, 0), value=0.0)
            if mask is not None:
                mask = F.pad(mask, (pad, 0), value=False)
        # eq. 2-3
        q, k, v = self.to_qkv(x).chunk(3, dim=-1)
        q, k, v = (t.reshape(b, -1, h, t.shape[-1] // h).transpose(1, 2) for t in (q, k, v))
        if mask is not None:
            mk = mask[:, None, :, None].to(q.dtype)
            q, k, v = q * mk, k * mk, v * mk
        q = q * self.scale
        # eq. 4: landmarks = mean over segments of l consecutive (padded) tokens
        seg = math.ceil(n / m)
        q_l = q.reshape(b, h, m, seg, -1).sum(dim=3)
        k_l = k.reshape(b, h, m, seg, -1).sum(dim=3)
        if mask is not None:
            msum = mask.reshape(b, m, seg).sum(dim=-1).to(q.dtype)
            div = msum[:, None, :, None] + self.eps
            mask_l = msum > 0
        else:
            div = seg
        q_l = q_l / div
        k_l = k_l / div
        # eq. 5
        sim1 = q @ k_l.transpose(-1, -2)
        sim2 = q_l @ k_l.transpose(-1, -2)
        sim3 = q_l @ k.transpose(-1, -2)
        if mask is not None:
            neg = -torch.finfo(q.dtype).max
            mq = mask[:, None, :, None]
            ml = mask_l[:, None, :, None]
            sim1 = sim1.masked_fill(~(mq & mask_l[:, None, None, :]), neg)
            sim2 = sim2.masked_fill(~(ml & mask_l[:, None, None, :]), neg)
            sim3 = sim3.masked_fill(~(ml & mask[:, None, None, :]), neg)
        # eq. 6-8
        a1, a2, a3 = (t.softmax(dim=-1) for t in (sim1, sim2, sim3))
        z = moore_penrose_iter_pinv(a2, self.pinv_iterations)
        out = (a1 @ z) @ (a3 @ v)
        # eq. 9: depthwise 33x1 conv of v along the sequence
        if self.residual:
            out = out + self.res_conv(v)
        # eq. 10
        out = out.transpose(1, 2).reshape(b, -1, h * out.shape[-1])
        out = self.to_out(out)
        out = out[:, -n:]
        if return_attn:
            # eq. 11
            return out, a1 @ z @ a3
        return out
