"""Drop-in ``models/AttMIL.py`` (code/models/AttMIL.py:20-110): gated attention MIL pooling
(Ilse et al. 2018) on the MI355X HIP kernels.

Same constructor, parameter names and ``forward(x) -> logits``.  The forward is
``_fc1`` (HIP GEMM Linear+GELU, Dropout, HIP LayerNorm, ...), then one fused pooling node:
``Z = H [Wv;Wu]^T + [bv;bu]`` on the HIP GEMM (f32 MFMA) and ``tm_attmil_fwd`` (scores
``w . tanh(Zv) sigmoid(Zu) + b``, softmax over the N instances, ``M = p H``, the classifier);
the backward is ``tm_attmil_bwd`` plus three GEMM/colsum launches.  fp32 throughout: the pooling
is a few GFLOP even at N = 8192, HBM-bound on the single pass over H.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import _lib, ops
from .._lib import F32
from ..engine import Pool, _p, _stream, colsum, gemm, weight_grad


class _GatedPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, H, wvu, bvu, w, b, wc, bc):
        N, L = H.shape
        D2, C = wvu.shape[0], wc.shape[0]
        D = D2 // 2
        dev = H.device
        Hc = H.contiguous()
        Z = torch.empty(N, D2, device=dev)
        gemm(Hc, wvu.contiguous(), Z, N, D2, L, lda=L, ldb=L, ldc=D2, dtype=F32, c_dtype=F32, bias=bvu.contiguous())
        work = torch.empty(_lib.query("tm_attmil_fwd_workspace", N, L) // 4, device=dev)
        a, p = torch.empty(N, device=dev), torch.empty(N, device=dev)
        M = torch.empty(L, device=dev)
        logits = torch.empty(1, C, device=dev)
        _lib.call("tm_attmil_fwd", _p(Z), _p(Hc), _p(w.contiguous()), _p(b.contiguous()), _p(wc.contiguous()),
                  _p(bc.contiguous()), N, L, D, C, _p(work), _p(a), _p(p), _p(M), _p(logits), _stream())
        ctx.save_for_backward(Hc, Z, wvu, w, p, M, wc)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        H, Z, wvu, w, p, M, wc = ctx.saved_tensors
        N, L = H.shape
        D2, C = wvu.shape[0], wc.shape[0]
        D = D2 // 2
        dev = H.device
        pool = Pool(dev)
        work = torch.empty(_lib.query("tm_attmil_bwd_workspace", N, L, D) // 4, device=dev)
        dZ, dH = torch.empty(N, D2, device=dev), torch.empty(N, L, device=dev)
        dM, dw, db = torch.empty(L, device=dev), torch.empty(1, D, device=dev), torch.empty(1, device=dev)
        dwc, dbc = torch.empty(C, L, device=dev), torch.empty(C, device=dev)
        _lib.call("tm_attmil_bwd", _p(Z), _p(H), _p(w.contiguous()), _p(p), _p(M), _p(wc.contiguous()),
                  _p(dlogits.float().contiguous()), N, L, D, C, _p(work), _p(dZ), _p(dH), _p(dM), _p(dw), _p(db),
                  _p(dwc), _p(dbc), _stream())
        gemm(dZ, wvu.contiguous(), dH, N, L, D2, lda=D2, ldb=L, ldc=L, b_kn=1, dtype=F32, c_dtype=F32,
             accumulate=True)
        dwvu = torch.empty(D2, L, device=dev)
        weight_grad(dZ, H, dwvu, D2, L, N, ldy=D2, ldx=L, dtype=F32, work_pool=pool)
        dbvu = torch.empty(D2, device=dev)
        colsum(dZ, N, D2, D2, F32, dbvu, pool)
        return dH, dwvu, dbvu, dw, db, dwc, dbc


class AttMIL(nn.Module):
    """``code/models/AttMIL.py:20-110``.  ``feature_extractor_part2`` is constructed (state_dict)
    but unused, as in the reference; ``in_features`` other than 2048 / 1024 leave ``_fc1``
    undefined there too (the forward then fails the same way)."""

    def __init__(self, n_classes, in_features=2048, out_features=512):
        super().__init__()
        self.L, self.D, self.K = out_features, 128, 1
        self.n_classes = n_classes
        if in_features == 2048:                                     # :55-59
            self._fc1 = nn.Sequential(nn.Linear(in_features, in_features // 2), nn.GELU(), nn.Dropout(p=0.6),
                                      ops.LayerNorm(in_features // 2),
                                      nn.Linear(in_features // 2, out_features), nn.GELU())
        elif in_features == 1024:                                   # :60-63
            self._fc1 = nn.Sequential(nn.Linear(in_features, out_features), nn.GELU(), nn.Dropout(p=0.6),
                                      ops.LayerNorm(out_features))
        self.feature_extractor_part2 = nn.Sequential(nn.Linear(in_features, self.L), nn.ReLU())
        self.attention_V = nn.Sequential(nn.Linear(self.L, self.D), nn.Tanh())
        self.attention_U = nn.Sequential(nn.Linear(self.L, self.D), nn.Sigmoid())
        self.attention_weights = nn.Linear(self.D, self.K)
        self.classifier = nn.Sequential(nn.Linear(self.L * self.K, self.n_classes))

    def _embed(self, x):
        """_fc1 on the HIP ops: x [1, N, F] -> H [1, N, L]."""
        f = self._fc1
        h = ops.linear_gelu(f[0], x)
        h = f[2](h)
        h = f[3](h)
        if len(f) == 6:
            h = ops.linear_gelu(f[4], h)
        return h

    def forward(self, x):
        x = x.squeeze()                                             # :93
        if not x.is_cuda:
            raise RuntimeError("AttMIL (HIP) needs a GPU tensor: there is no CPU path")
        if x.dim() == 1:
            x = x.unsqueeze(0)
        if x.dim() != 2:
            raise ValueError(f"AttMIL pools one bag: x.squeeze() must be [N, F], got {tuple(x.shape)}")
        h = self._embed(x.float()[None])[0]                         # :94
        V, U = self.attention_V[0], self.attention_U[0]
        return _GatedPoolFn.apply(h, torch.cat([V.weight, U.weight]), torch.cat([V.bias, U.bias]),
                                  self.attention_weights.weight, self.attention_weights.bias,
                                  self.classifier[0].weight, self.classifier[0].bias)
