"""Standalone (unfused) HIP ops behind the drop-in submodules.

``TransMIL.forward`` never uses these -- it runs the fused engine.  They back
``TransLayer.forward`` / ``PPEG.forward`` when a caller drives a submodule on
its own (e.g. the reference's GradCAM / attention visualisation scripts hook
``model.layer1.norm``, code/visualize_mil.py:225-234).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from ._lib import F32
from .engine import _p, _stream, LN_EPS


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        B, S, D = x.shape
        xc = x.contiguous()
        y = torch.empty_like(xc)
        mean = torch.empty(B * S, device=x.device)
        rstd = torch.empty(B * S, device=x.device)
        _lib.call("tm_layernorm_fwd", _p(xc), _p(w), _p(b), C.c_float(eps), B * S, D, S, S, 0, F32, _p(y),
                  _p(mean), _p(rstd), _stream())
        ctx.save_for_backward(xc, w, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        B, S, D = x.shape
        dx = torch.zeros_like(x)
        dw = torch.empty_like(w)
        db = torch.empty_like(w)
        rpb = 64
        work = torch.empty(_lib.query("tm_layernorm_bwd_workspace", B * S, D, rpb) // 4, device=x.device)
        _lib.call("tm_layernorm_bwd", _p(dy.float().contiguous()), F32, _p(x), _p(w), _p(mean), _p(rstd),
                  B * S, D, S, S, 0, rpb, _p(dx), _p(work), _p(dw), _p(db), _stream())
        return dx, dw, db, None


def layer_norm(module, x):
    """nn.LayerNorm(dim) forward on the HIP kernel (fp32)."""
    if not x.is_cuda:
        raise RuntimeError("HIP LayerNorm needs a GPU tensor")
    eps = getattr(module, "eps", LN_EPS)
    return _LayerNormFn.apply(x.float(), module.weight, module.bias, eps)


class _PPEGFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, G, w7, b7, w5, b5, w3, b3):
        B, S, D = x.shape
        xc = x.contiguous()
        wf = torch.empty(D * 49, device=x.device)
        bf = torch.empty(D, device=x.device)
        _lib.call("tm_ppeg_fold", _p(w7), _p(b7), _p(w5), _p(b5), _p(w3), _p(b3), D, _p(wf), _p(bf), _stream())
        y = torch.empty_like(xc)
        _lib.call("tm_ppeg_fwd", _p(xc), B, G, D, _p(wf), _p(bf), _p(y), _stream())
        ctx.save_for_backward(xc, wf)
        ctx.G = G
        ctx.shapes = (w7.shape, w5.shape, w3.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wf = ctx.saved_tensors
        B, S, D = x.shape
        G = ctx.G
        dx = torch.empty_like(x)
        work = torch.empty(_lib.query("tm_ppeg_bwd_workspace", B, G, D) // 4, device=x.device)
        dwsum = torch.empty(D * 50, device=x.device)
        s7, s5, s3 = ctx.shapes
        dw7, dw5, dw3 = (torch.empty(s, device=x.device) for s in (s7, s5, s3))
        db7, db5, db3 = (torch.empty(D, device=x.device) for _ in range(3))
        _lib.call("tm_ppeg_bwd", _p(x), _p(dy.float().contiguous()), B, G, D, _p(wf), _p(dx), _p(work), _p(dwsum),
                  _p(dw7), _p(db7), _p(dw5), _p(db5), _p(dw3), _p(db3), _stream())
        return dx, None, dw7, db7, dw5, db5, dw3, db3


def ppeg(module, x, G):
    if not x.is_cuda:
        raise RuntimeError("HIP PPEG needs a GPU tensor")
    if x.shape[1] != G * G + 1:
        raise ValueError(f"PPEG expects 1 + G*G tokens, got {x.shape[1]} for G={G}")
    return _PPEGFn.apply(x.float(), G, module.proj.weight, module.proj.bias, module.proj1.weight,
                         module.proj1.bias, module.proj2.weight, module.proj2.bias)
