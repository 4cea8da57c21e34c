"""Standalone (unfused) HIP ops behind the drop-in submodules.

``TransMIL.forward`` uses the fused engine unless a hook is registered on one of its
submodules.  These ops back the module-by-module path it then takes (and
``TransLayer.forward`` / ``PPEG.forward`` / the norms when a caller drives a submodule
on its own): the reference's GradCAM / attention visualisation hooks ``model.norm`` and
``model.layer{1,2}.norm`` (code/visualize_mil.py:225-234, test_visualize.py:122,127).
fp32 operands throughout (a visualisation / analysis path, not the benchmark step).
"""
from __future__ import annotations

import ctypes as C

import torch

import torch.nn as nn

from . import _lib
from ._lib import F32
from .engine import Geometry, Pool, _p, _stream, LN_EPS, colsum, gemm, weight_grad


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
                  B * S, D, S, S, 0, rpb, 0, _p(dx), _p(work), _p(dw), _p(db), C.c_void_p(0), _stream())
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
        s7, s5, s3 = ctx.shapes
        dw7, dw5, dw3 = (torch.empty(s, device=x.device) for s in (s7, s5, s3))
        db7, db5, db3 = (torch.empty(D, device=x.device) for _ in range(3))
        _lib.call("tm_ppeg_bwd", _p(x), _p(dy.float().contiguous()), B, G, D, _p(wf), _p(dx), _p(work), _p(dw7),
                  _p(db7), _p(dw5), _p(db5), _p(dw3), _p(db3), F32, None, 0, 0, C.c_float(0.0), C.c_uint64(0),
                  None, None, _stream())
        return dx, None, dw7, db7, dw5, db5, dw3, db3


def ppeg(module, x, G):
    if not x.is_cuda:
        raise RuntimeError("HIP PPEG needs a GPU tensor")
    if x.shape[1] != G * G + 1:
        raise ValueError(f"PPEG expects 1 + G*G tokens, got {x.shape[1]} for G={G}")
    return _PPEGFn.apply(x.float(), G, module.proj.weight, module.proj.bias, module.proj1.weight,
                         module.proj1.bias, module.proj2.weight, module.proj2.bias)


class LayerNorm(nn.LayerNorm):
    """``nn.LayerNorm`` (same parameters and state_dict keys) whose forward is the HIP
    kernel, so forward / backward hooks registered on it fire."""

    def forward(self, x):
        return layer_norm(self, x)


class _EmbedFn(torch.autograd.Function):
    """_fc1 (Linear + GELU), grid pad (repeat the first G*G - N tokens) and the class token
    (code/models/TransMIL.py:175-186): x [B, N, F] -> H [B, S, D] fp32 on the GEMM epilogue."""

    @staticmethod
    def forward(ctx, x, w, b, cls):
        B, N, F = x.shape
        D = w.shape[0]
        geo = Geometry(B, N, F, D, 8)
        x2 = x.reshape(B * N, F).contiguous()
        H = torch.empty(B * geo.S, D, device=x.device)
        pre = torch.empty(B * N, D, device=x.device)
        gemm(x2, w.contiguous(), H, B * N, D, F, lda=F, ldb=F, ldc=D, dtype=F32, c_dtype=F32, bias=b, gelu=True,
             pre=pre, ld_pre=D, rowmap=(N, 0, geo.S, 1, geo.add, 1 + N))
        _lib.call("tm_put_cls", _p(cls.contiguous()), B, geo.S, D, _p(H), _stream())
        ctx.save_for_backward(x2, w, pre)
        ctx.geo = geo
        return H.view(B, geo.S, D)

    @staticmethod
    def backward(ctx, dH):
        x2, w, pre = ctx.saved_tensors
        geo = ctx.geo
        B, N, F, D, S = geo.B, geo.N, geo.F, w.shape[0], geo.S
        pool = Pool(dH.device)
        dpre = torch.empty(B * N, D, device=dH.device)
        dcls = torch.empty(1, 1, D, device=dH.device)
        _lib.call("tm_fc1_gelu_bwd", F32, _p(dH.float().contiguous()), _p(pre), B, N, S, geo.add, D, _p(dpre),
                  _p(dcls), _stream())
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(B * N, F, device=dH.device)
            gemm(dpre, w.contiguous(), dx, B * N, F, D, lda=D, ldb=F, ldc=F, b_kn=1, dtype=F32, c_dtype=F32)
            dx = dx.view(B, N, F)
        dw = torch.empty(D, F, device=dH.device)
        weight_grad(dpre, x2, dw, D, F, B * N, ldy=D, ldx=F, dtype=F32, work_pool=pool)
        db = torch.empty(D, device=dH.device)
        colsum(dpre, B * N, D, D, F32, db, pool)
        return dx, dw, db, dcls


def embed(lin, cls_token, x):
    """The last ``Linear + GELU`` of ``_fc1`` + grid pad + class token on the HIP GEMM."""
    if not x.is_cuda:
        raise RuntimeError("HIP _fc1 needs a GPU tensor")
    return _EmbedFn.apply(x.float(), lin.weight, lin.bias, cls_token)


class _LinearGeluFn(torch.autograd.Function):
    """y = GELU(x W^T + b) (fp32) on the HIP GEMM epilogue (pre-activation kept); backward
    dpre = dy GELU'(pre) (tm_gelu_bwd), dX = dpre W, dW = dpre^T X, db = colsum dpre."""

    @staticmethod
    def forward(ctx, x, w, b):
        shp = x.shape
        K = shp[-1]
        x2 = x.reshape(-1, K).contiguous()
        M, Nout = x2.shape[0], w.shape[0]
        y = torch.empty(M, Nout, device=x.device)
        pre = torch.empty(M, Nout, device=x.device)
        gemm(x2, w.contiguous(), y, M, Nout, K, lda=K, ldb=K, ldc=Nout, dtype=F32, c_dtype=F32, bias=b, gelu=True,
             pre=pre, ld_pre=Nout)
        ctx.save_for_backward(x2, w, pre)
        ctx.shp = shp
        return y.view(*shp[:-1], Nout)

    @staticmethod
    def backward(ctx, dy):
        x2, w, pre = ctx.saved_tensors
        M, K = x2.shape
        Nout = w.shape[0]
        pool = Pool(dy.device)
        dpre = torch.empty(M, Nout, device=dy.device)
        _lib.call("tm_gelu_bwd", F32, _p(dy.float().reshape(M, Nout).contiguous()), _p(pre), M * Nout, _p(dpre),
                  _stream())
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, device=dy.device)
            gemm(dpre, w.contiguous(), dx, M, K, Nout, lda=Nout, ldb=K, ldc=K, b_kn=1, dtype=F32, c_dtype=F32)
            dx = dx.view(ctx.shp)
        dw = torch.empty(Nout, K, device=dy.device)
        weight_grad(dpre, x2, dw, Nout, K, M, ldy=Nout, ldx=K, dtype=F32, work_pool=pool)
        db = torch.empty(Nout, device=dy.device)
        colsum(dpre, M, Nout, Nout, F32, db, pool)
        return dx, dw, db


def linear_gelu(lin, x):
    """``Sequential(Linear, GELU)`` forward on the HIP GEMM (the inner stage of the 2048 _fc1 branch)."""
    if not x.is_cuda:
        raise RuntimeError("HIP Linear+GELU needs a GPU tensor")
    return _LinearGeluFn.apply(x.float(), lin.weight, lin.bias)


class _LinearFn(torch.autograd.Function):
    """y = x W^T (+ b) (fp32) on the HIP GEMM, x [..., K]; backward dX = dY W, dW = dY^T X,
    db = colsum dY."""

    @staticmethod
    def forward(ctx, x, w, b):
        shp = x.shape
        K = shp[-1]
        xc = x.reshape(-1, K).contiguous()
        M, Nout = xc.shape[0], w.shape[0]
        y = torch.empty(M, Nout, device=x.device)
        gemm(xc, w.contiguous(), y, M, Nout, K, lda=K, ldb=K, ldc=Nout, dtype=F32, c_dtype=F32, bias=b)
        ctx.save_for_backward(xc, w)
        ctx.shp, ctx.has_bias = shp, b is not None
        return y.view(*shp[:-1], Nout)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        M, K = x.shape
        Nout = w.shape[0]
        pool = Pool(dy.device)
        # the GEMM wants 16-B leading dimensions: pad the output features (n_classes) to 4
        Np = (Nout + 3) // 4 * 4
        dy2 = dy.float().reshape(M, Nout)
        if Np != Nout:
            dyp = torch.zeros(M, Np, device=dy.device)
            dyp[:, :Nout] = dy2
            wp = torch.zeros(Np, K, device=dy.device)
            wp[:Nout] = w
        else:
            dyp, wp = dy2.contiguous(), w.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(M, K, device=dy.device)
            gemm(dyp, wp, dx, M, K, Np, lda=Np, ldb=K, ldc=K, b_kn=1, dtype=F32, c_dtype=F32)
            dx = dx.view(ctx.shp)
        dw = torch.empty(Np, K, device=dy.device)
        weight_grad(dyp, x, dw, Np, K, M, ldy=Np, ldx=K, dtype=F32, work_pool=pool)
        db = None
        if ctx.has_bias:
            db = torch.empty(Np, device=dy.device)
            colsum(dyp, M, Np, Np, F32, db, pool)
            db = db[:Nout]
        return dx, dw[:Nout], db


def linear(module, x):
    """``nn.Linear`` forward on the HIP GEMM (x [..., K] fp32; bias optional)."""
    if not x.is_cuda:
        raise RuntimeError("HIP Linear needs a GPU tensor")
    return _LinearFn.apply(x.float(), module.weight, module.bias)
