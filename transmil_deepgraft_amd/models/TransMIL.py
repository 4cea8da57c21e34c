"""Drop-in ``models/TransMIL.py`` on the MI355X HIP kernels.

Same classes, constructor signatures, ``forward(x, return_attn=False)``
contract and state_dict keys as ``code/models/TransMIL.py`` (TransLayer :19-57,
PPEG :60-75, TransMIL :78-211), so ``ModelInterface.load_model`` /
``instancialize`` (code/models/model_interface.py:1256-1293) and Lightning
checkpoints (``model.``-prefixed keys) work unchanged.

``TransMIL.forward`` runs the whole model -- _fc1 + GELU, grid padding, class
token, TransLayer x2 (LayerNorm, NystromAttention, residual), PPEG and the
class-token head -- as one autograd node whose forward and backward are the
hand-written HIP kernels of ``libtransmil_hip.so`` (``engine.TransMILEngine``).
``compute_dtype`` selects bf16 MFMA operands (default, the benchmark mode) or
fp32 (the parity mode: f32 MFMA, results within fp32 rounding of the CPU
oracle).  There is no CPU / eager fallback: a CPU tensor raises.

Supported _fc1 branches: ``Linear(in, out) + GELU`` for ``in_features`` not in
{2048, 1024, 768} (:128-133, every d=512 config), and the RCC ``in_features = 2048``
branch ``Linear(2048,1024) + GELU + LayerNorm(1024) + Linear(1024,512) + GELU``
(:100-111, the RetCCL-feature config), and the 768 branch (:122-126: two Linear+GELU on the HIP
GEMM with Dropout and HIP LayerNorms, then the engine's pre-embedded-input mode).  The 1024
branch raises, as the reference's does (its LayerNorm(out_features) meets a 1024-wide input,
:117-121).  ``dim_head`` is fixed at 64 by TransLayer (dim // 8, dim = 512).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ..engine import TransMILEngine, NystromEngine, FC1_PLAIN, FC1_RCC2048, FC1_EMBED
from ..nystrom_attention import NystromAttention, AttentionMap
from .. import ops


class TransLayer(nn.Module):
    """``x + NystromAttention(LayerNorm(x))`` (code/models/TransMIL.py:19-57)."""

    def __init__(self, norm_layer=nn.LayerNorm, dim=512):
        super().__init__()
        self.norm = (ops.LayerNorm if norm_layer is nn.LayerNorm else norm_layer)(dim)
        heads = 8
        self.attn = NystromAttention(dim=dim, dim_head=dim // heads, heads=heads, num_landmarks=dim // 2,
                                     pinv_iterations=6, residual=True, dropout=0.7)

    def forward(self, x):
        out, attn = self.attn(self.norm(x), return_attn=True)   # module calls: hooks fire
        return x + out, attn


class PPEG(nn.Module):
    """7x7 + identity + 5x5 + 3x3 depthwise positional encoding (code/models/TransMIL.py:60-75)."""

    def __init__(self, dim=512):
        super().__init__()
        self.proj = nn.Conv2d(dim, dim, 7, 1, 7 // 2, groups=dim)
        self.proj1 = nn.Conv2d(dim, dim, 5, 1, 5 // 2, groups=dim)
        self.proj2 = nn.Conv2d(dim, dim, 3, 1, 3 // 2, groups=dim)

    def forward(self, x, H, W):
        if H != W:
            raise NotImplementedError("PPEG on the HIP path needs a square grid (TransMIL always builds one)")
        return ops.ppeg(self, x, H)


class _TransMILFn(torch.autograd.Function):
    """The fused engine as one autograd node.  ``ce = (label, class_stats)`` (TransMILTask's
    training step): the node also returns the CrossEntropy loss, Y_prob and Y_hat from the head's
    launch, and its backward takes the loss gradient into the head backward's launch."""

    @staticmethod
    def forward(ctx, engine, names, drop_p, seed_dev, holder, bucket, counter, ce, x, *params):
        prm = dict(zip(names, params))
        with torch.cuda.device(x.device):   # kernels go to x's device and its current stream
            logits, c = engine.forward(x, prm, drop_p, seed_dev=seed_dev, counter=counter, ce=ce)
        ctx.engine, ctx.c, ctx.names, ctx.prm, ctx.bucket = engine, c, names, prm, bucket
        if holder is not None:
            holder["ctx"] = c
        if ce is None:
            return logits
        _label, prob, loss, yhat = c["ce"]
        ctx.mark_non_differentiable(prob, yhat)
        ctx.set_materialize_grads(False)    # no zero-filled gradients for unused outputs
        return logits, loss, prob, yhat

    @staticmethod
    def backward(ctx, dlogits, *rest):
        if ctx.c is None:
            raise RuntimeError("TransMIL (fused HIP path): the saved activations were freed by the first "
                               "backward; retain_graph=True is not supported on the fused path -- set "
                               "model.fused = False (module-by-module path) to backpropagate twice")
        head = (None,) * 9
        gloss = rest[0] if rest else None
        bucket, prm = ctx.bucket, ctx.prm
        dl = None if dlogits is None else dlogits.float().contiguous()
        dev = ctx.c["H0"].device
        with torch.cuda.device(dev):
            if bucket is not None and all(p.grad is None for p in prm.values()):
                # first micro-batch after zero_grad: the kernels write straight into the bucket and
                # the parameters' .grad become its views (stable addresses: hipGraph-safe, no copy)
                views = {n: bucket.view(p) for n, p in prm.items()}
                dx = ctx.engine.backward(dl, ctx.c, prm, out=views, ready=bucket.ready,
                                         gloss=gloss, parts=len(bucket.ranges)).pop("__dx__", None)
                ctx.c = None
                with torch.no_grad():
                    for n, p in prm.items():
                        p.grad = views[n]
                return head[:8] + (dx,) + (None,) * len(ctx.names)
            g = ctx.engine.backward(dl, ctx.c, prm, gloss=gloss)
            dx = g.pop("__dx__", None)
            ctx.c = None
            if bucket is not None and all(bucket.owns(p) for p in prm.values()):
                # gradient accumulation (accumulate_grad_batches > 1): add into the bucket views
                with torch.no_grad():
                    torch._foreach_add_([p.grad for p in prm.values()], [g[n] for n in ctx.names])
                for i in range(len(bucket.ranges)):
                    bucket.ready(i)
                return head[:8] + (dx,) + (None,) * len(ctx.names)
        return head[:8] + (dx,) + tuple(g[n] for n in ctx.names)


class TransMIL(nn.Module):
    def __init__(self, n_classes, in_features, out_features=512):
        super().__init__()
        norm_layer = ops.LayerNorm     # nn.LayerNorm parameters, HIP forward (hookable)
        self.pos_layer = PPEG(dim=out_features)
        if in_features in (2048, 1024, 768):
            self._fc1 = _reference_fc1(in_features, out_features, norm_layer)
        else:
            self._fc1 = nn.Sequential(nn.Linear(in_features, out_features), nn.GELU())
        self.cls_token = nn.Parameter(torch.randn(1, 1, out_features))
        self.n_classes = n_classes
        self.in_features = in_features
        self.layer1 = TransLayer(norm_layer=norm_layer, dim=out_features)
        self.layer2 = TransLayer(norm_layer=norm_layer, dim=out_features)
        self.norm = norm_layer(out_features)
        self._fc = nn.Linear(out_features, self.n_classes)
        self.compute_dtype = torch.bfloat16
        # dropout stream: a device-side counter advanced by every train-mode forward
        # (hipGraph-safe); seeded from torch's generator so torch.manual_seed pins it
        self.register_buffer("_dropout_counter", torch.randint(0, 2 ** 62, (1,), dtype=torch.int64),
                             persistent=False)

    # False: always run module by module (what a hook on a submodule switches to by itself)
    fused = True
    _grad_bucket = None   # interface.GradBucket the fused backward writes into (attach_grad_bucket)
    _head = "_fc"     # class-token Linear (code/models/TransMIL.py:155)

    def _fc1_layout(self):
        if len(self._fc1) == 2:
            return FC1_PLAIN
        if self.in_features == 2048 and len(self._fc1) == 5:
            return FC1_RCC2048
        if self.in_features == 768 and len(self._fc1) == 8:
            return FC1_EMBED
        if self.in_features == 1024:
            raise NotImplementedError(
                "in_features=1024: the reference's branch (code/models/TransMIL.py:117-121) applies "
                "LayerNorm(out_features=512) to a 1024-wide activation and fails; it has no HIP path")
        raise NotImplementedError(
            f"in_features={self.in_features}: only the Linear+GELU (code/models/TransMIL.py:128-133), "
            "in_features=2048 (:100-111) and in_features=768 (:122-126) _fc1 branches run on the HIP path")

    def _pre_embed(self, x):
        """The 768 branch (code/models/TransMIL.py:122-126) on the HIP ops: Linear(768,768)+GELU,
        Dropout(0.6), LayerNorm(768), Linear(768,512)+GELU, Dropout(0.6), LayerNorm(512)."""
        f = self._fc1
        h = ops.linear_gelu(f[0], x)
        h = f[2](h)
        h = f[3](h)
        h = ops.linear_gelu(f[4], h)
        h = f[6](h)
        return f[7](h)

    def _engine_params(self, layout):
        """(names the engine reads, parameters): every parameter, minus an _fc1 the engine does
        not run (pre-embedded input)."""
        named = [(n, p) for n, p in self.named_parameters()
                 if not (layout is FC1_EMBED and n.startswith("_fc1."))]
        return tuple(n for n, _ in named), tuple(p for _, p in named)

    def grad_bucket_parts(self, split_layer1=False):
        """Parameters in the order their gradients become final in the fused backward: part 0 =
        head, norm, layer2, PPEG (ready before layer1's backward starts), part 1 = layer1,
        class token, _fc1.  ``split_layer1`` (world > 1): part 1 = layer1 alone (ready before the
        _fc1 backward starts, so its all-reduce overlaps it) and part 2 = class token, _fc1."""
        first = (self._head + ".", "norm.", "layer2.", "pos_layer.")
        named = list(self.named_parameters())
        p0 = [p for n, p in named if n.startswith(first)]
        rest = [(n, p) for n, p in named if not n.startswith(first)]
        if not split_layer1:
            return [p0, [p for _, p in rest]]
        return [p0, [p for n, p in rest if n.startswith("layer1.")], [p for n, p in rest if not n.startswith("layer1.")]]

    def attach_grad_bucket(self, bucket):
        """Route the fused backward's parameter gradients into ``bucket`` (interface.GradBucket).
        Not with a pre-embedded input: its _fc1 gradients come later, from autograd."""
        self._grad_bucket = None if self._fc1_layout() is FC1_EMBED else bucket

    def _hooked(self):
        """A forward / backward hook on any submodule (GradCAM on model.norm or
        model.layer{1,2}.norm, code/visualize_mil.py:225-234) needs the module-by-module path."""
        g = torch.nn.modules.module
        if any(getattr(g, n, None) for n in ("_global_forward_hooks", "_global_forward_pre_hooks",
                                              "_global_backward_hooks", "_global_backward_pre_hooks")):
            return True
        # a plain stack walk of the submodule tree (Module.modules()' generator chain with its memo
        # set was ~60 us of the eager step's host path)
        stack = list(self._modules.values())
        while stack:
            m = stack.pop()
            if m is None:
                continue
            if m._forward_hooks or m._forward_pre_hooks or m._backward_hooks or getattr(m, "_backward_pre_hooks", None):
                return True
            stack.extend(m._modules.values())
        return False

    def _forward_modules(self, x, return_attn):
        """code/models/TransMIL.py:175-211 as module calls on the HIP ops, so hooks on
        ``norm``, ``layer{1,2}.norm``, ``layer{1,2}``, ``pos_layer`` ... fire: _fc1 + pad +
        class token, layer1, PPEG, layer2, norm (all S tokens), _fc on the class token."""
        B, N, _ = x.shape
        G = int(math.ceil(math.sqrt(N)))
        layout = self._fc1_layout()
        if layout is FC1_RCC2048:           # :101-110 inner Linear + GELU + LayerNorm
            x = ops.linear_gelu(self._fc1[0], x)
            x = self._fc1[2](x)
            h = ops.embed(self._fc1[3], self.cls_token, x)
        elif layout is FC1_EMBED:
            x = self._pre_embed(x)
            add = G * G - N
            h = torch.cat([self.cls_token.expand(B, -1, -1), x, x[:, :add]], dim=1)
        else:
            h = ops.embed(self._fc1[0], self.cls_token, x)   # :175-186
        h, _ = self.layer1(h)                           # :196
        h = self.pos_layer(h, G, G)                     # :198
        h, attn = self.layer2(h)                        # :199
        h = self.norm(h)[:, 0]                          # :202-203
        logits = ops.linear(getattr(self, self._head), h)   # :204
        if return_attn:
            S = G * G + 1
            return logits, (attn, 256 - S % 256 if S % 256 else 0)
        return logits

    def set_compute_dtype(self, dtype):
        """torch.bfloat16 (bench) or torch.float32 (parity); propagates to submodules."""
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("compute dtype must be torch.bfloat16 or torch.float32")
        self.compute_dtype = dtype
        for m in self.modules():
            if isinstance(m, NystromAttention):
                m.compute_dtype = dtype
        return self

    def forward(self, x, return_attn=False):
        if x.dim() > 3:                        # :170-173
            x = x.squeeze(0)
        elif x.dim() == 2:
            x = x.unsqueeze(0)
        if not x.is_cuda:
            raise RuntimeError("TransMIL (HIP) needs a GPU tensor: there is no CPU path")
        layout = self._fc1_layout()
        x = x.float().contiguous()             # :174
        if not self.fused or self._hooked() or x.requires_grad:
            # hooks, or a gradient w.r.t. the input (feature saliency): the module-by-module path,
            # whose ops also return dL/dx; the fused node returns parameter gradients only
            return self._forward_modules(x, return_attn)
        if layout is FC1_EMBED:
            x = self._pre_embed(x).contiguous()
        return self._fused(x, layout, return_attn)

    def forward_ce(self, x, label, class_stats=None):
        """The training step's forward + CrossEntropyLoss(logits, one_hot(label).float()) with
        Y_prob / Y_hat / the per-class count-correct (code/models/model_interface.py:333-356) on
        the fused path, the loss computed in the head's launch: returns (logits, loss, Y_prob,
        Y_hat), or None where the fused path does not apply (hooks, input gradients,
        ``fused = False``) -- the caller then runs ``forward`` and the loss itself."""
        if x.dim() > 3:
            x = x.squeeze(0)
        elif x.dim() == 2:
            x = x.unsqueeze(0)
        if not x.is_cuda:
            raise RuntimeError("TransMIL (HIP) needs a GPU tensor: there is no CPU path")
        layout = self._fc1_layout()
        x = x.float().contiguous()
        if not self.fused or self._hooked() or x.requires_grad or self._forward_hooks or self._forward_pre_hooks:
            # hooks on this module itself run only through __call__: the caller's self(x) path
            return None
        if layout is FC1_EMBED:
            x = self._pre_embed(x).contiguous()
        if not label.is_cuda and label.numel() and not (0 <= int(label.min()) and int(label.max()) < self.n_classes):
            raise IndexError(f"forward_ce: labels must lie in [0, {self.n_classes})")   # as F.one_hot
        lab = label.reshape(-1).to(device=x.device, dtype=torch.int64).contiguous()
        if lab.numel() != x.shape[0]:
            raise ValueError(f"forward_ce: {lab.numel()} labels for {x.shape[0]} bags")
        return self._fused(x, layout, False, ce=(lab, class_stats))

    def _fused(self, x, layout, return_attn, ce=None):
        """The fused engine node: x [B, N, F] (F = D for a pre-embedded input) -> logits
        (with ``ce``: logits, loss, Y_prob, Y_hat)."""
        names, params = self._engine_params(layout)
        drop_p = self.layer1.attn.to_out[1].p if self.training else 0.0
        seed_dev = None
        if drop_p > 0:
            # this forward's seed: the engine's preparation launch advances the device counter and
            # writes the new value here (the snapshot its backward replays)
            seed_dev = torch.empty(1, dtype=torch.int64, device=x.device)
        holder = {} if return_attn else None
        engine = TransMILEngine(self.compute_dtype, fc1=layout, head=self._head)
        out = _TransMILFn.apply(engine, names, drop_p, seed_dev, holder, self._grad_bucket,
                                self._dropout_counter if drop_p > 0 else None, ce, x, *params)
        if ce is not None:
            return out
        logits = out
        if return_attn:
            c = holder["ctx"]
            S = c["geo"].S
            padding = 256 - S % 256 if S % 256 else 0      # :190-193
            attn2 = AttentionMap(c["s2"]["qkv"], c["s2"]["core"], c["geo"].heads)
            return logits, (attn2, padding)
        return logits


def _reference_fc1(in_features, out_features, norm_layer):
    """Parameter layout of the other _fc1 branches (:100-126), kept so their
    checkpoints load (the 2048 and 768 branches run on the HIP path, the 1024 one raises as in
    the reference)."""
    if in_features == 2048:
        return nn.Sequential(nn.Linear(in_features, in_features // 2), nn.GELU(), norm_layer(in_features // 2),
                             nn.Linear(in_features // 2, out_features), nn.GELU())
    if in_features == 1024:
        return nn.Sequential(nn.Linear(in_features, in_features), nn.GELU(), nn.Dropout(p=0.2),
                             norm_layer(out_features), nn.Linear(in_features, out_features), nn.GELU(),
                             nn.Dropout(p=0.6), norm_layer(out_features))
    return nn.Sequential(nn.Linear(in_features, in_features), nn.GELU(), nn.Dropout(p=0.6),
                         norm_layer(in_features), nn.Linear(in_features, out_features), nn.GELU(),
                         nn.Dropout(p=0.6), norm_layer(out_features))

