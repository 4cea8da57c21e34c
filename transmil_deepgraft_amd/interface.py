"""The Lightning-step surface of the hot path, without Lightning.

Mirrors the pieces of ``ModelInterface`` (code/models/model_interface.py:108)
that the TransMIL training step runs, with the same hook names and argument
meaning, so a Lightning user can swap the model in and a plain loop can drive
it on MI355X:

* ``create_loss``       -- ``nn.CrossEntropyLoss()`` (code/MyLoss/loss_factory.py:21-62; soft
                           one-hot target as at model_interface.py:346-347)
* ``add_weight_decay`` / ``create_optimizer`` -- no-decay groups + RAdam, optionally
                           wrapped in Lookahead (code/MyOptimizer/optim_factory.py:25-123)
* ``Lookahead``         -- k-step slow-weight wrapper (alpha 0.5, k 6; multi-tensor ops)
* ``GradAllReduce``     -- the DDP gradient all-reduce (Lightning DDP, code/train.py:178-201):
                           one flat fp32 bucket, averaged over ranks with one RCCL
                           all_reduce over xGMI (the model is 9.64 MB of fp32 grads)
* ``TransMILTask``      -- ``training_step`` / ``configure_optimizers`` with the reference's
                           batch format ``(bags[B,n,F], labels[B], (names, patients))``
"""
from __future__ import annotations

from collections import defaultdict

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


def create_loss(base_loss: str = "CrossEntropyLoss") -> nn.Module:
    if not hasattr(nn, base_loss):
        raise ValueError(f"unsupported loss {base_loss}")
    return getattr(nn, base_loss)()


def add_weight_decay(model: nn.Module, weight_decay: float = 1e-5, skip_list=()):
    """1-D tensors and ``.bias`` -> no decay (optim_factory.py:25-37)."""
    decay, no_decay = [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (no_decay if p.dim() == 1 or name.endswith(".bias") or name in skip_list else decay).append(p)
    return [{"params": no_decay, "weight_decay": 0.0}, {"params": decay, "weight_decay": weight_decay}]


class Lookahead(torch.optim.Optimizer):
    """Every k inner steps: slow += alpha * (fast - slow); fast = slow.

    Same schedule as the reference wrapper (code/MyOptimizer/lookahead.py; the
    first sync only initialises the slow weights), but branch-free on the device:
    the step counter and the "slow weights initialised" flag are device scalars
    and the update is masked, so the whole optimizer step can be captured in a
    hipGraph and replayed."""

    def __init__(self, base: torch.optim.Optimizer, alpha: float = 0.5, k: int = 6):
        if not 0.0 <= alpha <= 1.0 or k < 1:
            raise ValueError("Lookahead: alpha in [0,1], k >= 1")
        self.base_optimizer = base
        self.param_groups = base.param_groups
        self.defaults = dict(base.defaults, lookahead_alpha=alpha, lookahead_k=k, lookahead_step=0)
        self.state = defaultdict(dict)
        self._dev = None
        for g in self.param_groups:
            g.setdefault("lookahead_alpha", alpha)
            g.setdefault("lookahead_k", k)
            g.setdefault("lookahead_step", 0)

    @torch.no_grad()
    def _sync_group(self, gi, g):
        fast = [p for p in g["params"] if p.grad is not None]
        if not fast:
            return
        key = ("group", gi)
        st = self.state[key]
        if "slow" not in st:
            dev = fast[0].device
            st["slow"] = [torch.zeros_like(p) for p in fast]
            st["step"] = torch.zeros((), device=dev)
            st["init"] = torch.zeros((), device=dev)
        slow, step, init = st["slow"], st["step"], st["init"]
        step.add_(1.0)
        m = (torch.remainder(step, float(g["lookahead_k"])) == 0).float()
        coef = m * (1.0 - init * (1.0 - g["lookahead_alpha"]))
        diff = torch._foreach_sub(fast, slow)
        torch._foreach_add_(slow, torch._foreach_mul(diff, coef))
        back = torch._foreach_sub(slow, fast)
        torch._foreach_add_(fast, torch._foreach_mul(back, m))
        torch.maximum(init, m, out=init)

    def step(self, closure=None):
        loss = self.base_optimizer.step(closure)
        for gi, g in enumerate(self.param_groups):
            g["lookahead_step"] += 1
            self._sync_group(gi, g)
        return loss

    def zero_grad(self, set_to_none: bool = True):
        self.base_optimizer.zero_grad(set_to_none=set_to_none)


def create_optimizer(model: nn.Module, opt: str = "lookahead_radam", lr: float = 2e-4,
                     weight_decay: float = 0.01, eps=None, betas=None):
    """optim_factory.create_optimizer for the optimizers TransMIL configs use (radam / adam / adamw / sgd)."""
    params = add_weight_decay(model, weight_decay) if weight_decay else model.parameters()
    kw = dict(lr=lr, weight_decay=0.0)
    if eps is not None:
        kw["eps"] = eps
    if betas is not None:
        kw["betas"] = betas
    parts = opt.lower().split("_")
    name = parts[-1]
    fused = torch.cuda.is_available()
    if name == "radam":
        base = torch.optim.RAdam(params, foreach=True, capturable=fused, **kw)
    elif name == "adam":
        base = torch.optim.Adam(params, foreach=not fused, fused=fused, **kw)
    elif name == "adamw":
        base = torch.optim.AdamW(params, foreach=not fused, fused=fused, **kw)
    elif name == "sgd":
        kw.pop("eps", None)
        base = torch.optim.SGD(params, momentum=0.9, nesterov=True, **kw)
    else:
        raise ValueError(f"optimizer {opt} not supported on this path")
    if len(parts) > 1 and parts[0] == "lookahead":
        return Lookahead(base)
    return base


class GradAllReduce:
    """Average gradients over ranks: one flat fp32 bucket, one all_reduce (RCCL on ROCm).

    Replaces the Lightning DDP reducer (``strategy='ddp_find_unused_parameters_true'``,
    code/train.py:184).  Every TransMIL parameter receives a gradient each step, so
    the unused-parameter search is unnecessary; the bucket is sized to the whole
    model (9.64 MB fp32 for 2 classes) because xGMI ring steps are per-link
    bound and one large message beats several small ones.
    """

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.empty(n, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()

    def __call__(self):
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(self.group) == 1:
            return
        grads = [p.grad for p in self.params]
        torch._foreach_copy_(self.views, grads)
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        self.flat.mul_(1.0 / dist.get_world_size(self.group))
        torch._foreach_copy_(grads, self.views)


class TransMILTask(nn.Module):
    """``ModelInterface`` training-step subset for the feature-bag path."""

    def __init__(self, model: nn.Module, lr: float = 2e-4, opt: str = "lookahead_radam",
                 weight_decay: float = 0.01, loss: str = "CrossEntropyLoss"):
        super().__init__()
        self.model = model
        self.n_classes = model.n_classes
        self.loss = create_loss(loss)
        self.lr, self.opt, self.weight_decay = lr, opt, weight_decay
        self._last_loss = None

    def forward(self, x):
        return self.model(x)

    def step(self, bags):
        logits = self(bags.float().contiguous())
        y_hat = torch.argmax(logits, dim=1)
        y_prob = F.softmax(logits, dim=1)
        return logits, y_prob, y_hat

    def training_step(self, batch):
        bags, label, _ = batch
        logits, y_prob, y_hat = self.step(bags)
        one_hot = F.one_hot(label, num_classes=self.n_classes).float()
        loss = self.loss(logits, one_hot)
        if loss.ndim == 0:
            loss = loss.unsqueeze(0)
        # the reference logs loss.item() with sync_dist every step (model_interface.py:364),
        # a host sync + scalar all-reduce per step; here the value stays on the device.
        self._last_loss = loss.detach()
        return loss

    def configure_optimizers(self):
        opt = create_optimizer(self.model, self.opt, self.lr, self.weight_decay)
        sched = {"scheduler": torch.optim.lr_scheduler.ReduceLROnPlateau(
            opt.base_optimizer if isinstance(opt, Lookahead) else opt, mode="min", factor=0.5),
            "monitor": "val_loss", "frequency": 10}
        return [opt], [sched]
