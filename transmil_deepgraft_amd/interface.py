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
* ``FusedRAdamLookahead`` -- RAdam + Lookahead for the GPU as one HIP elementwise launch
* ``GradBucket`` / ``GradAllReduce`` -- the DDP gradient all-reduce (Lightning DDP,
                           code/train.py:178-201): gradients live as views of one flat fp32
                           bucket in two parts, each averaged with one RCCL all_reduce over
                           xGMI, part 0 overlapping layer1's backward (9.64 MB of fp32 grads)
* ``TransMILTask``      -- ``training_step`` / ``configure_optimizers`` with the reference's
                           batch format ``(bags[B,n,F], labels[B], (names, patients))``
"""
from __future__ import annotations

import ctypes as C
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

    def state_dict(self):
        """``{'state': base state, 'slow_state': ..., 'param_groups': ...}`` as the reference
        wrapper saves it (code/MyOptimizer/lookahead.py:56-68); the slow state is keyed by group
        index and also carries the device step counter and init flag."""
        fast = self.base_optimizer.state_dict()
        slow = {}
        for (_, gi), st in self.state.items():
            slow[gi] = {"slow": [t.detach().clone() for t in st["slow"]],
                        "step": st["step"].detach().clone(), "init": st["init"].detach().clone()}
        return {"state": fast["state"], "slow_state": slow, "param_groups": fast["param_groups"]}

    def load_state_dict(self, state_dict):
        """Restores the base optimizer (its moments and the lookahead_* group fields) and the
        slow weights with their step counter / init flag (lookahead.py:70-88)."""
        self.base_optimizer.load_state_dict({"state": state_dict["state"],
                                             "param_groups": state_dict["param_groups"]})
        self.param_groups = self.base_optimizer.param_groups
        self.state = defaultdict(dict)
        for gi, st in state_dict.get("slow_state", {}).items():
            dev = self.param_groups[int(gi)]["params"][0].device
            self.state[("group", int(gi))] = {"slow": [t.to(dev).clone() for t in st["slow"]],
                                              "step": st["step"].to(dev).clone(),
                                              "init": st["init"].to(dev).clone()}


class FusedRAdamLookahead(torch.optim.Optimizer):
    """``Lookahead(torch.optim.RAdam(groups))`` as ONE HIP launch pair per step.

    Same update as ``torch.optim.RAdam`` (L2 weight decay folded into the gradient,
    ``decoupled_weight_decay=False``; code/MyOptimizer/optim_factory.py:77-79) followed
    by the reference Lookahead sync every ``k`` steps (code/MyOptimizer/lookahead.py,
    wrapped at optim_factory.py:118-121; ``lookahead_k=0`` gives plain RAdam).  The
    moments and slow weights of every parameter live in three flat fp32 buffers, the
    step counters on the device, and the kernel reads each parameter/gradient through
    a pointer table passed by value (``tm_radam_lookahead_step``, csrc/optim.hip), so
    the step is hipGraph-capturable.  ``lr`` / ``weight_decay`` reach the kernel through a
    small device array (``tm_optim_table.hyper``) that every eager step -- and, before each
    replay, ``GraphedOptimizationStep`` via ``refresh_hyper()`` -- rewrites from the groups, so an
    LR scheduler (``configure_optimizers``' ReduceLROnPlateau) also acts on a replayed graph."""

    def __init__(self, params, lr=2e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 lookahead_alpha=0.5, lookahead_k=6):
        if not 0.0 <= lookahead_alpha <= 1.0 or lookahead_k < 0:
            raise ValueError("Lookahead: alpha in [0,1], k >= 0")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                        lookahead_alpha=lookahead_alpha, lookahead_k=lookahead_k, lookahead_step=0)
        super().__init__(params, defaults)
        from . import _lib
        self._lib = _lib
        plist = [p for g in self.param_groups for p in g["params"]]
        if any(p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous() for p in plist):
            raise ValueError("fused RAdam: parameters must be contiguous fp32 CUDA tensors")
        for g in self.param_groups:
            for key in ("betas", "eps", "lookahead_alpha", "lookahead_k"):
                if g[key] != self.param_groups[0][key]:
                    raise ValueError(f"fused RAdam: '{key}' must be equal across groups")
        self._all = plist
        self._params = None     # the parameters that receive gradients: fixed at the first step

    def _activate(self, plist):
        """Lay the state of ``plist`` (the parameters with a gradient, in group order) out in three
        flat fp32 buffers.  Parameters that never receive a gradient (modules kept only for the
        state_dict, e.g. CTMIL._fc1) are skipped, as torch.optim.RAdam skips ``grad is None``."""
        if len(plist) > self._lib.OPTIM_MAX_TENSORS:
            raise ValueError(f"fused RAdam: at most {self._lib.OPTIM_MAX_TENSORS} parameter tensors with "
                             "gradients (create_optimizer falls back to torch.optim.RAdam above that)")
        if not plist:
            raise RuntimeError("fused RAdam: no parameter has a gradient")
        self._params = plist
        self._index = {id(p): i for i, p in enumerate(plist)}
        total = sum((p.numel() + 3) // 4 * 4 for p in plist)
        dev = plist[0].device
        self._flat = torch.zeros(3, total, dtype=torch.float32, device=dev)  # exp_avg, exp_avg_sq, slow
        # one (RAdam step, Lookahead step) pair per workgroup of the update launch; pair 0 is checkpointed
        self._counters = torch.zeros(max(3, int(self._lib.query("tm_radam_counters_len", total))),
                                     dtype=torch.int32, device=dev)
        self._offsets = [0]
        for p in plist:     # each tensor's flat state padded to a multiple of 4 (16-B vectors)
            self._offsets.append(self._offsets[-1] + (p.numel() + 3) // 4 * 4)
        self._hyper = torch.zeros(len(plist), 2, dtype=torch.float32, device=dev)   # (lr, weight_decay)
        self._hyper_host = None
        self._bind_state()

    def _hyper_values(self):
        vals = []
        for g in self.param_groups:
            for p in g["params"]:
                if id(p) in self._index:
                    vals.append((float(g["lr"]), float(g["weight_decay"])))
        return vals

    @torch.no_grad()
    def refresh_hyper(self):
        """Write the groups' current lr / weight_decay into the device array the update kernel reads
        (a no-op when they have not changed).  Must run outside stream capture: a captured step
        reads whatever the array holds when it is replayed."""
        if self._params is None:
            return
        vals = self._hyper_values()
        if vals != self._hyper_host:
            self._hyper.copy_(torch.tensor(vals, dtype=torch.float32))
            self._hyper_host = vals

    def _bind_state(self):
        for i, p in enumerate(self._params):
            a, b = self._offsets[i], self._offsets[i] + p.numel()
            self.state[p] = {"exp_avg": self._flat[0, a:b].view_as(p),
                             "exp_avg_sq": self._flat[1, a:b].view_as(p),
                             "slow_buffer": self._flat[2, a:b].view_as(p)}

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = self._lib
        if self._params is None:
            self._activate([p for p in self._all if p.grad is not None])
        if not torch.cuda.is_current_stream_capturing():
            self.refresh_hyper()
        tab = lib.OptimTable()
        tab.hyper = self._hyper.data_ptr()
        tab.count = len(self._params)
        i = 0
        for g in self.param_groups:
            for p in g["params"]:
                if id(p) not in self._index:
                    if p.grad is not None:
                        raise RuntimeError("fused RAdam: a parameter without a gradient at the first step has "
                                           "one now (its step count would differ from torch.optim.RAdam's); "
                                           "use opt='radam' on a model whose parameter set is fixed")
                    continue
                if p.grad is None:
                    raise RuntimeError("fused RAdam: a parameter that had a gradient at the first step has "
                                       "none now")
                t = tab.t[i]
                t.param, t.grad, t.numel = p.data_ptr(), p.grad.data_ptr(), p.numel()
                t.lr, t.weight_decay = float(g["lr"]), float(g["weight_decay"])
                tab.offset[i] = self._offsets[i]
                i += 1
            g["lookahead_step"] += 1
        tab.offset[i] = self._offsets[i]
        g0 = self.param_groups[0]
        b1, b2 = g0["betas"]
        lib.call("tm_radam_lookahead_step", C.byref(tab), self._flat[0].data_ptr(), self._flat[1].data_ptr(),
                 self._flat[2].data_ptr(), self._counters.data_ptr(), float(b1), float(b2), float(g0["eps"]),
                 int(g0["lookahead_k"]), float(g0["lookahead_alpha"]),
                 torch.cuda.current_stream(self._flat.device).cuda_stream)
        return loss

    def state_dict(self):
        sd = super().state_dict()
        if self._params is not None:
            sd["fused_counters"] = self._counters[:3].cpu()
        return sd

    def load_state_dict(self, state_dict):
        counters = state_dict.get("fused_counters")
        super().load_state_dict({k: v for k, v in state_dict.items() if k != "fused_counters"})
        with torch.no_grad():
            loaded = {p: {k: v.detach().clone() for k, v in self.state[p].items() if torch.is_tensor(v)}
                      for p in self._all if p in self.state}
            if self._params is None:
                stateful = [p for p in self._all if "exp_avg" in loaded.get(p, {})]
                if not stateful:
                    return
                self._activate(stateful)
            self._bind_state()
            self._hyper_host = None
            for i, p in enumerate(self._params):
                st = loaded.get(p, {})
                a, b = self._offsets[i], self._offsets[i] + p.numel()
                for row, key in enumerate(("exp_avg", "exp_avg_sq", "slow_buffer")):
                    if key in st:
                        self._flat[row, a:b].copy_(st[key].reshape(-1))
            if counters is not None:
                self._counters.zero_()
                npairs = self._counters.numel() // 2
                self._counters[:2 * npairs].view(npairs, 2).copy_(counters[:2].to(self._counters).expand(npairs, 2))


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
    on_gpu = fused and all(p.is_cuda for p in model.parameters())
    n_tensors = sum(1 for p in model.parameters() if p.requires_grad)
    if name == "radam" and on_gpu and n_tensors <= _lib_max_tensors():
        la = len(parts) > 1 and parts[0] == "lookahead"
        return FusedRAdamLookahead(params, lookahead_k=6 if la else 0, **kw)
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


def _lib_max_tensors():
    from . import _lib
    return _lib.OPTIM_MAX_TENSORS


class GradBucket:
    """One flat fp32 buffer that holds every parameter gradient as a view, laid out in parts in
    the order the fused backward finishes them (``TransMIL.grad_bucket_parts``).

    The fused backward writes its gradient kernels' outputs straight into these views and
    sets ``p.grad`` to them (models/TransMIL.py ``_TransMILFn.backward``), so the bucket IS
    the gradient storage: no copy in or out around the all-reduce, and the addresses are
    stable across steps (a captured hipGraph and the fused optimizer's pointer table stay
    valid).  ``ready(i)`` is called by the backward when part ``i`` is final; ``hooks`` get it."""

    def __init__(self, parts, device=None):
        self.parts_params = [list(part) for part in parts if part]
        self.params = [p for part in self.parts_params for p in part]
        if len({id(p) for p in self.params}) != len(self.params):
            raise ValueError("GradBucket: a parameter appears in two parts")
        dev = device if device is not None else self.params[0].device
        self._off = {}
        self.ranges = []
        off = 0
        for i, part in enumerate(self.parts_params):
            start = off
            for p in part:
                self._off[id(p)] = (off, p.numel())
                off += (p.numel() + 15) // 16 * 16     # every view 64-B aligned (vector stores)
            if i == len(self.parts_params) - 1:
                # the has-gradient flags (one float per parameter) ride at the end of the last part, so
                # the unused-parameter exchange is part of that part's all_reduce (no collective of its own)
                self._flag_off = off
                off += (len(self.params) + 15) // 16 * 16
            self.ranges.append((start, off))
        self.flat = torch.zeros(off, dtype=torch.float32, device=dev)
        # > 0 on every rank that has not written them: averaging keeps them > 0 (see GradAllReduce)
        self.flags = self.flat[self._flag_off:self._flag_off + len(self.params)]
        self.flags.fill_(1.0)
        self.hooks = []

    def view(self, p):
        """A fresh view of ``p``'s slice (fresh, so autograd could steal it without a clone)."""
        o, n = self._off[id(p)]
        return self.flat[o:o + n].view_as(p)

    def owns(self, p):
        """True when ``p.grad`` is this bucket's view of ``p``."""
        g = p.grad
        if g is None or id(p) not in self._off:
            return False
        o, _ = self._off[id(p)]
        return g.data_ptr() == self.flat.data_ptr() + 4 * o and g.shape == p.shape

    def part(self, i):
        a, b = self.ranges[i]
        return self.flat[a:b]

    def bind(self):
        """Make every existing ``p.grad`` the bucket's view (keeps its values by copying them in).
        A parameter without a gradient (a module kept only for the state_dict) keeps ``None``, so
        the optimizer skips it as torch.optim.RAdam does; its slice is zeroed and sums zeros."""
        with torch.no_grad():
            for p in self.params:
                if not self.owns(p):
                    v = self.view(p)
                    if p.grad is None:
                        v.zero_()
                    else:
                        v.copy_(p.grad)
                        p.grad = v

    def ready(self, i):
        for h in self.hooks:
            h(i)


class GradAllReduce:
    """Average gradients over ranks: the DDP gradient all-reduce on a ``GradBucket``.

    Replaces the Lightning DDP reducer (``strategy='ddp_find_unused_parameters_true'``,
    code/train.py:184).  On the fused path every TransMIL parameter receives a gradient each step,
    so no unused-parameter search runs; on the module-by-module path the rank's has-gradient flags
    travel in the bucket's own all_reduce (a tail of the last part) and parameters used on another
    rank adopt the averaged gradient.  With ``model=`` (a TransMIL with
    ``grad_bucket_parts``) the bucket is cut where the fused backward finishes gradients: part 0
    (head, norm, layer2, PPEG; 4.4 MB fp32) is final before layer1's backward is enqueued and, with
    ``overlap``, its RCCL all_reduce is issued right then on RCCL's stream, overlapping layer1 +
    _fc1 backward on the compute stream.  At world > 1 (``split_layer1``) part 1 is layer1 alone
    (4.2 MB), issued before the _fc1 backward, and part 2 (class token, _fc1 + the flags; 1.05 MB)
    is the only message after the whole backward (``exposed_bytes``); at world 1 (no collective)
    layer1 and _fc1 stay one part (5.2 MB), which saves the extra flush launch.  Few ~1-5 MB
    messages keep each xGMI ring step large (per-link bound).

    ``sync = False`` skips the reduction (Lightning's no-sync micro-batches under
    ``accumulate_grad_batches``, code/train.py:199); ``force`` runs the collective even at
    world size 1 (tests of the RCCL path inside a captured hipGraph)."""

    def __init__(self, params, group=None, model=None, overlap=True, force=False, split_layer1=None):
        self.params = [p for p in params if p.requires_grad]
        self.group, self.overlap, self.force = group, overlap, force
        if split_layer1 is None:
            # a third part only where a collective runs: at world 1 its extra flush launch buys nothing
            split_layer1 = self._world() > 1
        parts = [self.params]
        if model is not None and hasattr(model, "grad_bucket_parts"):
            try:
                mp = model.grad_bucket_parts(split_layer1=True) if split_layer1 else model.grad_bucket_parts()
            except TypeError:       # a model whose bucket layout has no layer1 cut
                mp = model.grad_bucket_parts()
            if {id(p) for part in mp for p in part} == {id(p) for p in self.params}:
                parts = mp
        self.bucket = GradBucket(parts, self.params[0].device)
        self.flat = self.bucket.flat
        self._model = model
        if model is not None and hasattr(model, "attach_grad_bucket"):
            model.attach_grad_bucket(self.bucket)
        self.bucket.hooks.append(self._on_ready)
        self.sync = True
        self._works = {}
        self._closed = False

    def exposed_bytes(self):
        """fp32 bytes all-reduced after the whole backward (the last part: nothing left to hide it
        behind); the earlier parts are issued from the backward and overlap what follows them."""
        a, b = self.bucket.ranges[-1]
        return 4 * (b - a) if self.overlap else 4 * self.flat.numel()

    def close(self):
        """Release everything that refers to the process group's communicator, BEFORE
        ``dist.destroy_process_group()``: waits on and drops the outstanding async works, detaches
        the bucket hook (the model's bucket keeps a bound method of this object alive) and the model's
        bucket.  A hipGraph captured over this all-reduce holds the communicator's kernels and
        its registered buffers: release it first (``GraphedOptimizationStep.close()`` or
        ``graph.reset()``).  Idempotent; a closed instance raises when called."""
        if self._closed:
            return
        for w in self._works.values():
            w.wait()
        self._works.clear()
        if self._on_ready in self.bucket.hooks:
            self.bucket.hooks.remove(self._on_ready)
        m = self._model
        if m is not None and getattr(m, "_grad_bucket", None) is self.bucket:
            m.attach_grad_bucket(None)
        self._model = None
        self._closed = True

    def _world(self):
        if not (dist.is_available() and dist.is_initialized()):
            return 0
        return dist.get_world_size(self.group)

    def _active(self):
        w = self._world()
        return self.sync and (w > 1 or (w == 1 and self.force))

    def _on_ready(self, i):
        """Backward hook: issue part ``i``'s all_reduce now (async, on RCCL's stream)."""
        if not (self.overlap and self._active()) or i in self._works:
            return
        self._works[i] = dist.all_reduce(self.bucket.part(i), op=dist.ReduceOp.SUM, group=self.group,
                                         async_op=True)

    def __call__(self):
        if self._closed:
            raise RuntimeError("GradAllReduce: called after close()")
        if not self._active():
            self._works.clear()
            return
        owned = all(self.bucket.owns(p) for p in self.params if p.grad is not None)
        local = None
        if not owned:
            # gradients produced outside the fused backward (module-by-module path): bind them, and
            # write this rank's has-gradient flags into the bucket's flag tail.  Every rank issues
            # the same all_reduces in the same order whichever path it took (the fused path's early
            # part-0 reduce from the backward hook included), so ranks on different paths cannot
            # mismatch collectives; the flags are summed with the gradients.
            local = [p.grad is not None for p in self.params]
            self.bucket.bind()
            self.bucket.flags.copy_(torch.tensor(local, dtype=torch.float32))
        for i in range(len(self.bucket.ranges)):
            if i not in self._works:
                self._works[i] = dist.all_reduce(self.bucket.part(i), op=dist.ReduceOp.SUM, group=self.group,
                                                 async_op=True)
        for i in sorted(self._works):
            self._works[i].wait()       # the compute stream waits on RCCL's stream
        self._works.clear()
        self.flat.mul_(1.0 / self._world())
        if local is not None:
            # as DDP's find_unused_parameters: a parameter without a gradient HERE but with one on
            # another rank receives the averaged gradient (its zeroed slice summed with theirs), so
            # the ranks' optimizer steps stay identical; one used on no rank keeps grad None.  A rank
            # on the fused path never writes its flags: they stay > 0 (1 at creation, then averages
            # of positive and non-negative values), i.e. "used".  (Host read: module path only.)
            used = (self.bucket.flags > 0).tolist()
            for p, here, anywhere in zip(self.params, local, used):
                if anywhere and not here:
                    p.grad = self.bucket.view(p)
        # back to "used" for the next step on EVERY rank, whichever path it took: a fused rank never
        # writes its flags, so it would otherwise carry the average forward and, beside a module-path
        # rank that never uses a parameter, halve it each step until it underflows to 0.  (One tiny
        # launch per reducing step; it runs only where a collective runs.)
        self.bucket.flags.fill_(1.0)


class _CrossEntropyOneHot(torch.autograd.Function):
    """CE(logits, one_hot(label).float()) + softmax + argmax as one HIP launch (tm_ce_fwd) and its
    backward as one (tm_ce_bwd), instead of ~17 small PyTorch kernels per step."""

    @staticmethod
    def forward(ctx, logits, label, stats):
        from . import _lib
        from .engine import _p, _stream
        B, C = logits.shape
        lg = logits.float().contiguous()
        lab = label.to(torch.int64).contiguous()
        loss = torch.empty((), device=logits.device)
        prob = torch.empty(B, C, device=logits.device)
        yhat = torch.empty(B, dtype=torch.int64, device=logits.device)
        _lib.call("tm_ce_fwd", _p(lg), _p(lab), B, C, _p(loss), _p(prob), _p(yhat), _p(stats), _stream())
        ctx.save_for_backward(prob, lab)
        ctx.mark_non_differentiable(prob, yhat)
        ctx.set_materialize_grads(False)    # no zero-filled gradients for prob / yhat (two launches)
        return loss, prob, yhat

    @staticmethod
    def backward(ctx, gloss, _gprob, _gyhat):
        from . import _lib
        from .engine import _p, _stream
        if gloss is None:
            return None, None, None
        prob, lab = ctx.saved_tensors
        B, C = prob.shape
        dl = torch.empty(B, C, device=prob.device)
        _lib.call("tm_ce_bwd", _p(prob), _p(lab), B, C, _p(gloss.float().contiguous()), _p(dl), _stream())
        return dl, None, None


class TransMILTask(nn.Module):
    """``ModelInterface`` training-step subset for the feature-bag path."""

    def __init__(self, model: nn.Module, lr: float = 2e-4, opt: str = "lookahead_radam",
                 weight_decay: float = 0.01, loss: str = "CrossEntropyLoss", accumulate_grad_batches: int = 1):
        super().__init__()
        if accumulate_grad_batches < 1:
            raise ValueError("accumulate_grad_batches >= 1")
        self.model = model
        self.class_stats = None     # int32 [C][2] per-class count / correct (model_interface.py:350-356)
        self.accumulate_grad_batches = accumulate_grad_batches
        self._micro = 0
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
        if bags.is_cuda and isinstance(self.loss, nn.CrossEntropyLoss):
            # fused: loss, Y_prob, Y_hat and the per-class count/correct of :350-356 in one launch --
            # the head's own launch where the model offers it (TransMIL.forward_ce), else tm_ce_fwd
            x = bags.float().contiguous()
            if self.class_stats is None or self.class_stats.device != x.device:
                self.class_stats = torch.zeros(self.n_classes, 2, dtype=torch.int32, device=x.device)
            fused = getattr(self.model, "forward_ce", None)
            if self._forward_hooks or self._forward_pre_hooks:
                fused = None            # hooks on the task run only through self(x)
            out = fused(x, label, self.class_stats) if fused is not None else None
            if out is not None:
                logits, loss, y_prob, y_hat = out
            else:
                logits = self(x)
                loss, y_prob, y_hat = _CrossEntropyOneHot.apply(logits, label, self.class_stats)
        else:
            logits, y_prob, y_hat = self.step(bags)
            one_hot = F.one_hot(label, num_classes=self.n_classes).float()
            loss = self.loss(logits, one_hot)
        self._last_outputs = (y_prob, y_hat)
        if loss.ndim == 0:
            loss = loss.unsqueeze(0)
        # the reference logs loss.item() with sync_dist every step (model_interface.py:364),
        # a host sync + scalar all-reduce per step; here the value stays on the device.
        self._last_loss = loss.detach()
        return loss

    def backward(self, loss):
        """``loss.backward()`` with the seed gradient taken from a persistent ones tensor (no
        ``ones_like`` fill launch per step; Lightning's manual_backward equivalent)."""
        one = getattr(self, "_one", None)
        if one is None or one.device != loss.device or one.shape != loss.shape:
            one = self._one = torch.ones_like(loss)
        loss.backward(one)

    def optimization_step(self, batch, opt, allreduce=None):
        """One micro-batch of Lightning's automatic optimization with
        ``accumulate_grad_batches = K`` (code/train.py:199 uses K = 10 under DDP): the closure
        loss is ``training_step / K``, backward accumulates into the gradient bucket, and only
        every K-th micro-batch all-reduces (DDP no-sync before it), steps the optimizer and
        zeroes the gradients.  Returns the un-normalised training_step loss."""
        k = self.accumulate_grad_batches
        self._micro += 1
        boundary = self._micro % k == 0
        if allreduce is not None:
            allreduce.sync = boundary
        loss = self.training_step(batch)
        self.backward(loss / k if k > 1 else loss)
        if boundary:
            if allreduce is not None:
                allreduce()
            opt.step()
            opt.zero_grad(set_to_none=True)
        return loss

    def configure_optimizers(self):
        opt = create_optimizer(self.model, self.opt, self.lr, self.weight_decay)
        sched = {"scheduler": torch.optim.lr_scheduler.ReduceLROnPlateau(
            opt.base_optimizer if isinstance(opt, Lookahead) else opt, mode="min", factor=0.5),
            "monitor": "val_loss", "frequency": 10}
        return [opt], [sched]


class GraphedOptimizationStep:
    """``TransMILTask.optimization_step`` replayed as captured hipGraphs: each micro-batch (forward,
    fused CE, backward into the gradient bucket; on the accumulation boundary also the all-reduce
    and the optimizer step) is ONE graph launch instead of ~100 host-issued kernel launches -- the
    execution ``bench.py`` times, offered to training loops (a graph in place of a tracing
    compiler; an eager step is host-bound at ~2.2 ms on the bench shape against 1.2 ms replayed).

    The first ``accumulate_grad_batches`` micro-batches run eagerly through
    ``task.optimization_step`` (they are real steps: they also create the optimizer state and the
    engine's buffers); then one graph per accumulation phase (``first`` writes the gradients,
    ``mid`` adds, ``last`` adds, all-reduces and steps -- with K = 1 only ``last``, which writes)
    is captured over static input buffers, and every later call copies the batch in and replays
    the phase's graph.  Capture records, it does not execute, so the sequence of updates is the
    eager one (``tests/test_interface.py``: parameters bitwise equal to ``optimization_step``).
    Dropout keeps drawing fresh masks: its counter lives on the device.

    One bag shape per instance (the reference's loaders sample bags to a fixed size); a batch of
    another shape raises.  Returns the training_step loss tensor of the replayed graph (a static
    buffer: it is overwritten by the next call of the same phase).

    Learning rate / weight decay: with ``FusedRAdamLookahead`` the replayed update reads them from
    a device array refreshed from the param groups before every replayed optimizer step, so an LR
    scheduler keeps working; any other optimizer bakes the captured values into the graph, and a
    change of a group's lr / weight_decay after the capture raises instead of being ignored.
    ``lookahead_step`` of every group advances per replayed optimizer step as in the eager path."""

    def __init__(self, task: "TransMILTask", opt, allreduce=None):
        self.task, self.opt, self.allreduce = task, opt, allreduce
        self.k = task.accumulate_grad_batches
        self.graphs = None
        self.shape = None

    def _phase(self, micro):
        k = self.k
        return "last" if micro % k == 0 else ("first" if micro % k == 1 else "mid")

    def _capture(self, bags, label):
        task, opt, ar, k = self.task, self.opt, self.allreduce, self.k
        self.x = bags.detach().clone()
        self.y = label.detach().clone()
        self.loss = {}

        def body(phase):
            if ar is not None:
                ar.sync = phase == "last"
            loss = task.training_step((self.x, self.y, None))
            task.backward(loss / k if k > 1 else loss)
            if phase == "last":
                if ar is not None:
                    ar()
                opt.step()
            return loss

        self._fingerprint = self._hyper_fingerprint()
        la_steps = [g.get("lookahead_step") for g in opt.param_groups]   # capture runs opt.step()'s host side
        pool = torch.cuda.graph_pool_handle()
        self.graphs = {}
        opt.zero_grad(set_to_none=True)        # the first capture takes the writing (=) path,
        for ph in (["last"] if k == 1 else (["first", "mid", "last"] if k > 2 else ["first", "last"])):
            g = torch.cuda.CUDAGraph()          # the ones after it the accumulating (+=) path
            with torch.cuda.graph(g, pool=pool):
                self.loss[ph] = body(ph)
            self.graphs[ph] = g
        for grp, v in zip(opt.param_groups, la_steps):     # ... without a step having run
            if v is not None:
                grp["lookahead_step"] = v

    def _hyper_fingerprint(self):
        return [(g.get("lr"), g.get("weight_decay")) for g in self.opt.param_groups]

    def _before_step_replay(self):
        """The host side of opt.step() that a replay does not run: the fused optimizer's device
        hyper-parameters, the groups' lookahead_step counters; a non-fused optimizer whose lr /
        weight decay changed since the capture raises (its graph holds the old values)."""
        opt = self.opt
        refresh = getattr(opt, "refresh_hyper", None)
        if refresh is not None:
            refresh()
        elif self._hyper_fingerprint() != self._fingerprint:
            raise RuntimeError("GraphedOptimizationStep: lr / weight_decay changed after the capture, and "
                               f"{type(opt).__name__} bakes them into the captured graph (use FusedRAdamLookahead, "
                               "or build a new GraphedOptimizationStep)")
        for g in opt.param_groups:
            if "lookahead_step" in g:
                g["lookahead_step"] += 1

    def close(self):
        """Release the captured graphs, then the all-reduce (``GradAllReduce.close``): a graph
        captured over the RCCL all-reduce holds the communicator's kernels and registered
        buffers, so it must be gone -- destroyed and drained -- before
        ``dist.destroy_process_group()``.  Later calls raise."""
        if self.graphs:
            torch.cuda.synchronize()            # no replay in flight
            for g in self.graphs.values():
                g.reset()
            torch.cuda.synchronize()
        self.graphs, self.loss = None, {}
        self._closed = True
        if self.allreduce is not None:
            self.allreduce.close()

    def __call__(self, batch):
        if getattr(self, "_closed", False):
            raise RuntimeError("GraphedOptimizationStep: called after close()")
        bags, label = batch[0], batch[1]
        task = self.task
        if self.graphs is None:
            if self.shape is None:
                self.shape = (tuple(bags.shape), tuple(label.shape))
            loss = task.optimization_step(batch, self.opt, allreduce=self.allreduce)
            if task._micro % self.k == 0:        # the eager window is complete: capture
                self._capture(bags, label)
            return loss
        if (tuple(bags.shape), tuple(label.shape)) != self.shape:
            raise ValueError(f"GraphedOptimizationStep was captured for bags {self.shape[0]} and labels "
                             f"{self.shape[1]}, got {tuple(bags.shape)} / {tuple(label.shape)}")
        task._micro += 1
        ph = self._phase(task._micro)
        if ph == "last":
            self._before_step_replay()
        self.x.copy_(bags)
        self.y.copy_(label)
        self.graphs[ph].replay()
        return self.loss[ph]
