"""The reference's YAML configuration for this path, without Lightning.

Reads the same files (`Camelyon/TransMIL.yaml`, `DeepGraft/TransMIL_*.yaml`; read_yaml at
code/utils/utils.py:63-66, but with yaml.SafeLoader) and maps the keys `train.py` hands to
`ModelInterface` / the Trainer (code/train.py:118-160, 178-217, 392-397) onto this framework:

* ``Model.name / n_classes / in_features / out_features`` -> ``models.{name}(...)``
  (ModelInterface.load_model, code/models/model_interface.py:1256-1293); ``in_features``
  follows ``Data.feature_extractor`` as train.py:392-397 sets it (retccl 2048, histoencoder 384,
  ctranspath 784), default 1024 as ModelInterface's default.
* ``Model.backbone`` -> ``features`` runs on bags of features; ``retccl`` wraps the model in the
  on-GPU RetCCL encoder (``encoder.ImageBagModel``, model_interface.py:237-247, 300-316).
* ``General.precision`` -> ``compute_dtype``: the reference's 16 / '16-mixed' (fp16 autocast)
  and 'bf16' / 'bf16-mixed' run the bf16 MFMA mode, 32 / '32-true' the fp32 parity mode.
* ``Optimizer.opt / lr / weight_decay``, ``Loss.base_loss`` -> ``TransMILTask``;
  ``General.grad_acc`` -> ``accumulate_grad_batches`` (multi-GPU runs use 10,
  code/train.py:199; single-GPU runs ``grad_acc``, :217).
"""
from __future__ import annotations

import torch
import yaml


class AttrDict(dict):
    """``addict.Dict``-style attribute access (missing keys read as None, as the reference's
    ``cfg.Data.mixup`` etc. do when absent)."""

    def __getattr__(self, key):
        v = self.get(key)
        if isinstance(v, dict) and not isinstance(v, AttrDict):
            v = self[key] = AttrDict(v)      # nested sections stay the same object (writable)
        return v

    def __setattr__(self, key, value):
        self[key] = value


def read_yaml(path) -> AttrDict:
    with open(path) as f:
        return AttrDict(yaml.load(f, Loader=yaml.SafeLoader) or {})


_FEATURE_WIDTH = {"retccl": 2048, "histoencoder": 384, "ctranspath": 784}


def compute_dtype_for(precision) -> torch.dtype:
    """Lightning precision flag -> the engine's compute dtype."""
    p = str(precision).lower() if precision is not None else "32"
    if p in ("16", "16-mixed", "bf16", "bf16-mixed", "16-true", "bf16-true"):
        return torch.bfloat16
    if p in ("32", "32-true"):
        return torch.float32
    raise ValueError(f"General.precision {precision!r} has no MI355X mode (16 / bf16 / 32)")


def in_features_of(cfg) -> int:
    fe = (cfg.Data or {}).get("feature_extractor") if cfg.Data else None
    if fe in _FEATURE_WIDTH:                                   # code/train.py:392-397
        return _FEATURE_WIDTH[fe]
    return int(cfg.Model.in_features or 1024)


def build_model(cfg, device="cuda"):
    """``models.{Model.name}(n_classes, in_features, out_features)`` on the device, in the compute
    dtype of ``General.precision``; wrapped in the RetCCL encoder for ``backbone: retccl`` on
    images (``Model.backbone == 'features'`` keeps feature bags)."""
    from . import models
    name = cfg.Model.name
    if not hasattr(models, name):
        raise ValueError(f"Model.name {name!r} is not on the MI355X path "
                         "(TransMIL, MDMIL, CTMIL, TransformerMIL, AttMIL)")
    klass = getattr(models, name)
    n_classes = int(cfg.Model.n_classes)
    if name == "MDMIL":
        model = klass(n_classes)
    else:
        model = klass(n_classes, in_features_of(cfg), int(cfg.Model.out_features or 512))
    model = model.to(device)
    dtype = compute_dtype_for(cfg.General.precision if cfg.General else None)
    if hasattr(model, "set_compute_dtype"):
        model.set_compute_dtype(dtype)
    if cfg.Model.backbone == "retccl" and (cfg.Data or {}).get("feature_extractor") is None:
        from .encoder import ImageBagModel, retccl_resnet50
        enc = retccl_resnet50().to(device).set_compute_dtype(dtype)
        model = ImageBagModel(enc, model)
    return model


def build_task(cfg, model, n_gpus: int = 1):
    """``TransMILTask`` with the config's optimizer, loss and gradient accumulation."""
    from .interface import TransMILTask
    opt = cfg.Optimizer or AttrDict()
    acc = 10 if n_gpus > 1 else int((cfg.General or {}).get("grad_acc") or 1)
    task = TransMILTask(model, lr=float(opt.lr or 2e-4), opt=opt.opt or "lookahead_radam",
                        weight_decay=float(opt.weight_decay if opt.weight_decay is not None else 0.01),
                        loss=(cfg.Loss or {}).get("base_loss") or "CrossEntropyLoss", accumulate_grad_batches=acc)
    return task
