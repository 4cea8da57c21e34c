"""Golden fixtures for the sibling heads and the 768 _fc1 branch, made by importing the
REFERENCE model files:

  code/models/TransMIL.py        TransMIL(2, 768, 512): the 768 branch (:122-126)
  code/models/CTMIL.py           CTMIL (imports ._transformer, so the models directory is
                                 bound as a package path without running its __init__)
  code/models/TransformerMIL.py  TransformerMIL
  code/models/AttMIL.py          AttMIL (its ``import torchvision.models`` is bound to an empty
                                 module: torchvision is not installed and AttMIL never uses it)

``nystrom_attention`` is the restatement oracle/nystrom_ref.py (as in make_golden.py), the
reference's ``.cuda()`` calls are identity (cuda_noop), weights come from
``deterministic_params_(seed=2021)`` and inputs from numpy PCG64 (``case_input``), eval mode.
Stored: fp32 and fp64 logits per case (data only).

    python tests/golden/make_golden_siblings.py
"""
from __future__ import annotations

import contextlib
import importlib
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from oracle import nystrom_ref  # noqa: E402
from oracle.transmil_ref import deterministic_params_  # noqa: E402
from make_golden import cuda_noop, load_reference_module  # noqa: E402

MODELS_DIR = "/root/reference/code/models"

# name -> (reference module, class, ctor kwargs, input shape)
CASES = {
    "transmil768_n300": ("TransMIL", "TransMIL", dict(n_classes=2, in_features=768, out_features=512), (1, 300, 768)),
    "ctmil_c64_g20_b2": ("CTMIL", "CTMIL", dict(n_classes=2, in_features=64, out_features=512), (1, 2, 64, 20, 20)),
    "ctmil_c128_g36": ("CTMIL", "CTMIL", dict(n_classes=3, in_features=128, out_features=512), (1, 1, 128, 36, 36)),
    "transformermil768_n200_b2": ("TransformerMIL", "TransformerMIL",
                                  dict(n_classes=2, in_features=768, out_features=512), (1, 2, 200, 768)),
    "transformermil2048_n64": ("TransformerMIL", "TransformerMIL",
                               dict(n_classes=3, in_features=2048, out_features=512), (1, 1, 64, 2048)),
    "attmil2048_n500": ("AttMIL", "AttMIL", dict(n_classes=2, in_features=2048, out_features=512), (1, 500, 2048)),
    "attmil1024_n300": ("AttMIL", "AttMIL", dict(n_classes=3, in_features=1024, out_features=512), (1, 300, 1024)),
}


def case_input(name: str) -> np.ndarray:
    """Uniform [0, 1) input of the case's shape from PCG64(seed = 7 + index of the case)."""
    shape = CASES[name][3]
    return np.random.default_rng(7 + sorted(CASES).index(name)).random(shape, dtype=np.float32)


def load_models_package():
    sys.modules["nystrom_attention"] = nystrom_ref
    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        tv.models = types.ModuleType("torchvision.models")
        sys.modules["torchvision"], sys.modules["torchvision.models"] = tv, tv.models
    pkg = types.ModuleType("refmodels")
    pkg.__path__ = [MODELS_DIR]
    sys.modules["refmodels"] = pkg


def reference_class(module, cls):
    if module == "TransMIL":
        return getattr(load_reference_module(), cls)
    load_models_package()
    with contextlib.redirect_stdout(open(os.devnull, "w")):
        return getattr(importlib.import_module(f"refmodels.{module}"), cls)


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    path = os.path.join(HERE, "index.json")
    index = json.load(open(path))
    for name, (module, cls, kw, shape) in CASES.items():
        klass = reference_class(module, cls)
        payload = {}
        for dt, key in ((torch.float32, "logits"), (torch.float64, "logits.f64")):
            torch.manual_seed(0)
            with contextlib.redirect_stdout(open(os.devnull, "w")):
                model = klass(**kw)
            deterministic_params_(model, 2021)
            model = model.to(dt).eval()
            x = torch.from_numpy(case_input(name)).to(dt)
            with cuda_noop(dt == torch.float64), torch.no_grad():
                payload[key] = model(x).detach().numpy()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **payload)
        index[name] = {"model": cls, "ctor": kw, "input_shape": list(shape), "seed": 7 + sorted(CASES).index(name),
                       "weights": "deterministic_params_(seed=2021)", "input": "make_golden_siblings.case_input",
                       "source": f"reference code/models/{module}.py (make_golden_siblings.py)"}
        print(name, payload["logits"].tolist(), flush=True)
    with open(path, "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
