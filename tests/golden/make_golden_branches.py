"""Golden logits for the other model entry points on the same kernels, from the REFERENCE.

Run once where ``/root/reference`` exists:  python tests/golden/make_golden_branches.py

  * ``fc2048_n300``: ``code/models/TransMIL.py`` TransMIL(2, in_features=2048, out_features=512),
    the RCC ``_fc1`` branch Linear(2048,1024)+GELU+LayerNorm(1024)+Linear(1024,512)+GELU
    (:100-111);
  * ``mdmil_n300``: ``code/models/MDMIL.py`` MDMIL(2) (Linear(1024,512)+GELU, head ``_fc2``,
    returns (logits, attn2)).

Both import the reference file by path with ``sys.modules['nystrom_attention']`` = the
restated package (``oracle/nystrom_ref.py``) and ``.cuda()`` neutralised, exactly as
``make_golden.py`` does.  Weights come from ``oracle.transmil_ref.deterministic_params_``
(seed 2021) and the bag from ``bag_input(300, F, 2021 + 1000 + 300)``, so the fixture holds
only the expected outputs: logits (fp32 and fp64), the CE loss and the gradients of the
small parameters (class token, the final norm, the head), eval mode.
"""
from __future__ import annotations

import contextlib
import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import nystrom_ref  # noqa: E402
from oracle.transmil_ref import deterministic_params_  # noqa: E402
from make_golden import bag_input, cuda_noop  # noqa: E402

SMALL_GRADS = ("cls_token", "norm.weight", "norm.bias")


def load_ref(fname, modname):
    sys.modules["nystrom_attention"] = nystrom_ref
    spec = importlib.util.spec_from_file_location(modname, f"/root/reference/code/models/{fname}")
    mod = importlib.util.module_from_spec(spec)
    with contextlib.redirect_stdout(open(os.devnull, "w")):
        spec.loader.exec_module(mod)
    return mod


def run(make, feat, head, n=300, label=1):
    payload = {}
    for dt, tag in ((torch.float32, ""), (torch.float64, ".f64")):
        torch.manual_seed(0)
        with contextlib.redirect_stdout(open(os.devnull, "w")):
            model = make()
        deterministic_params_(model, 2021)
        model = model.to(dt).eval()
        x = torch.from_numpy(bag_input(n, feat, 2021 + 1000 + n)).to(dt)
        with cuda_noop(dt == torch.float64):
            out = model(x)
            logits = out[0] if isinstance(out, tuple) else out
            loss = torch.nn.CrossEntropyLoss()(logits, torch.nn.functional.one_hot(
                torch.tensor([label]), 2).to(dt))
            loss.backward()
        payload["logits" + tag] = logits.detach().numpy()
        payload["loss" + tag] = loss.detach().numpy().reshape(1)
        for pname, p in model.named_parameters():
            if pname in SMALL_GRADS or pname.startswith(head + "."):
                payload["grad." + pname + tag] = p.grad.detach().numpy().copy()
    return payload


def main():
    tm = load_ref("TransMIL.py", "ref_transmil")
    md = load_ref("MDMIL.py", "ref_mdmil")
    index = json.load(open(os.path.join(HERE, "index.json")))
    cases = {
        "fc2048_n300": (lambda: tm.TransMIL(n_classes=2, in_features=2048, out_features=512), 2048, "_fc"),
        "mdmil_n300": (lambda: md.MDMIL(n_classes=2), 1024, "_fc2"),
    }
    for name, (make, feat, head) in cases.items():
        payload = run(make, feat, head)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **payload)
        index[name] = {"n_classes": 2, "feat": feat, "n": 300, "batch": 1, "label": 1, "head": head,
                       "model": "MDMIL" if name.startswith("mdmil") else "TransMIL(in_features=2048)",
                       "weights": "deterministic_params_(seed=2021)",
                       "input": "bag_input(n, feat, seed=2021+1000+n)",
                       "source": "reference import; see make_golden_branches.py"}
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)
    print("wrote", sorted(cases))


if __name__ == "__main__":
    main()
