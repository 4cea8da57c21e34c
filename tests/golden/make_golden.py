"""Generate the golden fixtures by running the REFERENCE ``code/models/TransMIL.py``.

Run once in the survey container (where ``/root/reference`` exists):

    python tests/golden/make_golden.py

What it does:
  * imports ``/root/reference/code/models/TransMIL.py`` by file path, with
    ``sys.modules['nystrom_attention']`` set to the restated package class
    (``oracle/nystrom_ref.py``; the real package is not vendored and not
    installed -- SURVEY.md section 8 c);
  * makes ``Tensor.cuda()`` a no-op for the duration of each forward (the
    reference hard-codes it at ``code/models/TransMIL.py:184``; no GPU here);
  * fills weights with ``oracle.transmil_ref.deterministic_params_`` and runs
    fp32 and fp64 forwards (eval mode, dropout off), plus an fp32/fp64
    backward of ``CrossEntropyLoss(logits, one_hot(label).float())``
    (``code/models/model_interface.py:346-347``) for the small cases.

Fixtures are data only (inputs, weights for the small model, expected outputs);
no reference source is copied.  The d=512 cases store no weights or inputs:
both come from the documented PCG64 generators (``bag_input`` below and
``deterministic_params_``), so the fixture holds only the expected logits.
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
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import nystrom_ref  # noqa: E402
from oracle.transmil_ref import deterministic_params_  # noqa: E402

REF_FILE = "/root/reference/code/models/TransMIL.py"


def bag_input(n: int, feat: int, seed: int, batch: int = 1) -> np.ndarray:
    """Synthetic bag like ``torch.rand([bag, F])`` (code/sustainability_train.py:43)."""
    return np.random.default_rng(seed).random((batch, n, feat), dtype=np.float32)


def load_reference_module():
    sys.modules["nystrom_attention"] = nystrom_ref
    spec = importlib.util.spec_from_file_location("ref_transmil", REF_FILE)
    mod = importlib.util.module_from_spec(spec)
    with contextlib.redirect_stdout(open(os.devnull, "w")):
        spec.loader.exec_module(mod)
    return mod


@contextlib.contextmanager
def cuda_noop(keep_f64=False):
    """``.cuda()`` -> identity; for the fp64 noise-floor run also ``.float()``
    (``code/models/TransMIL.py:174`` casts the bag to fp32)."""
    orig, orig_f = torch.Tensor.cuda, torch.Tensor.float
    torch.Tensor.cuda = lambda self, *a, **k: self
    if keep_f64:
        torch.Tensor.float = lambda self, *a, **k: self
    try:
        yield
    finally:
        torch.Tensor.cuda, torch.Tensor.float = orig, orig_f


def run_case(ref, name, n_classes, feat, n, batch=1, seed=2021, dtype=torch.float32,
             peaky=None, want_inter=True, want_attn=False, want_grad=False, label=None):
    torch.manual_seed(0)
    with contextlib.redirect_stdout(open(os.devnull, "w")):
        model = ref.TransMIL(n_classes=n_classes, in_features=feat, out_features=feat)
    deterministic_params_(model, seed)
    if peaky is not None:
        with torch.no_grad():
            for layer in (model.layer1, model.layer2):
                w = layer.attn.to_qkv.weight
                w[: w.shape[0] // 3] *= peaky
    model = model.to(dtype).eval()
    x = torch.from_numpy(bag_input(n, feat, seed + 1000 + n, batch)).to(dtype)
    inter = {}
    hooks = []
    if want_inter:
        def grab(key, idx=None):
            def f(_m, _i, o):
                inter[key] = (o[idx] if idx is not None else o).detach().clone()
            return f
        hooks += [model._fc1.register_forward_hook(grab("fc1")),
                  model.layer1.register_forward_hook(grab("layer1", 0)),
                  model.pos_layer.register_forward_hook(grab("ppeg")),
                  model.layer2.register_forward_hook(grab("layer2", 0))]
    out = {}
    with cuda_noop(dtype == torch.float64):
        if want_grad:
            logits, (attn, padding) = model(x, return_attn=True)
            y = torch.tensor([label if label is not None else 1] * batch)
            loss = torch.nn.CrossEntropyLoss()(
                logits, torch.nn.functional.one_hot(y, n_classes).to(dtype))
            loss.backward()
            for pname, p in model.named_parameters():
                out["grad." + pname] = p.grad.detach().numpy().copy()
            out["label"] = y.numpy()
            out["loss"] = loss.detach().numpy().reshape(1)
        else:
            with torch.no_grad():
                logits, (attn, padding) = model(x, return_attn=True)
    for h in hooks:
        h.remove()
    out["logits"] = logits.detach().numpy()
    out["padding"] = np.array(padding)
    for k, v in inter.items():
        out["inter." + k] = v.numpy()
    if want_attn:
        out["attn"] = attn.detach().numpy()
    return model, x, out


def main():
    ref = load_reference_module()
    index = {}
    small = [("small_n1", 2, 1), ("small_n2", 2, 2), ("small_n3", 2, 3),
             ("small_n100", 2, 100), ("small_n1000", 2, 1000), ("small3_n257", 3, 257)]
    for name, ncls, n in small:
        for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
            model, x, out = run_case(ref, name, ncls, 64, n, dtype=dt,
                                     want_attn=(n <= 100), want_grad=True)
            if tag == "f32":
                payload = {"x": x.numpy()}
                for pname, p in model.state_dict().items():
                    payload["w." + pname] = p.numpy()
                payload.update(out)
            else:
                payload.update({k + ".f64": v for k, v in out.items()
                                if k.startswith(("logits", "grad.", "loss"))})
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **payload)
        index[name] = {"n_classes": ncls, "feat": 64, "n": n, "batch": 1}
    # batch coupling of the pinv global max (B=4 bags of 100)
    for name, kw in (("batch4_n100", dict(n=100, batch=4)),
                     ("peaky16_n300", dict(n=300, peaky=16.0))):
        payload = {}
        for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
            model, x, out = run_case(ref, name, 2, 64, want_grad=True, dtype=dt, **kw)
            if tag == "f32":
                payload["x"] = x.numpy()
                for pname, p in model.state_dict().items():
                    payload["w." + pname] = p.numpy()
                payload.update(out)
            else:
                payload.update({k + ".f64": v for k, v in out.items()
                                if k.startswith(("logits", "grad.", "loss"))})
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **payload)
        index[name] = {"n_classes": 2, "feat": 64, "n": kw["n"], "batch": kw.get("batch", 1)}
    # d = 512: logits only; weights and inputs regenerated from seeds
    for name, ncls, n in (("d512_n1024", 2, 1024), ("d512_n8192", 2, 8192)):
        payload = {}
        for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
            _, _, out = run_case(ref, name, ncls, 512, n, dtype=dt, want_inter=False)
            payload["logits" if tag == "f32" else "logits.f64"] = out["logits"]
            payload["padding"] = out["padding"]
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **payload)
        index[name] = {"n_classes": ncls, "feat": 512, "n": n, "batch": 1,
                       "weights": "deterministic_params_(seed=2021)",
                       "input": "bag_input(n, 512, seed=2021+1000+n)"}
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)
    print("wrote", sorted(index))


if __name__ == "__main__":
    main()
