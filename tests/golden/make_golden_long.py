"""Golden logits for the long-sequence config C3 (SURVEY.md section 8 d): TransMIL_feat
3-class, N = 32768 x 512 (n' = 33280, 256 landmarks, l = 130).

The reference's as-written forward cannot run here at this size: every TransLayer asks
NystromAttention for ``return_attn=True`` (code/models/TransMIL.py:47), materialising
[1, 8, 33280, 33280] = 35 GB (fp32; 71 GB fp64) per layer on a 64 GB host.  So this
fixture comes from the CPU oracle (``oracle/transmil_ref.py``) with that unused product
switched off (``TransLayer.compute_attn = False``) -- the logits are the same function,
and the oracle is pinned against the reference itself at N = 1024 / 8192 by
``make_golden.py``'s d512 fixtures (tests/test_oracle.py).

    python tests/golden/make_golden_long.py        (about a minute on 8 cores)

Weights: ``deterministic_params_(seed=2021)``; input: ``bag_input(n, 512, 2021+1000+n)``.
Only the expected logits are stored (fp32 and the fp64 noise-floor run).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle.transmil_ref import TransMIL, TransLayer, deterministic_params_  # noqa: E402
sys.path.insert(0, HERE)
from make_golden import bag_input  # noqa: E402


def main(name="d512c3_n32768", ncls=3, n=32768, seed=2021):
    TransLayer.compute_attn = False
    torch.set_num_threads(os.cpu_count() or 8)
    payload = {}
    for dt, key in ((torch.float32, "logits"), (torch.float64, "logits.f64")):
        torch.manual_seed(0)
        model = TransMIL(ncls, 512, 512)
        deterministic_params_(model, seed)
        model = model.to(dt).eval()
        x = torch.from_numpy(bag_input(n, 512, seed + 1000 + n)).to(dt)
        orig = torch.Tensor.float
        if dt == torch.float64:
            torch.Tensor.float = lambda self, *a, **k: self   # keep the fp64 run in fp64
        try:
            with torch.no_grad():
                payload[key] = model(x).numpy()
        finally:
            torch.Tensor.float = orig
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **payload)
    path = os.path.join(HERE, "index.json")
    index = json.load(open(path))
    index[name] = {"n_classes": ncls, "feat": 512, "n": n, "batch": 1,
                   "weights": "deterministic_params_(seed=2021)",
                   "input": "bag_input(n, 512, seed=2021+1000+n)",
                   "source": "oracle (TransLayer.compute_attn=False); see make_golden_long.py"}
    with open(path, "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)
    print(name, payload["logits"], payload["logits.f64"])


if __name__ == "__main__":
    main()
