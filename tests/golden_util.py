"""Helpers to load the golden fixtures (data only; see tests/golden/make_golden.py)."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def index():
    with open(os.path.join(GOLDEN, "index.json")) as f:
        return json.load(f)


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def bag_input(n, feat, seed, batch=1):
    """Same generator as tests/golden/make_golden.py::bag_input."""
    return np.random.default_rng(seed).random((batch, n, feat), dtype=np.float32)


def oracle_model(fx, dtype=torch.float64):
    """Oracle TransMIL with the fixture's weights (small cases)."""
    from oracle.transmil_ref import TransMIL
    meta = {k[2:]: v for k, v in fx.items() if k.startswith("w.")}
    feat = meta["_fc1.0.weight"].shape[1]
    ncls = meta["_fc.weight"].shape[0]
    torch.manual_seed(0)
    m = TransMIL(n_classes=ncls, in_features=feat, out_features=feat)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in meta.items()})
    return m.to(dtype).eval()


def sibling_input(name):
    """Input of a make_golden_siblings.py case: PCG64(seed).random(input_shape) (float32)."""
    meta = index()[name]
    return np.random.default_rng(meta["seed"]).random(tuple(meta["input_shape"]), dtype=np.float32)
