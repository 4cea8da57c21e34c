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


def deterministic_encoder_params_(model, seed=2021):
    """Fill a (RetCCL) ResNet-50's parameters and BN running statistics by name: each tensor
    from PCG64(seed ^ crc32(name)), so module registration order does not matter.  Conv
    weights ~ U(+-sqrt(3 / fan_in)); BN weight ~ U(0.5, 1) (bn3 of each block ~ U(0, 0.2), which
    keeps the 16 residual additions bounded); BN bias / running_mean ~ U(-0.1, 0.1);
    running_var ~ U(0.5, 1.5)."""
    import zlib
    import torch
    with torch.no_grad():
        for name, t in list(model.named_parameters()) + list(model.named_buffers()):
            if name.endswith("num_batches_tracked"):
                continue
            rng = np.random.default_rng(seed ^ zlib.crc32(name.encode()))
            shape = tuple(t.shape)
            if t.dim() == 4:
                a = float(np.sqrt(3.0 / (t.numel() // shape[0])))
                val = rng.uniform(-a, a, shape)
            elif name.endswith("running_var"):
                val = rng.uniform(0.5, 1.5, shape)
            elif name.endswith(("running_mean", ".bias")):
                val = rng.uniform(-0.1, 0.1, shape)
            elif name.endswith(".weight") and (".bn3." in name or name.endswith("bn3.weight")):
                val = rng.uniform(0.0, 0.2, shape)
            elif name.endswith(".weight"):
                val = rng.uniform(0.5, 1.0, shape)
            else:
                raise ValueError(f"unexpected encoder tensor {name}")
            t.copy_(torch.from_numpy(np.asarray(val)).to(t.dtype))
    return model


def encoder_tiles(n, seed=77):
    """Synthetic 224x224 RGB tiles, ImageNet-normalised range: PCG64(seed).standard_normal."""
    return np.random.default_rng(seed).standard_normal((n, 3, 224, 224)).astype(np.float32)
