"""Golden fixture for the C5 tile encoder, made by running the REFERENCE
``code/models/ResNet.py`` (imported by file path; torch-only) as model_interface.py:238-245
builds it: ``resnet50(num_classes=128, mlp=False, two_branch=False, normlinear=True)``,
``fc = Identity``, eval mode.  Weights and BN statistics come from
``golden_util.deterministic_encoder_params_(seed=2021)`` (no checkpoint ships with the
reference), tiles from ``golden_util.encoder_tiles(4)``.  Stored: the [4, 2048] features in
fp32 and fp64.

    python tests/golden/make_golden_encoder.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from golden_util import deterministic_encoder_params_, encoder_tiles  # noqa: E402

REF = "/root/reference/code/models/ResNet.py"


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    spec = importlib.util.spec_from_file_location("ref_resnet", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    x = torch.from_numpy(encoder_tiles(4))
    payload = {}
    for dt, key in ((torch.float32, "feats"), (torch.float64, "feats.f64")):
        torch.manual_seed(0)
        m = mod.resnet50(num_classes=128, mlp=False, two_branch=False, normlinear=True)
        m.fc = torch.nn.Identity()
        deterministic_encoder_params_(m, 2021)
        m = m.to(dt).eval()
        with torch.no_grad():
            payload[key] = m(x.to(dt)).numpy()
        print(key, payload[key].shape, float(np.abs(payload[key]).mean()), flush=True)
    payload["state_dict_keys"] = np.array(list(m.state_dict().keys()))
    payload["state_dict_numel"] = np.array([v.numel() for v in m.state_dict().values()])
    np.savez_compressed(os.path.join(HERE, "retccl_r50_tiles4.npz"), **payload)
    path = os.path.join(HERE, "index.json")
    index = json.load(open(path))
    index["retccl_r50_tiles4"] = {"model": "ResNet.resnet50(num_classes=128, mlp=False, two_branch=False, "
                                           "normlinear=True), fc=Identity, eval",
                                  "weights": "golden_util.deterministic_encoder_params_(seed=2021)",
                                  "input": "golden_util.encoder_tiles(4)",
                                  "source": "reference code/models/ResNet.py (make_golden_encoder.py)"}
    with open(path, "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
