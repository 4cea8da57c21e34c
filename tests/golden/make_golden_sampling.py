"""Golden fixtures for feature-bag sampling, made by calling the REFERENCE
``FeatureBagLoader.__getitem__`` (code/datasets/feature_dataloader.py:335-431) on in-memory bags.

The module is imported by file path.  Its top-level imports of libraries that this image lacks
and that the sampling code never touches (torchsampler, torchvision, zarr, cv2, PIL, h5py) are
bound to empty modules.  The loader object is made without its file-scanning ``__init__`` and
given the cached-bag attributes the cached branch reads (``cache``, ``feature_bags``,
``labels``, ``wsi_names``, ``coords``, ``patients``, ``mode``, ``max_bag_size``, ``mixup``).
Each case seeds torch's default generator with ``torch.manual_seed(seed)`` and then calls
``loader[i]``; the stored data are the sampled bags (and, for the collate case,
``DataInterface.simple_collate``'s stacked output, code/datasets/data_interface.py:238-246,
called unbound).  Bags: PCG64(1000 + n).random((n, F)), float32.

    python tests/golden/make_golden_sampling.py
"""
from __future__ import annotations

import contextlib
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF_LOADER = "/root/reference/code/datasets/feature_dataloader.py"
REF_INTERFACE = "/root/reference/code/datasets/data_interface.py"
F = 32

# name -> (mode, bag sizes, max_bag_size, mixup, seed, item indices)
CASES = {
    "sample_train_n1500": ("train", [1500], 1000, False, 11, [0]),
    "sample_train_pad_n300": ("train", [300], 1000, False, 12, [0]),
    "sample_finetune_n50": ("fine_tune", [50], 64, False, 13, [0]),
    "sample_mixup_pad_n300": ("train", [300], 1000, True, 14, [0]),
    "sample_mixup_small_n40": ("train", [40], 1000, True, 15, [0]),
    "sample_mixup_full_n1500": ("train", [1500], 1000, True, 16, [0]),
    "sample_test_n1234": ("test", [1234], 1000, False, 17, [0]),
    "sample_val_n95": ("val", [95], 1000, False, 18, [0]),
    "sample_collate_b3": ("train", [700, 1300, 20], 512, False, 19, [2, 0, 1]),
}


def bag(n):
    return np.random.default_rng(1000 + n).random((n, F), dtype=np.float32)


def _stub(name, *children):
    m = types.ModuleType(name)
    sys.modules[name] = m
    for c in children:
        sub = types.ModuleType(f"{name}.{c}")
        setattr(m, c, sub)
        sys.modules[f"{name}.{c}"] = sub
    return m


def load_reference():
    _stub("torchsampler").ImbalancedDatasetSampler = object
    _stub("torchvision", "datasets", "transforms")
    _stub("zarr")
    _stub("cv2")
    _stub("PIL", "Image")
    _stub("h5py")
    mods = {}
    for key, path in (("loader", REF_LOADER), ("interface", REF_INTERFACE)):
        spec = importlib.util.spec_from_file_location(f"ref_{key}", path)
        mod = importlib.util.module_from_spec(spec)
        try:
            with contextlib.redirect_stdout(open(os.devnull, "w")):
                spec.loader.exec_module(mod)
        except Exception as exc:  # noqa: BLE001 - the interface module needs more than the sampling
            mod = exc
        mods[key] = mod
    return mods


def make_loader(ref, mode, sizes, max_bag_size, mixup):
    cls = ref.FeatureBagLoader
    obj = cls.__new__(cls)
    obj.cache = True
    obj.mode, obj.max_bag_size, obj.mixup = mode, max_bag_size, mixup
    obj.feature_bags = [torch.from_numpy(bag(n)) for n in sizes]
    obj.labels = [i % 2 for i in range(len(sizes))]
    obj.wsi_names = [f"slide{i}" for i in range(len(sizes))]
    obj.patients = [f"patient{i}" for i in range(len(sizes))]
    obj.coords = [torch.arange(2 * n).reshape(n, 2) for n in sizes]
    return obj


def collate(items):
    """data_interface.py:238-246 restated only where the module cannot be imported."""
    bags = torch.stack([i[0] for i in items])
    labels = torch.Tensor(np.stack([i[1] for i in items], axis=0)).long()
    return bags, labels, ([i[2][0] for i in items], [i[2][1] for i in items])


def main():
    mods = load_reference()
    ref = mods["loader"]
    if isinstance(ref, Exception):
        raise ref
    iface = mods["interface"]
    path = os.path.join(HERE, "index.json")
    index = json.load(open(path))
    for name, (mode, sizes, mbs, mixup, seed, items) in CASES.items():
        loader = make_loader(ref, mode, sizes, mbs, mixup)
        torch.manual_seed(seed)
        outs = [loader[i] for i in items]
        payload = {}
        if name.startswith("sample_collate"):
            if not isinstance(iface, Exception):
                bags, labels, (names, patients) = iface.DataInterface.simple_collate(None, outs)
                source = "FeatureBagLoader.__getitem__ + DataInterface.simple_collate (reference)"
            else:
                bags, labels, (names, patients) = collate(outs)
                source = f"FeatureBagLoader.__getitem__ (reference) + simple_collate restated ({type(iface).__name__})"
            payload["bags"], payload["labels"] = bags.numpy(), labels.numpy()
        else:
            payload["bag"] = outs[0][0].numpy()
            source = "FeatureBagLoader.__getitem__ (reference)"
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **payload)
        index[name] = {"sampling": {"mode": mode, "sizes": sizes, "max_bag_size": mbs, "mixup": mixup, "seed": seed,
                                    "items": items, "F": F},
                       "input": "PCG64(1000 + n).random((n, 32)) float32 per bag", "source": source}
        print(name, {k: v.shape for k, v in payload.items()}, flush=True)
    with open(path, "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
