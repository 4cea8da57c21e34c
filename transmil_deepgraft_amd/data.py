"""Feature-bag ingest and train-time sampling with the bags resident in HBM.

Mirrors ``FeatureBagLoader`` (code/datasets/feature_dataloader.py:26-431) for the feature-bag
path of the hot loop and ``DataInterface.simple_collate`` (code/datasets/data_interface.py:238-246):

* ``FeatureBagStore``   every bag of a split in ONE device slab ``[total_rows, F]`` (fp32, or
                        bf16 to halve it) plus row offsets: 288 GB of HBM holds whole cohorts
                        (a 40k-tile RetCCL bag is 328 MB fp32), so ingest happens once and the
                        per-step work is a gather, not an HDF5 read + host->device copy.  Loads
                        ``.npy`` / ``.pt`` (``weights_only=True``) / ``.safetensors`` files; the
                        reference's HDF5 reader (h5py, :228-276) is not available in this image.
* ``FeatureBagLoader``  ``__getitem__`` with the reference's sampling, drawing its indices with
                        the SAME RNG calls in the same order (torch.randperm / torch.rand /
                        torch.randint on torch's default CPU generator for train / fine_tune,
                        :346-362 and mixup :305-330; numpy ``seed(0)`` + ``choice`` with
                        replacement for val / test, :421-431), then ONE ``tm_gather_rows``
                        launch builds the sampled, zero-padded, reshuffled bag on the device.
* ``collate``           a whole batch of train bags in one launch -> ``simple_collate``'s
                        ``(bags [B, max_bag_size, F], labels, (names, patients))``.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import _lib
from ._lib import BF16, F32
from .engine import _p, _stream


def _load_array(path):
    ext = os.path.splitext(path)[1]
    if ext == ".npy":
        return torch.from_numpy(np.load(path, allow_pickle=False))
    if ext == ".pt":
        obj = torch.load(path, map_location="cpu", weights_only=True)
        return obj if torch.is_tensor(obj) else obj["features"]
    if ext == ".safetensors":
        from safetensors.torch import load_file
        return load_file(path)["features"]
    raise ValueError(f"unsupported feature file {path} (.npy / .pt / .safetensors)")


class FeatureBagStore:
    """All bags of one split as rows of one HBM slab."""

    def __init__(self, bags, device="cuda", dtype=torch.float32):
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("feature store dtype must be float32 or bfloat16")
        bags = [torch.as_tensor(b) for b in bags]
        if not bags or any(b.dim() != 2 for b in bags):
            raise ValueError("bags must be a non-empty list of [n_i, F] arrays")
        F = bags[0].shape[1]
        if any(b.shape[1] != F for b in bags):
            raise ValueError("every bag must have the same feature width")
        self.F, self.dtype = F, dtype
        self.sizes = [int(b.shape[0]) for b in bags]
        self.offsets = np.concatenate([[0], np.cumsum(self.sizes)]).astype(np.int64)
        self.slab = torch.empty(int(self.offsets[-1]), F, dtype=dtype, device=device)
        for b, o, n in zip(bags, self.offsets, self.sizes):
            self.slab[o:o + n].copy_(b.to(dtype), non_blocking=False)

    @classmethod
    def from_files(cls, paths, device="cuda", dtype=torch.float32):
        return cls([_load_array(p) for p in paths], device=device, dtype=dtype)

    def __len__(self):
        return len(self.sizes)

    def bag(self, i):
        o = int(self.offsets[i])
        return self.slab[o:o + self.sizes[i]]


class _Rows:
    """Host description of one sampled bag: row ids (global, -1 = zero row) and blend rows."""

    def __init__(self, i0, i1=None, wa=None, wb=None):
        self.i0 = i0
        self.i1, self.wa, self.wb = i1, wa, wb


class FeatureBagLoader:
    """``FeatureBagLoader.__getitem__`` (feature_dataloader.py:335-431) over a FeatureBagStore.

    ``labels``, ``wsi_names``, ``patients``, ``coords`` are per bag, as the reference caches
    them (:338-344).  Train / fine_tune return ``(bag [max_bag_size, F], label, (wsi_name,
    patient))``; other modes ``(bag [ceil(0.1 n), F], label, (wsi_name, coords, patient))``."""

    def __init__(self, store: FeatureBagStore, labels, mode, n_classes, max_bag_size=1000, mixup=False,
                 wsi_names=None, patients=None, coords=None):
        self.store, self.labels, self.mode, self.n_classes = store, list(labels), mode, n_classes
        self.max_bag_size, self.mixup = max_bag_size, mixup
        n = len(store)
        self.wsi_names = list(wsi_names) if wsi_names is not None else [f"bag{i}" for i in range(n)]
        self.patients = list(patients) if patients is not None else list(self.wsi_names)
        self.coords = list(coords) if coords is not None else [None] * n

    def __len__(self):
        return len(self.store)

    # ---------------------------------------------------------------- host-side index draws
    def _mixup_rows(self, idx):
        """get_mixup_bag (:305-330) on the drawn rows ``idx`` (global row ids)."""
        m = idx.numel()
        a = torch.rand([m])
        rand_x = torch.randint(0, m, [m])
        rand_y = torch.randint(0, m, [m])
        if m < self.max_bag_size:
            sel = torch.randperm(m)[:self.max_bag_size - m]
            i0 = torch.cat([idx, idx[rand_x[sel]]])
            i1 = torch.cat([torch.full([m], -1, dtype=torch.int64), idx[rand_y[sel]]])
            wa = torch.cat([torch.ones(m), a[sel]])
            wb = torch.cat([torch.zeros(m), (1.0 - a)[sel]])
            return _Rows(i0, i1, wa, wb)
        keep = torch.rand(m)
        if not bool((keep != 0).all()):
            # the reference builds a bool row there and torch.stack fails (:327-328)
            raise RuntimeError("mixup: a zero draw makes the reference's stack fail")
        return _Rows(idx)

    def _train_rows(self, index):
        base = int(self.store.offsets[index])
        n = self.store.sizes[index]
        idx = torch.randperm(n)[:self.max_bag_size] + base          # :349-351
        rows = self._mixup_rows(idx) if self.mixup else _Rows(idx)  # :353-354
        k = rows.i0.numel()
        if k < self.max_bag_size:                                   # :356-357 zero padding
            pad = self.max_bag_size - k
            rows.i0 = torch.cat([rows.i0, torch.full([pad], -1, dtype=torch.int64)])
            if rows.i1 is not None:
                rows.i1 = torch.cat([rows.i1, torch.full([pad], -1, dtype=torch.int64)])
                rows.wa = torch.cat([rows.wa, torch.zeros(pad)])
                rows.wb = torch.cat([rows.wb, torch.zeros(pad)])
        perm = torch.randperm(rows.i0.numel())                      # :360-361 shuffle again
        rows.i0 = rows.i0[perm]
        if rows.i1 is not None:
            rows.i1, rows.wa, rows.wb = rows.i1[perm], rows.wa[perm], rows.wb[perm]
        return rows

    def _eval_rows(self, index):
        n = self.store.sizes[index]
        draw = np.random.RandomState(0).choice(n, math.ceil(n * 0.1))    # :421-427 (seed(0) + choice)
        return _Rows(torch.from_numpy(draw.astype(np.int64)) + int(self.store.offsets[index]))

    # ---------------------------------------------------------------- device gather
    def _gather(self, rows_list):
        i0 = torch.cat([r.i0 for r in rows_list])
        blend = any(r.i1 is not None for r in rows_list)
        dev = self.store.slab.device
        out = torch.empty(i0.numel(), self.store.F, dtype=self.store.dtype, device=dev)
        if i0.numel() == 0:
            return out
        i0d = i0.to(dev)
        i1d = wad = wbd = None
        if blend:
            i1 = torch.cat([r.i1 if r.i1 is not None else torch.full_like(r.i0, -1) for r in rows_list])
            wa = torch.cat([r.wa if r.wa is not None else torch.ones(r.i0.numel()) for r in rows_list])
            wb = torch.cat([r.wb if r.wb is not None else torch.zeros(r.i0.numel()) for r in rows_list])
            i1d, wad, wbd = i1.to(dev), wa.float().to(dev), wb.float().to(dev)
        for s in range(0, i0.numel(), 65535):
            e = min(i0.numel(), s + 65535)
            _lib.call("tm_gather_rows", BF16 if self.store.dtype == torch.bfloat16 else F32, _p(self.store.slab),
                      self.store.F, _p(i0d[s:e]), _p(i1d[s:e] if blend else None),
                      _p(wad[s:e] if blend else None), _p(wbd[s:e] if blend else None), e - s, _p(out[s:e]),
                      _stream())
        return out

    def __getitem__(self, index):
        label = self.labels[index]
        name, patient, coords = self.wsi_names[index], self.patients[index], self.coords[index]
        if self.mode in ("train", "fine_tune"):
            return self._gather([self._train_rows(index)]), label, (name, patient)
        return self._gather([self._eval_rows(index)]), label, (name, coords, patient)

    def collate(self, indices):
        """The items ``indices`` (train / fine_tune mode) drawn in order, as
        ``simple_collate`` returns them (data_interface.py:238-246), gathered in one launch."""
        if self.mode not in ("train", "fine_tune"):
            raise ValueError("collate stacks fixed-size bags: train / fine_tune mode only")
        rows = [self._train_rows(i) for i in indices]
        bags = self._gather(rows).view(len(indices), self.max_bag_size, self.store.F)
        labels = torch.tensor(np.stack([self.labels[i] for i in indices], axis=0)).long()
        return bags, labels, ([self.wsi_names[i] for i in indices], [self.patients[i] for i in indices])


def simple_collate(data):
    """``DataInterface.simple_collate`` (data_interface.py:238-246) for items already on the device."""
    bags = torch.stack([d[0] for d in data])
    labels = torch.Tensor(np.stack([d[1] for d in data], axis=0)).long()
    return bags, labels, ([d[2][0] for d in data], [d[2][1] for d in data])
