"""Feature-bag sampling (transmil_deepgraft_amd/data.py) against the reference's own
FeatureBagLoader.__getitem__ output (fixtures from tests/golden/make_golden_sampling.py).

CPU: the host-side index draws (same RNG calls, same order) applied by a numpy gather give the
fixture bit for bit.  GPU: the tm_gather_rows launch on an HBM-resident store gives it bit for
bit (plain rows are copies; mixup rows are two rounded fp32 products and one add)."""
import numpy as np
import pytest
import torch

from golden_util import index, load

CASES = sorted(k for k, v in index().items() if "sampling" in v)


def _bag(n, F):
    return np.random.default_rng(1000 + n).random((n, F), dtype=np.float32)


def _loader(name, device):
    from transmil_deepgraft_amd.data import FeatureBagLoader, FeatureBagStore
    s = index()[name]["sampling"]
    store = FeatureBagStore([_bag(n, s["F"]) for n in s["sizes"]], device=device)
    loader = FeatureBagLoader(store, [i % 2 for i in range(len(s["sizes"]))], s["mode"], 2,
                              max_bag_size=s["max_bag_size"], mixup=s["mixup"],
                              wsi_names=[f"slide{i}" for i in range(len(s["sizes"]))],
                              patients=[f"patient{i}" for i in range(len(s["sizes"]))])
    return loader, s


def _emulate(slab, rows):
    """numpy gather with the kernel's arithmetic (fp32 products rounded, then added)."""
    i0 = rows.i0.numpy()
    out = np.zeros((i0.size, slab.shape[1]), np.float32)
    plain = i0 >= 0
    out[plain] = slab[i0[plain]]
    if rows.i1 is not None:
        i1 = rows.i1.numpy()
        bl = (i0 >= 0) & (i1 >= 0)
        wa, wb = rows.wa.numpy().astype(np.float32), rows.wb.numpy().astype(np.float32)
        out[bl] = slab[i0[bl]] * wa[bl, None] + slab[i1[bl]] * wb[bl, None]
    return out


@pytest.mark.parametrize("name", CASES)
def test_sampling_index_draws_match_reference(name):
    loader, s = _loader(name, "cpu")
    fx = load(name)
    slab = loader.store.slab.numpy()
    torch.manual_seed(s["seed"])
    outs = []
    for i in s["items"]:
        rows = loader._train_rows(i) if s["mode"] in ("train", "fine_tune") else loader._eval_rows(i)
        outs.append(_emulate(slab, rows))
    if "bags" in fx:
        assert np.array_equal(np.stack(outs), fx["bags"])
        assert np.array_equal(np.array([i % 2 for i in s["items"]]), fx["labels"])
    else:
        assert np.array_equal(outs[0], fx["bag"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_sampling_on_device_matches_reference(name):
    loader, s = _loader(name, "cuda")
    fx = load(name)
    torch.manual_seed(s["seed"])
    if "bags" in fx:
        bags, labels, (names, patients) = loader.collate(s["items"])
        assert np.array_equal(bags.cpu().numpy(), fx["bags"])
        assert np.array_equal(labels.numpy(), fx["labels"])
        assert names == [f"slide{i}" for i in s["items"]]
    else:
        out = loader[s["items"][0]]
        assert out[0].is_cuda
        assert np.array_equal(out[0].cpu().numpy(), fx["bag"])
        assert len(out[2]) == (2 if s["mode"] in ("train", "fine_tune") else 3)


@pytest.mark.gpu
def test_sampling_bf16_store_and_large_gather():
    """A bf16 store (half the HBM) gathers exact bf16 rows; a 3 x 8192 x 2048 batch (the C5
    feature width) in one call equals torch indexing."""
    from transmil_deepgraft_amd.data import FeatureBagLoader, FeatureBagStore
    g = torch.Generator().manual_seed(5)
    bags = [torch.rand(n, 2048, generator=g) for n in (9000, 5000, 12000)]
    store = FeatureBagStore(bags, device="cuda", dtype=torch.bfloat16)
    loader = FeatureBagLoader(store, [0, 1, 0], "train", 2, max_bag_size=8192)
    torch.manual_seed(3)
    got, _, _ = loader.collate([0, 1, 2])
    torch.manual_seed(3)
    want = []
    for i, b in enumerate(bags):
        rows = loader._train_rows(i)
        full = torch.cat([b.to(torch.bfloat16), torch.zeros(1, 2048, dtype=torch.bfloat16)])
        want.append(full[torch.where(rows.i0 >= 0, rows.i0 - int(store.offsets[i]), b.shape[0])])
    assert torch.equal(got.cpu(), torch.stack(want))
