"""C5 tile encoder (transmil_deepgraft_amd/encoder.py) against the reference's own ResNet.py
(fixture tests/golden/make_golden_encoder.py: resnet50 as model_interface.py:238-245 builds it,
fc = Identity, eval, deterministic weights and BN statistics)."""
import numpy as np
import pytest
import torch

from golden_util import deterministic_encoder_params_, encoder_tiles, load


def _encoder(dtype=torch.float32):
    from transmil_deepgraft_amd.encoder import retccl_resnet50
    m = retccl_resnet50()
    deterministic_encoder_params_(m, 2021)
    return m.set_compute_dtype(dtype).eval()


def test_encoder_state_dict_matches_reference_layout():
    fx = load("retccl_r50_tiles4")
    sd = _encoder().state_dict()
    assert list(sd.keys()) == [str(k) for k in fx["state_dict_keys"]]
    assert [v.numel() for v in sd.values()] == list(fx["state_dict_numel"])


def test_encoder_folding_math_on_host():
    """The eval-mode BN folding (host-side weight preparation) reproduces the reference
    features; the unfolded module path too (both run here on CPU tensors as a logic check --
    the product forward refuses CPU tensors)."""
    fx = load("retccl_r50_tiles4")
    m = _encoder()
    x = torch.from_numpy(encoder_tiles(2))
    with torch.no_grad():
        m._fold_all()
        folded = m._forward_folded(x).numpy()
        plain = m._forward_modules(x).numpy()
    np.testing.assert_allclose(folded, fx["feats.f64"][:2], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(plain, fx["feats"][:2], rtol=1e-5, atol=1e-6)
    with pytest.raises(RuntimeError, match="GPU"):
        m(x)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,rtol", [(torch.float32, 2e-3), (torch.bfloat16, 6e-2)])
def test_encoder_gpu_matches_reference(dtype, rtol):
    fx = load("retccl_r50_tiles4")
    torch.backends.cudnn.allow_tf32 = False
    m = _encoder(dtype).cuda()
    with torch.no_grad():
        got = m(torch.from_numpy(encoder_tiles(4)).cuda()).cpu().numpy()
    ref = fx["feats.f64"]
    err = np.linalg.norm(got - ref, axis=1) / np.linalg.norm(ref, axis=1)
    assert err.max() < rtol, err


@pytest.mark.gpu
def test_image_path_end_to_end():
    """ModelInterface.forward's image branch: [B, bag, 3, 224, 224] -> encoder -> [B, bag, 2048]
    -> TransMIL(2, 2048) fused engine, features never leave the device; equals running the
    encoder and the model separately; fp32 backward reaches the TransMIL parameters only."""
    from transmil_deepgraft_amd.encoder import ImageBagModel
    from transmil_deepgraft_amd.models import TransMIL
    torch.manual_seed(0)
    mil = TransMIL(2, 2048).cuda().eval().set_compute_dtype(torch.float32)   # eval: no dropout
    enc = _encoder(torch.float32).cuda()
    model = ImageBagModel(enc, mil)
    x = torch.from_numpy(encoder_tiles(6, seed=5)).cuda().view(1, 6, 3, 224, 224)
    lo = model(x)
    with torch.no_grad():
        ref = mil(enc(x[0])[None])
    torch.testing.assert_close(lo.detach(), ref, rtol=0, atol=1e-5)
    lo.sum().backward()
    assert all(p.grad is None for p in enc.parameters())
    assert all(p.grad is not None for p in mil.parameters())


@pytest.mark.gpu
def test_folded_weights_follow_parent_loads_and_inplace_edits():
    """The eval-mode folded conv+BN weights are re-derived after a checkpoint loaded through a
    parent module (ImageBagModel.load_state_dict goes through _load_from_state_dict, not the
    encoder's own load_state_dict) and after an in-place BatchNorm statistics edit."""
    from transmil_deepgraft_amd.encoder import ImageBagModel
    from transmil_deepgraft_amd.models import TransMIL
    torch.backends.cudnn.allow_tf32 = False
    enc = _encoder(torch.float32).cuda()
    x = torch.from_numpy(encoder_tiles(2, seed=9)).cuda()
    with torch.no_grad():
        first = enc(x)
    other = _encoder(torch.float32)
    with torch.no_grad():
        other.bn1.running_mean.add_(0.5)
        other.layer1[0].conv1.weight.mul_(1.5)
    parent = ImageBagModel(enc, TransMIL(2, 2048).cuda())
    sd = {"model_ft." + k: v for k, v in other.state_dict().items()}
    sd.update({"model." + k: v for k, v in parent.model.state_dict().items()})
    parent.load_state_dict(sd)
    with torch.no_grad():
        after_load = enc(x)
        expect = other.cuda()(x)
    torch.testing.assert_close(after_load, expect, rtol=1e-5, atol=1e-5)
    assert not torch.allclose(after_load, first)
    with torch.no_grad():
        enc.bn1.running_mean.sub_(0.5)          # in place: back to the first statistics for bn1
        other.bn1.running_mean.sub_(0.5)
        torch.testing.assert_close(enc(x), other(x), rtol=1e-5, atol=1e-5)
