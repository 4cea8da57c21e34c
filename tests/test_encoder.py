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
