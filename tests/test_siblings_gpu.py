"""The sibling heads and the 768 _fc1 branch on the GPU against the reference.

Forward: logits of the reference's own CTMIL.py / TransformerMIL.py / AttMIL.py / TransMIL.py
(fixtures from tests/golden/make_golden_siblings.py), fp32 compute mode.  Backward: every
parameter gradient against autograd through the oracle restatement (oracle/siblings_ref.py,
pinned by the same fixtures; CPU fp64), normwise.  bf16 mode: logits close, argmax equal."""
import numpy as np
import pytest
import torch

from golden_util import load, sibling_input
from test_oracle import SIBLINGS, sibling_oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ours(name, dtype=torch.float32):
    from transmil_deepgraft_amd import models
    from golden_util import index
    meta = index()[name]
    ref = sibling_oracle(name)
    ours = getattr(models, meta["model"])(**meta["ctor"])
    missing = ours.load_state_dict(ref.state_dict(), strict=True)
    assert not missing.missing_keys and not missing.unexpected_keys
    ours = ours.to(DEV).eval()
    if hasattr(ours, "set_compute_dtype"):
        ours.set_compute_dtype(dtype)
    return ref, ours


def _loss(logits, ncls):
    y = torch.zeros(logits.shape[0], dtype=torch.long, device=logits.device)
    return torch.nn.CrossEntropyLoss()(logits, torch.nn.functional.one_hot(y, ncls).to(logits.dtype))


@pytest.mark.parametrize("name", SIBLINGS)
def test_sibling_logits_and_grads_fp32(name):
    fx = load(name)
    ref, ours = _ours(name)
    x = torch.from_numpy(sibling_input(name))
    lo = ours(x.to(DEV))
    np.testing.assert_allclose(lo.detach().cpu().numpy(), fx["logits"], rtol=0, atol=2e-4)
    ncls = lo.shape[1]
    _loss(lo, ncls).backward()
    # gradients against the fp64 oracle: some are ill-conditioned in fp32 (CTMIL's res_conv
    # weight differs by 9e-2 between the fp32 and fp64 oracle; AttMIL's attention bias is
    # exactly 0 in exact arithmetic), so the reference point is fp64 with an absolute floor
    ref = ref.double()
    orig = torch.Tensor.float
    torch.Tensor.float = lambda self, *a, **k: self
    try:
        _loss(ref(x.double()), ncls).backward()
    finally:
        torch.Tensor.float = orig
    for (n, pr), po in zip(ref.named_parameters(), ours.parameters()):
        if pr.grad is None:
            assert po.grad is None or not po.grad.any(), n      # unused modules stay unused
            continue
        assert po.grad is not None, n
        g, gr = po.grad.cpu().double(), pr.grad
        err = (g - gr).norm()
        assert err < 2e-3 * gr.norm() + 1e-6, f"{n}: err {err:.2e} vs norm {gr.norm():.2e}"


@pytest.mark.parametrize("name", ["transmil768_n300", "ctmil_c128_g36", "transformermil768_n200_b2",
                                  "attmil2048_n500"])
def test_sibling_bf16_mode(name):
    fx = load(name)
    _, ours = _ours(name, torch.bfloat16)
    with torch.no_grad():
        lo = ours(torch.from_numpy(sibling_input(name)).to(DEV)).cpu().numpy()
    np.testing.assert_allclose(lo, fx["logits"], rtol=0, atol=6e-2)


def test_attmil_pool_kernel_large_bag():
    """N = 8192 (the bench bag size): gated pooling forward/backward against the same math in
    torch fp64 on the GPU's own _fc1 output."""
    from transmil_deepgraft_amd.models import AttMIL
    torch.manual_seed(0)
    m = AttMIL(2, 1024, 512).to(DEV).eval()
    x = torch.rand(1, 8192, 1024, device=DEV)
    h = m._embed(x)[0].detach().requires_grad_(True)
    from transmil_deepgraft_amd.models.AttMIL import _GatedPoolFn
    V, U = m.attention_V[0], m.attention_U[0]
    args = (torch.cat([V.weight, U.weight]), torch.cat([V.bias, U.bias]), m.attention_weights.weight,
            m.attention_weights.bias, m.classifier[0].weight, m.classifier[0].bias)
    lo = _GatedPoolFn.apply(h, *args)
    dl = torch.tensor([[0.3, -0.7]], device=DEV)
    (lo * dl).sum().backward()
    hd = h.detach().double().requires_grad_(True)
    ad = [a.detach().double().requires_grad_(True) for a in args]
    z = hd @ ad[0].T + ad[1]
    s = (torch.tanh(z[:, :128]) * torch.sigmoid(z[:, 128:])) @ ad[2].T + ad[3]
    p = torch.softmax(s.T, dim=1)
    ld = (p @ hd) @ ad[4].T + ad[5]
    (ld * dl.double()).sum().backward()
    torch.testing.assert_close(lo.double(), ld, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(h.grad.double(), hd.grad, rtol=1e-4, atol=1e-8)


@pytest.mark.parametrize("name", SIBLINGS + ["mdmil_n300"])
def test_sibling_configure_optimizers_steps_like_torch_radam(name):
    """``TransMILTask(model).configure_optimizers()`` (the reference's lookahead_radam,
    code/MyOptimizer/optim_factory.py:77-79,118-121) on every sibling head: parameters that never
    get a gradient (CTMIL._fc1, AttMIL.feature_extractor_part2, TransformerMIL's pos_layer_0 /
    conv / layer modules) are skipped as torch.optim.RAdam skips ``grad is None``, and a model
    with more than 40 parameter tensors (TransformerMIL) falls back to torch RAdam.  7 steps (one
    Lookahead sync) against torch.optim.RAdam + the reference Lookahead on an identical model."""
    from test_interface import RefLookahead
    from transmil_deepgraft_amd.interface import TransMILTask, add_weight_decay
    from golden_util import index
    meta = index()[name]
    if name.startswith("mdmil"):
        from oracle.mdmil_ref import MDMIL as RefMD
        from oracle.transmil_ref import deterministic_params_
        from transmil_deepgraft_amd.models import MDMIL
        from golden_util import bag_input
        pair = []
        for _ in range(2):
            torch.manual_seed(0)
            m = MDMIL(2)
            m.load_state_dict(deterministic_params_(RefMD(2), 2021).state_dict())
            pair.append(m.to(DEV).train().set_compute_dtype(torch.float32))
        x = torch.from_numpy(bag_input(meta["n"], meta["feat"], 2021 + 1000 + meta["n"])).to(DEV)
    else:
        pair = [_ours(name)[1].train() for _ in range(2)]
        x = torch.from_numpy(sibling_input(name)).to(DEV)
    a, b = pair
    for m in pair:
        if hasattr(m, "_dropout_counter"):
            m._dropout_counter.fill_(12345)
    opt_a = TransMILTask(a).configure_optimizers()[0][0]
    opt_b = RefLookahead(torch.optim.RAdam(add_weight_decay(b, 0.01), lr=2e-4))
    for step in range(7):
        for m, opt in ((a, opt_a), (b, opt_b)):
            torch.manual_seed(100 + step)       # the same torch Dropout draws in both models
            out = m(x)
            lo = out[0] if isinstance(out, tuple) else out
            _loss(lo, lo.shape[1]).backward()
            opt.step()
            (opt.zero_grad if hasattr(opt, "zero_grad") else opt.base.zero_grad)(set_to_none=True)
    torch.cuda.synchronize()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=2e-5, atol=2e-6, msg=lambda m, n=n: f"{n}: {m}")
    start = _ours(name)[1].state_dict() if not name.startswith("mdmil") else None
    if start is not None:
        moved = max((p.detach() - start[n].to(DEV)).abs().max().item() for n, p in a.named_parameters())
        assert moved > 0
