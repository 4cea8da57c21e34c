"""Pin the CPU oracle against the golden fixtures made from the reference itself.

The fixtures (tests/golden/*.npz) were produced by importing
``/root/reference/code/models/TransMIL.py`` (tests/golden/make_golden.py).
Everything here runs on the CPU.
"""
import numpy as np
import pytest
import torch

from golden_util import index, load, oracle_model, bag_input

SMALL = [k for k, v in index().items() if v.get("feat") == 64]


def _forward(model, x, grad=False, label=None, ncls=2):
    out = {}
    if grad:
        logits, (attn, padding) = model(x, return_attn=True)
        y = torch.tensor([label] * x.shape[0])
        loss = torch.nn.CrossEntropyLoss()(logits, torch.nn.functional.one_hot(y, ncls).to(logits.dtype))
        loss.backward()
        out["grads"] = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    else:
        with torch.no_grad():
            logits, (attn, padding) = model(x, return_attn=True)
    out.update(logits=logits.detach(), attn=attn.detach(), padding=padding)
    return out


@pytest.mark.parametrize("name", SMALL)
def test_oracle_matches_reference_fixture_fp32(name):
    fx = load(name)
    model = oracle_model(fx, torch.float32)
    x = torch.from_numpy(fx["x"])
    ncls = fx["w._fc.weight"].shape[0]
    r = _forward(model, x, grad=True, label=int(fx["label"][0]), ncls=ncls)
    np.testing.assert_allclose(r["logits"].numpy(), fx["logits"], rtol=0, atol=1e-6)
    assert int(r["padding"]) == int(fx["padding"])
    if "attn" in fx:
        np.testing.assert_allclose(r["attn"].numpy(), fx["attn"], rtol=0, atol=1e-6)
    for pname, g in r["grads"].items():
        np.testing.assert_allclose(g.numpy(), fx["grad." + pname], rtol=1e-5, atol=1e-6, err_msg=pname)


@pytest.mark.parametrize("name", SMALL)
def test_oracle_fp64_matches_reference_fp64(name):
    fx = load(name)
    model = oracle_model(fx, torch.float64)
    x = torch.from_numpy(fx["x"]).double()
    ncls = fx["w._fc.weight"].shape[0]
    # the reference casts the bag to fp32 (:174); the oracle does too, so feed fp64 weights via float()->double
    model_x = x
    orig = torch.Tensor.float
    torch.Tensor.float = lambda self, *a, **k: self
    try:
        r = _forward(model, model_x, grad=True, label=int(fx["label"][0]), ncls=ncls)
    finally:
        torch.Tensor.float = orig
    np.testing.assert_allclose(r["logits"].numpy(), fx["logits.f64"], rtol=0, atol=1e-12)
    for pname, g in r["grads"].items():
        np.testing.assert_allclose(g.numpy(), fx["grad." + pname + ".f64"], rtol=1e-9, atol=1e-12, err_msg=pname)


def test_fixture_noise_floor_fp32_vs_fp64():
    """fp32 vs fp64 reference logits differ far below the 1e-4 parity bar."""
    for name in SMALL + ["d512_n1024", "d512_n8192"]:
        fx = load(name)
        d = np.abs(fx["logits"] - fx["logits.f64"]).max()
        assert d < 2e-5, (name, d)


def test_oracle_d512_n1024_matches_fixture():
    from oracle.transmil_ref import TransMIL, deterministic_params_
    fx = load("d512_n1024")
    torch.manual_seed(0)
    m = deterministic_params_(TransMIL(2, 512, 512), 2021).eval()
    x = torch.from_numpy(bag_input(1024, 512, 2021 + 1000 + 1024))
    with torch.no_grad():
        logits = m(x)
    np.testing.assert_allclose(logits.numpy(), fx["logits"], rtol=0, atol=2e-6)


def test_pinv_matches_hf_iterative_inv():
    """Cross-check App. A eq. 7 against transformers' NystromformerSelfAttention.iterative_inv
    (init_option='original').  Their Z0 divides by max(colsum) only; for a softmax matrix
    max(rowsum) == 1 up to rounding, so both agree to rounding."""
    from transformers import NystromformerConfig
    from transformers.models.nystromformer.modeling_nystromformer import NystromformerSelfAttention
    from oracle.nystrom_ref import moore_penrose_iter_pinv
    cfg = NystromformerConfig(hidden_size=64, num_attention_heads=2, num_landmarks=8, segment_means_seq_len=64,
                              inv_coeff_init_option=False)
    att = NystromformerSelfAttention(cfg)
    att.init_option = "original"
    g = torch.Generator().manual_seed(3)
    x = torch.softmax(torch.randn(2, 8, 32, 32, generator=g, dtype=torch.float64) * 2, dim=-1)
    ours = moore_penrose_iter_pinv(x, 6)
    theirs = att.iterative_inv(x, 6)
    torch.testing.assert_close(ours, theirs, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("n,B", [(300, 2), (1025, 1), (8282, 1)])
def test_nystrom_eq2_to_9_match_hf_nystromformer(n, B):
    """Independent pin of SURVEY.md App. A eq. 2-9 (the arithmetic of the third-party
    ``nystrom_attention`` the reference calls at code/models/TransMIL.py:26-34,47) against
    transformers' ``NystromformerSelfAttention.forward``, which implements the same algorithm:
    segment-mean landmarks over the padded sequence (eq. 4), the three softmaxes (eq. 5-6),
    ``iterative_inv`` (eq. 7, init 'original'), ``(A1 Z)(A3 V)`` (eq. 8) and a depthwise (33, 1)
    conv on V (eq. 9).  HF scales q and k by dh^-1/4 each; the oracle scales q by dh^-1/2: the
    same products.  HF's Z0 divides by max(colsum) only; the oracle also by max(rowsum), which is
    1 up to rounding for a softmax.

    Mapping: the oracle's ``to_qkv`` row blocks become HF's query / key / value weights (zero
    biases), ``res_conv.weight`` becomes ``conv.weight``; HF is fed the already front-padded
    input (eq. 1, n' = n rounded up to 256) and its context layer is compared with the oracle's
    pre-``to_out`` activation (captured by a pre-hook on ``to_out[0]``), fp64, to 1e-9 relative.
    n' = 512 (B = 2: the global max couples the bags), 1280 (config C1) and 8448 (config C2)."""
    from transformers import NystromformerConfig
    from transformers.models.nystromformer.modeling_nystromformer import NystromformerSelfAttention
    from oracle.nystrom_ref import NystromAttention
    m = 256
    npad = (n + m - 1) // m * m
    g = torch.Generator().manual_seed(11 + n)
    ours = NystromAttention(dim=512, dim_head=64, heads=8, num_landmarks=m, pinv_iterations=6,
                            residual=True, dropout=0.7).double().eval()
    with torch.no_grad():
        for p in ours.parameters():
            p.copy_(torch.randn(p.shape, generator=g, dtype=torch.float64) * 0.05)
    cfg = NystromformerConfig(hidden_size=512, num_attention_heads=8, num_landmarks=m,
                              segment_means_seq_len=npad, conv_kernel_size=33,
                              inv_coeff_init_option=False, attention_probs_dropout_prob=0.0)
    hf = NystromformerSelfAttention(cfg).double().eval()
    assert hf.init_option == "original"
    w = ours.to_qkv.weight.detach()
    with torch.no_grad():
        for i, lin in enumerate((hf.query, hf.key, hf.value)):
            lin.weight.copy_(w[i * 512:(i + 1) * 512])
            lin.bias.zero_()
        hf.conv.weight.copy_(ours.res_conv.weight)
    x = torch.randn(B, n, 512, generator=g, dtype=torch.float64)
    got = {}
    handle = ours.to_out[0].register_forward_pre_hook(lambda _m, inp: got.__setitem__("ctx", inp[0]))
    try:
        with torch.no_grad():
            ours(x)
    finally:
        handle.remove()
    xpad = torch.cat([torch.zeros(B, npad - n, 512, dtype=torch.float64), x], dim=1)
    with torch.no_grad():
        theirs = hf(xpad)[0]
    ctx = got["ctx"]
    assert ctx.shape == theirs.shape == (B, npad, 512)
    rel = ((ctx - theirs).abs().max() / theirs.abs().max()).item()
    assert rel < 1e-9, rel


def test_pinv_global_max_couples_bags():
    """The Z0 scale uses maxima over the WHOLE [B,h,m,m] tensor (App. A eq. 7)."""
    from oracle.nystrom_ref import moore_penrose_iter_pinv
    g = torch.Generator().manual_seed(5)
    a = torch.softmax(torch.randn(1, 2, 16, 16, generator=g, dtype=torch.float64), dim=-1)
    b = torch.softmax(torch.randn(1, 2, 16, 16, generator=g, dtype=torch.float64) * 6, dim=-1)
    joint = moore_penrose_iter_pinv(torch.cat([a, b]), 6)
    alone = moore_penrose_iter_pinv(a, 6)
    assert (joint[0] - alone[0]).abs().max() > 1e-6


def _branch_oracle(name, dtype):
    from oracle.transmil_ref import TransMIL, deterministic_params_
    from oracle.mdmil_ref import MDMIL
    meta = index()[name]
    torch.manual_seed(0)
    m = MDMIL(2) if meta["model"] == "MDMIL" else TransMIL(2, meta["feat"], 512)
    deterministic_params_(m, 2021)
    x = torch.from_numpy(bag_input(meta["n"], meta["feat"], 2021 + 1000 + meta["n"]))
    return m.to(dtype).eval(), x.to(dtype), meta


@pytest.mark.parametrize("name", ["fc2048_n300", "mdmil_n300"])
def test_oracle_branches_match_reference_fixture(name):
    """The in_features=2048 TransMIL branch (code/models/TransMIL.py:100-111) and MDMIL
    (code/models/MDMIL.py:60-114) in the oracle against the reference's own outputs
    (tests/golden/make_golden_branches.py): fp32 logits 1e-6, fp64 logits / loss / small
    gradients 1e-10."""
    fx = load(name)
    for dt, tag, tol in ((torch.float32, "", 1e-6), (torch.float64, ".f64", 1e-10)):
        m, x, meta = _branch_oracle(name, dt)
        orig = torch.Tensor.float
        if dt == torch.float64:
            torch.Tensor.float = lambda self, *a, **k: self
        try:
            out = m(x)
        finally:
            torch.Tensor.float = orig
        logits = out[0] if isinstance(out, tuple) else out
        loss = torch.nn.CrossEntropyLoss()(logits, torch.nn.functional.one_hot(
            torch.tensor([meta["label"]]), 2).to(dt))
        loss.backward()
        np.testing.assert_allclose(logits.detach().numpy(), fx["logits" + tag], rtol=0, atol=tol)
        np.testing.assert_allclose(loss.detach().numpy().reshape(1), fx["loss" + tag], rtol=0, atol=tol)
        grads = dict(m.named_parameters())
        for k in fx:
            if k.startswith("grad.") and k.endswith(tag) and (tag or not k.endswith(".f64")):
                pname = k[5:len(k) - len(tag)] if tag else k[5:]
                np.testing.assert_allclose(grads[pname].grad.numpy(), fx[k], rtol=0, atol=tol * 10)


@pytest.mark.parametrize("name", ["d512_b4_n300", "d512_peaky_n1024"])
def test_oracle_matches_reference_d512_round2(name):
    """The CPU oracle (fp64) against the reference-run d=512 fixtures of round 2: B = 4 bags in one
    forward (global-max coupling) and q x 8 (tests/golden/make_golden_r2.py)."""
    from golden_util import index, load, bag_input
    from oracle.transmil_ref import TransMIL, deterministic_params_
    meta = index()[name]
    fx = load(name)
    torch.manual_seed(0)
    m = deterministic_params_(TransMIL(meta["n_classes"], 512, 512), 2021)
    if "peaky" in name:
        with torch.no_grad():
            for layer in (m.layer1, m.layer2):
                w = layer.attn.to_qkv.weight
                w[: w.shape[0] // 3] *= 8.0
    m = m.double().eval()
    x = torch.from_numpy(bag_input(meta["n"], 512, 2021 + 1000 + meta["n"], meta["batch"])).double()
    orig = torch.Tensor.float
    torch.Tensor.float = lambda self, *a, **k: self
    try:
        with torch.no_grad():
            lo = m(x).numpy()
    finally:
        torch.Tensor.float = orig
    np.testing.assert_allclose(lo, fx["logits.f64"], rtol=0, atol=1e-9)


def test_c3_oracle_fixture_matches_reference_fixture():
    """Config C3 (N = 32768): the round-1 oracle-generated fixture and the round-2 fixture from the
    reference's own TransMIL.py (placeholder return_attn value) hold the same logits."""
    from golden_util import load
    a, b = load("d512c3_n32768"), load("d512c3_ref_n32768")
    np.testing.assert_allclose(a["logits.f64"], b["logits.f64"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(a["logits"], b["logits"], rtol=0, atol=1e-5)


SIBLINGS = ["transmil768_n300", "ctmil_c64_g20_b2", "ctmil_c128_g36", "transformermil768_n200_b2",
            "transformermil2048_n64", "attmil2048_n500", "attmil1024_n300"]


def sibling_oracle(name, dtype=torch.float32):
    """The oracle model of a make_golden_siblings.py case, deterministic weights, eval mode."""
    from oracle import siblings_ref
    from oracle.transmil_ref import TransMIL, deterministic_params_
    meta = index()[name]
    klass = TransMIL if meta["model"] == "TransMIL" else getattr(siblings_ref, meta["model"])
    torch.manual_seed(0)
    m = klass(**meta["ctor"])
    deterministic_params_(m, 2021)
    return m.to(dtype).eval()


@pytest.mark.parametrize("name", SIBLINGS)
def test_sibling_oracles_match_reference_fixture(name):
    """oracle/siblings_ref.py (and the 768 branch of oracle/transmil_ref.py) against logits of
    the reference's own CTMIL.py / TransformerMIL.py / AttMIL.py / TransMIL.py (fp32 within
    summation-order noise; fp64 to 1e-10)."""
    from golden_util import sibling_input
    ref = load(name)
    x = torch.from_numpy(sibling_input(name))
    orig = torch.Tensor.float
    with torch.no_grad():
        out = sibling_oracle(name)(x).numpy()
        torch.Tensor.float = lambda self, *a, **k: self     # TransMIL casts the bag to fp32 (:174)
        try:
            out64 = sibling_oracle(name, torch.float64)(x.double()).numpy()
        finally:
            torch.Tensor.float = orig
    np.testing.assert_allclose(out, ref["logits"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(out64, ref["logits.f64"], rtol=1e-10, atol=1e-12)
