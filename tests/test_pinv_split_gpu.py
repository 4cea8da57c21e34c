"""The split-operand pseudo-inverse chain (pinv_split.hip, bf16 bench mode) against the fp64
restatement of moore_penrose_iter_pinv (oracle/nystrom_ref.py, SURVEY.md App. A eq. 7) and
against the fp32-storage bf16x3 chain (pinv.hip) it replaces.  Tolerances: the split planes hold
every chain matrix to ~2^-17 relative and the products drop lo*lo (~2^-16), so Z and the
softmax-side gradient agree with fp64 to a few 1e-4 (the exact-fp32 chain reaches 2e-4 / 2e-3)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _split(x):
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd.engine import _p, _stream
    y = torch.empty(2 * x.numel(), dtype=torch.bfloat16, device=DEV)
    _lib.call("tm_split_f32", _p(x), _p(y), x.numel(), _stream())
    return y


def _run_split(X, gz, nbh, softmax=1, iters=6):
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd.engine import _p, _stream
    Xs = _split(X)
    saved = torch.full((_lib.query("tm_pinv_split_saved_floats", nbh, iters),), float("nan"), device=DEV)
    _lib.call("tm_pinv_fwd_split", _p(X), _p(Xs), nbh, iters, _p(saved), _stream())
    z = saved[:nbh * 65536].view(nbh, 256, 256).clone()
    work = torch.full((_lib.query("tm_pinv_bwd_split_workspace_floats", nbh),), float("nan"), device=DEV)
    _lib.call("tm_split_f32", _p(gz), _p(work), gz.numel(), _stream())
    out = torch.full((nbh, 256, 256), float("nan"), device=DEV)
    _lib.call("tm_pinv_bwd_split", _p(X), _p(Xs), nbh, iters, _p(saved), _p(work), softmax, _p(out), _stream())
    torch.cuda.synchronize()
    return z, out


def test_split_planes_roundtrip():
    x = torch.randn(8 * 65536, device=DEV) * torch.logspace(-6, 3, 8 * 65536, device=DEV)
    y = _split(x)
    hi, lo = y[:x.numel()].float(), y[x.numel():].float()
    assert torch.equal(y[:x.numel()], x.to(torch.bfloat16))
    assert ((hi + lo - x).abs() <= x.abs() * 2.0 ** -16).all()


def test_sim2_softmax_split_matches_fp32():
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd.engine import _p, _stream
    nbh = 8
    g = torch.Generator().manual_seed(3)
    ql = (torch.randn(nbh, 256, 64, generator=g) * 0.2).to(DEV)
    kl = (torch.randn(nbh, 256, 64, generator=g) * 0.2).to(DEV)
    a2 = torch.empty(nbh, 256, 256, device=DEV)
    a2s = torch.empty(2 * nbh * 65536, dtype=torch.bfloat16, device=DEV)
    _lib.call("tm_nys_sim2_softmax_split", _p(ql), _p(kl), nbh, _p(a2), _p(a2s), _stream())
    ref = torch.empty_like(a2)
    _lib.call("tm_nys_sim2_softmax", _p(ql), _p(kl), nbh, _p(ref), _stream())
    torch.cuda.synchronize()
    assert torch.equal(a2, ref)
    assert torch.equal(a2s[:nbh * 65536].view_as(a2), a2.to(torch.bfloat16))
    rec = a2s[:nbh * 65536].float() + a2s[nbh * 65536:].float()
    assert ((rec - a2.flatten()).abs() <= a2.flatten().abs() * 2.0 ** -16).all()
    exact = torch.softmax(ql.double() @ kl.double().transpose(1, 2), -1)
    assert ((ref.double() - exact).abs().max() / exact.abs().max()).item() < 1e-6
    assert ((a2.double() - exact).abs().max() / exact.abs().max()).item() < 1e-4
    assert torch.allclose(a2.double().sum(-1), torch.ones(nbh, 256, dtype=torch.float64, device=DEV), atol=1e-5)


@pytest.mark.parametrize("nbh", [8, 16, 24])
def test_pinv_split_fwd_bwd_vs_fp64(nbh):
    """Z_6 and dL/ds (s the sim2 logits, A2 = softmax(s)) against fp64 autograd through the
    restatement; nbh = 16 / 24 are B = 2 / 3 bags sharing one global max (App. A eq. 7)."""
    from oracle.nystrom_ref import moore_penrose_iter_pinv
    g = torch.Generator().manual_seed(100 + nbh)
    s64 = (torch.randn(nbh, 256, 256, generator=g, dtype=torch.float64) * 0.3).requires_grad_()
    a64 = torch.softmax(s64, dim=-1)
    z_ref = moore_penrose_iter_pinv(a64, 6)
    gz = torch.randn(nbh, 256, 256, generator=g, dtype=torch.float64) * 1e-3
    z_ref.backward(gz)
    X = a64.detach().float().to(DEV).contiguous()
    z, ds = _run_split(X, gz.float().to(DEV).contiguous(), nbh)
    assert torch.isfinite(z).all() and torch.isfinite(ds).all()
    assert _rel(z.cpu(), z_ref.detach()) < 5e-4
    assert _rel(ds.cpu(), s64.grad) < 4e-3


def test_pinv_split_matches_fp32_storage_chain():
    """Same products as tm_pinv_fwd / tm_pinv_bwd (prec 1): Z and the softmax-side gradient agree
    closely (dL/dA2 itself differs by the row-constant max-tie term wherever fp32 rounding makes
    the two chains' |X| sums tie differently; the softmax backward annihilates it)."""
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd.engine import _p, _stream
    nbh = 8
    g = torch.Generator().manual_seed(21)
    X = torch.softmax(torch.randn(nbh, 256, 256, generator=g) * 0.3, dim=-1).to(DEV)
    gz = (torch.randn(nbh, 256, 256, generator=g) * 1e-3).to(DEV)
    saved = torch.empty(_lib.query("tm_pinv_saved_floats", nbh, 6), device=DEV)
    _lib.call("tm_pinv_fwd", _p(X), nbh, 6, 1, _p(saved), _stream())
    z_old = saved[6 * nbh * 65536:7 * nbh * 65536].view(nbh, 256, 256).clone()
    work = torch.empty(_lib.query("tm_pinv_bwd_workspace_floats", nbh), device=DEV)
    dX_old = torch.empty(nbh, 256, 256, device=DEV)
    _lib.call("tm_pinv_bwd", _p(X), nbh, 6, 1, _p(saved), _p(gz.clone()), _p(work), _p(dX_old), _stream())
    ds_old = torch.empty_like(dX_old)
    _lib.call("tm_softmax_bwd_rows256", _p(X), _p(dX_old), _p(ds_old), nbh * 256, _stream())
    z, ds = _run_split(X, gz, nbh, softmax=1)
    _, dX = _run_split(X, gz, nbh, softmax=0)
    ds2 = torch.empty_like(dX)
    _lib.call("tm_softmax_bwd_rows256", _p(X), _p(dX), _p(ds2), nbh * 256, _stream())
    torch.cuda.synchronize()
    assert _rel(z.cpu(), z_old.cpu()) < 5e-4
    assert _rel(ds.cpu(), ds_old.cpu()) < 4e-3
    assert _rel(ds2.cpu(), ds.cpu()) < 1e-6   # the fused softmax backward = the separate kernel


def test_pinv_split_peaky_and_iters():
    """Sharper softmax rows (logits x 4) and a shorter chain (iters = 2, 3) stay finite and
    close to fp64."""
    from oracle.nystrom_ref import moore_penrose_iter_pinv
    nbh = 8
    for iters, scale in ((6, 1.2), (2, 0.3), (3, 0.3)):
        g = torch.Generator().manual_seed(7 + iters)
        a64 = torch.softmax(torch.randn(nbh, 256, 256, generator=g, dtype=torch.float64) * scale, dim=-1)
        z_ref = moore_penrose_iter_pinv(a64, iters)
        gz = torch.zeros(nbh, 256, 256, device=DEV)
        z, _ = _run_split(a64.float().to(DEV).contiguous(), gz, nbh, iters=iters)
        assert torch.isfinite(z).all()
        assert _rel(z.cpu(), z_ref) < 1e-3, (iters, scale)


@pytest.mark.parametrize("nbh,n", [(8, 8448), (16, 1280)])
def test_pinv_fwd_with_a3_combine_equals_separate_launches(nbh, n):
    """tm_pinv_fwd_split_a3 (the A3 forward's partial combine inside the chain's last launch) =
    tm_nys_a3_fwd's own combine launch + tm_pinv_fwd_split, bit for bit (same routine, same order)."""
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd._lib import BF16
    from transmil_deepgraft_amd.engine import _p, _stream
    g = torch.Generator().manual_seed(n + nbh)
    ql = (torch.randn(nbh, 256, 64, generator=g) * 0.4).to(DEV)
    k = (torch.randn(nbh, n, 64, generator=g) * 0.4).to(torch.bfloat16).to(DEV)
    v = torch.randn(nbh, n, 64, generator=g).to(torch.bfloat16).to(DEV)
    X = torch.softmax(torch.randn(nbh, 256, 256, generator=g) * 0.3, dim=-1).to(DEV)
    Xs = _split(X)
    work = torch.empty(_lib.query("tm_nys_a3_workspace", nbh, n) // 4 + 16, device=DEV)
    w_ref = torch.full((nbh, 256, 64), float("nan"), device=DEV)
    lse_ref = torch.full((nbh, 256), float("nan"), device=DEV)
    _lib.call("tm_nys_a3_fwd", BF16, _p(ql), _p(k), _p(v), nbh, n, _p(work), _p(w_ref), _p(lse_ref), _stream())
    saved_ref = torch.full((_lib.query("tm_pinv_split_saved_floats", nbh, 6),), float("nan"), device=DEV)
    _lib.call("tm_pinv_fwd_split", _p(X), _p(Xs), nbh, 6, _p(saved_ref), _stream())
    w = torch.full_like(w_ref, float("nan"))
    lse = torch.full_like(lse_ref, float("nan"))
    _lib.call("tm_nys_a3_fwd", BF16, _p(ql), _p(k), _p(v), nbh, n, _p(work), _p(None), _p(None), _stream())
    saved = torch.full_like(saved_ref, float("nan"))
    _lib.call("tm_pinv_fwd_split_a3", _p(X), _p(Xs), nbh, 6, _p(saved), _p(work), _lib.query("tm_nys_a3_partials", nbh, n),
              _p(w), _p(lse), _stream())
    torch.cuda.synchronize()
    assert torch.equal(w, w_ref) and torch.equal(lse, lse_ref)
    zn = nbh * 65536
    assert torch.equal(saved[:zn], saved_ref[:zn])


@pytest.mark.gpu
@pytest.mark.parametrize("nbh,n", [(8, 8448), (16, 1280), (8, 256), (2, 4096)])
def test_a3_fwd_with_sim2_equals_separate_launches(nbh, n):
    """tm_nys_a3_fwd_sim2 (the A2 rows written by the A3 forward's workgroups) = tm_nys_a3_fwd
    (deferred combine) + tm_nys_sim2_softmax_split, bit for bit: same partials, same A2 and planes
    (the split tiles the 256 rows at (8, 8448) and (16, 1280); the others take the two-launch path)."""
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd._lib import BF16
    from transmil_deepgraft_amd.engine import _p, _stream
    g = torch.Generator().manual_seed(7 * n + nbh)
    ql = (torch.randn(nbh, 256, 64, generator=g) * 0.4).to(DEV)
    kl = (torch.randn(nbh, 256, 64, generator=g) * 0.4).to(DEV)
    k = (torch.randn(nbh, n, 64, generator=g) * 0.4).to(torch.bfloat16).to(DEV)
    v = torch.randn(nbh, n, 64, generator=g).to(torch.bfloat16).to(DEV)
    nw = _lib.query("tm_nys_a3_workspace", nbh, n) // 4
    work_ref = torch.full((nw,), float("nan"), device=DEV)
    a2_ref = torch.full((nbh, 256, 256), float("nan"), device=DEV)
    a2s_ref = torch.full((2 * nbh * 65536,), float("nan"), device=DEV).to(torch.bfloat16)
    _lib.call("tm_nys_a3_fwd", BF16, _p(ql), _p(k), _p(v), nbh, n, _p(work_ref), _p(None), _p(None), _stream())
    _lib.call("tm_nys_sim2_softmax_split", _p(ql), _p(kl), nbh, _p(a2_ref), _p(a2s_ref), _stream())
    work = torch.full_like(work_ref, float("nan"))
    a2 = torch.full_like(a2_ref, float("nan"))
    a2s = torch.full_like(a2s_ref, float("nan"))
    _lib.call("tm_nys_a3_fwd_sim2", _p(ql), _p(kl), _p(k), _p(v), nbh, n, _p(work), _p(a2), _p(a2s), _stream())
    torch.cuda.synchronize()
    P = _lib.query("tm_nys_a3_partials", nbh, n)
    # the partial sums are bf16 in the first half of an fp32-sized region, then (m, l) fp32
    o_half, o_full = P * nbh * 256 * 32, P * nbh * 256 * 64
    wb, wr = work.view(torch.int32), work_ref.view(torch.int32)   # bit patterns (two bf16 per word)
    assert torch.equal(wb[:o_half], wr[:o_half])
    assert torch.equal(wb[o_full:o_full + 2 * P * nbh * 256], wr[o_full:o_full + 2 * P * nbh * 256])
    assert torch.equal(a2, a2_ref) and torch.equal(a2s, a2s_ref)
    assert torch.allclose(a2.sum(-1), torch.ones(nbh, 256, device=DEV), atol=1e-5)
