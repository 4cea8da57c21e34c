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


def test_encoder_oracle_pinned_by_reference_fixture():
    """oracle/encoder_ref.py (functional ResNet-50, eval BN) reproduces the features the reference's
    own ResNet.py computed for the fixture's 4 tiles (fp64: to rounding; fp32: 1e-5)."""
    from oracle.encoder_ref import features
    fx = load("retccl_r50_tiles4")
    sd = _encoder().state_dict()
    x = torch.from_numpy(encoder_tiles(4))
    np.testing.assert_allclose(features(x, sd).numpy(), fx["feats.f64"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(features(x, sd, torch.float32).numpy(), fx["feats"], rtol=1e-5, atol=1e-5)


def test_library_calls_stay_below_2_gib():
    """Every library convolution / pooling of the encoder is handed < 2 GiB per tensor (MIOpen's
    implicit-GEMM NHWC kernels wrap 32-bit offsets beyond that: scripts/dev/c5_drift.py measured
    wrong outputs for tiles >= 2674 of a one-pass 4096-tile fp32 bag).  The guard refuses a
    669-tile fp32 stem input (its output, 669 x 64 x 112 x 112 x 4 B, reaches 2^31 bytes) before it
    reaches MIOpen, a 668-tile one passes; bf16 doubles the cap (meta tensors: shapes only)."""
    from transmil_deepgraft_amd import encoder as E
    assert E.tile_elems_max(224, 224) == 64 * 112 * 112
    for dt, esz, cap_expect in ((torch.float32, 4, 668), (torch.bfloat16, 2, 1337)):
        cap = E.max_tiles_per_call(224, 224, esz)
        assert cap == cap_expect and cap * 64 * 112 * 112 * esz <= 2 ** 31 - 1 < (cap + 1) * 64 * 112 * 112 * esz
        w = torch.empty(64, 3, 7, 7, device="meta", dtype=dt)
        y = E._lib_conv2d(torch.empty(cap, 3, 224, 224, device="meta", dtype=dt), w, stride=2, padding=3)
        assert tuple(y.shape) == (cap, 64, 112, 112)
        with pytest.raises(RuntimeError, match="2\\^31"):
            E._lib_conv2d(torch.empty(cap + 1, 3, 224, 224, device="meta", dtype=dt), w, stride=2, padding=3)
        with pytest.raises(RuntimeError, match="2\\^31"):
            E._lib_max_pool(torch.empty(cap + 1, 64, 112, 112, device="meta", dtype=dt))
        E._lib_max_pool(torch.empty(cap, 64, 112, 112, device="meta", dtype=dt))


def test_train_pieces_respect_the_statistics_call_and_the_library_limit():
    """Train-mode bag pieces: at least ``chunk`` tiles, at most 64 pieces per BatchNorm statistics
    call (tm_bn_train_stats), never more than max_tiles_per_call() tiles; a bag no piece size can
    serve raises instead of failing inside the statistics call."""
    from transmil_deepgraft_amd.encoder import max_tiles_per_call, train_pieces
    cap4, cap2 = max_tiles_per_call(elem_bytes=4), max_tiles_per_call(elem_bytes=2)
    assert train_pieces(4096, 512) == 512                          # C5 fp32: 8 pieces
    assert train_pieces(4096, 1024, elem_bytes=2) == 1024          # C5 bf16 (bench_c5): 4 pieces
    assert train_pieces(4096, 4096) == cap4                        # chunk above the cap: clamped
    assert train_pieces(4096, 4096, elem_bytes=2) == cap2
    assert train_pieces(6, 2) == 2
    assert train_pieces(40000, 512, elem_bytes=2) == 625           # 64 pieces of 625 tiles
    assert train_pieces(64 * cap4, 512) == cap4
    with pytest.raises(RuntimeError, match="64 pieces"):
        train_pieces(64 * cap4 + 1, 512)


C5_TILES = 4096     # BASELINE config C5: one slide of 4096 224x224 tiles


@pytest.mark.gpu
@pytest.mark.parametrize("enc_dtype,mil_dtype,rtol,ltol,gtol", [
    (torch.float32, torch.float32, 2e-3, 1e-4, 2e-3),       # parity mode end to end
    (torch.bfloat16, torch.bfloat16, 6e-2, 5e-2, 6e-2),     # the bench mode (C2 bf16 tolerances)
])
def test_c5_full_bag_4096_tiles(enc_dtype, mil_dtype, rtol, ltol, gtol):
    """Config C5 at its own size on one GPU (code/models/model_interface.py:237-247,297-316;
    code/models/ResNet.py:130-277): a 4096-tile bag [1, 4096, 3, 224, 224] through ImageBagModel ->
    RetCCL ResNet-50 (eval, BN folded) -> TransMIL(2, 2048) (RCC _fc1 branch).
      * 16 tiles spread over the bag: encoder features against the fixture-pinned fp64 oracle
        (oracle/encoder_ref.py), per-tile relative L2 error < rtol;
      * the whole-bag features (the encoder's internal 512-tile chunks) equal to running the 8
        chunks of 512 tiles one by one (fp32 bitwise, bf16 within a rounding);
      * TransMIL logits / every parameter gradient on the GPU-computed features against the fp64
        TransMIL oracle on the same features (C2 tolerances for the mode);
      * one train step of the image model (dropout on, Lookahead(RAdam)) finite and moving."""
    from oracle.encoder_ref import features
    from test_parity_gpu import _pair, _ref_forward_backward, _ours_forward_backward
    from transmil_deepgraft_amd.encoder import ImageBagModel
    from transmil_deepgraft_amd.interface import TransMILTask
    torch.backends.cudnn.allow_tf32 = False
    enc = _encoder(enc_dtype).cuda()
    g = torch.Generator(device="cuda").manual_seed(4096)
    tiles = torch.randn(1, C5_TILES, 3, 224, 224, device="cuda", generator=g)
    with torch.no_grad():
        whole = enc(tiles[0])
        chunks = torch.cat([enc(tiles[0, s:s + 512]) for s in range(0, C5_TILES, 512)])
    torch.cuda.synchronize()
    assert torch.isfinite(whole).all()
    idx = torch.linspace(0, C5_TILES - 1, 16).round().long()
    ref = features(tiles[0, idx.cuda()].float().cpu(), enc.state_dict())
    got = whole[idx.cuda()].double().cpu()
    err = ((got - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    assert err < rtol, err
    # the bag goes through in the encoder's 512-tile chunks: the same kernels as 8 separate calls.
    # (A one-pass 4096-tile batch is refused by encoder._lib_guard: MIOpen's NHWC implicit-GEMM
    # kernel for layer2.0's stride-2 3x3 convolution returned wrong outputs for tiles >= 2674 of it,
    # profiles/r05_c5_drift.json -- the round-4 one-pass drift.)
    # fp32: bit-identical.  bf16: the hipBLASLt 1x1 algorithm of each shape is chosen by timing
    # (tm_conv1x1_tune) and some candidates sum split-K / stream-K partials in a run-dependent order,
    # so an M tile that straddles two images may round differently run to run (two adjacent tiles
    # of 4096 seen, scripts/dev/c5_whole_vs_chunks.py); the chunking property is then held to a
    # bf16 rounding instead -- the offset-wrap defect this guards against was a 0.12-0.35 error
    diff = (whole - chunks).norm(dim=1) / chunks.norm(dim=1)
    if enc_dtype == torch.float32:
        assert torch.equal(whole, chunks), (whole != chunks).any(dim=1).nonzero().flatten().tolist()[:16]
    else:
        assert diff.max().item() < 1e-2, (diff.max().item(), diff.argmax().item())

    # TransMIL(2, 2048) on the GPU features against the fp64 oracle on the same features
    refm, ours = _pair(2, feat=2048, dtype=mil_dtype)
    feats = whole.view(1, C5_TILES, 2048).cpu()
    lo, go = _ours_forward_backward(ours, feats, 1, 2)
    lr, gr = _ref_forward_backward(refm, feats, 1, 2)
    np.testing.assert_allclose(lo.numpy(), lr.numpy(), rtol=0, atol=ltol)
    bad = [(n, e) for n, e in (((n, ((go[n].double() - g_).abs().max() / g_.abs().max().clamp_min(1e-12)).item())
                                for n, g_ in gr.items())) if e > gtol]
    assert not bad, bad

    # one train step of the image model
    ours.train().zero_grad(set_to_none=True)
    model = ImageBagModel(enc, ours)
    task = TransMILTask(ours)
    opt = task.configure_optimizers()[0][0]
    before = {n: p.detach().clone() for n, p in ours.named_parameters()}
    logits = model(tiles)
    loss = task.loss(logits, torch.nn.functional.one_hot(torch.tensor([1], device="cuda"), 2).float())
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all() and loss.item() > 0
    assert all(p.grad is None for p in enc.parameters())
    moved = max((p.detach() - before[n]).abs().max().item() for n, p in ours.named_parameters())
    assert 0 < moved < 1 and all(torch.isfinite(p).all() for p in ours.parameters())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,rtol,stol", [(torch.float32, 2e-3, 1e-3), (torch.bfloat16, 6e-2, 3e-2)])
def test_train_mode_bn_uses_whole_bag_statistics(dtype, rtol, stol):
    """Train-mode encoder (frozen parameters, BatchNorm in training mode, as the reference's
    model_ft under Lightning's model.train()): the batch statistics span every tile of the bag,
    because ModelInterface.forward feeds model_ft the whole [B*bag] batch in one call
    (model_interface.py:303-309).  With chunk (2) < bag (6) the features and the updated running
    statistics still equal the fp64 oracle's whole-batch train-mode BN."""
    from oracle.encoder_ref import features
    enc = _encoder(dtype)
    enc.chunk = 2
    sd0 = {k: v.clone() for k, v in enc.state_dict().items()}
    enc = enc.cuda().train()
    x = torch.from_numpy(encoder_tiles(6, seed=3))
    with torch.no_grad():
        got = enc(x.cuda()).double().cpu()
    stats = {}
    ref = features(x, sd0, train=True, momentum=0.1, stats_out=stats)
    err = ((got - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    assert err < rtol, err
    sd = enc.state_dict()
    worst = max(((sd[k].double().cpu() - v).abs().max() / v.abs().max().clamp_min(1e-6)).item()
                for k, v in stats.items())
    assert worst < stol, worst


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("rows,cin,cout", [(3136 * 2, 64, 256), (49 * 3 + 5, 512, 2048), (100, 1024, 256)])
@pytest.mark.parametrize("relu,res", [(True, True), (True, False), (False, False)])
def test_conv1x1_epilogue_matches_torch(dtype, tol, rows, cin, cout, relu, res):
    """tm_conv1x1 (hipBLASLt GEMM, bias / residual / ReLU epilogue) against an fp32 torch
    reference act(x w^T + b (+ r)) -- the order ResNet.py:95-117 applies them."""
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd.encoder import _dtype_code
    from transmil_deepgraft_amd.engine import _p, _stream
    g = torch.Generator(device="cuda").manual_seed(rows + cin)
    x = torch.randn(rows, cin, device="cuda", generator=g).to(dtype)
    w = (torch.randn(cout, cin, device="cuda", generator=g) / cin ** 0.5).to(dtype)
    b = torch.randn(cout, device="cuda", generator=g).to(dtype)
    r = torch.randn(rows, cout, device="cuda", generator=g).to(dtype) if res else None
    y = torch.full((rows, cout), float("nan"), device="cuda", dtype=dtype)
    _lib.call("tm_conv1x1", _dtype_code(x), _p(x), _p(w), _p(b), _p(r), _p(y), rows, cin, cout, int(relu), None, 0,
              _stream())
    ref = x.float() @ w.float().t() + b.float() + (r.float() if res else 0)
    ref = ref.clamp_min(0) if relu else ref
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol * ref.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bias_act_matches_torch(dtype):
    from transmil_deepgraft_amd.encoder import _bias_act_
    g = torch.Generator(device="cuda").manual_seed(5)
    y = torch.randn(3, 128, 7, 9, device="cuda", generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
    b = torch.randn(128, device="cuda", generator=g).to(dtype)
    ref = (y.float() + b.float()[None, :, None, None]).clamp_min(0).to(dtype)
    out = _bias_act_(y, b)
    assert out.data_ptr() == y.data_ptr()
    torch.testing.assert_close(out, ref, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,C", [(4096 * 49, 2048), (512 * 3136 + 7, 64), (33, 256)])
def test_bn_train_kernels_match_fp64(dtype, rows, C):
    """tm_bn_train_stats / tm_bn_apply against fp64 batch statistics on the same (rounded)
    input: values offset by 3 with spread 0.5 (E[x^2] - E[x]^2 would cancel in fp32 without the
    shift), running statistics with momentum 0.1 and the unbiased variance (nn.BatchNorm2d)."""
    from transmil_deepgraft_amd.encoder import _bn_apply_, _bn_train_stats
    g = torch.Generator(device="cuda").manual_seed(rows % 1000 + C)
    x = (3 + 0.5 * torch.randn(rows, C, device="cuda", generator=g)).to(dtype)
    x4 = x.view(1, rows, 1, C).permute(0, 3, 1, 2)               # channels-last [1, C, rows, 1]
    bn = torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.2, 0.2, generator=g)
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    ws = torch.empty(4 * 2048 * 2048, device="cuda")
    cut = rows // 3 if rows > 64 else rows          # two pieces (or one): statistics span them
    st = _bn_train_stats([x4[:, :, :cut]] + ([x4[:, :, cut:]] if cut < rows else []), bn, ws)
    xd = x.double()
    mean, var = xd.mean(0), xd.var(0, unbiased=False)
    sc = bn.weight.double() / torch.sqrt(var + bn.eps)
    torch.testing.assert_close(st[0].double(), sc, rtol=1e-5, atol=0)
    torch.testing.assert_close(st[1].double(), bn.bias.double() - mean * sc, rtol=0, atol=1e-5 * sc.abs().max().item() * 4)
    torch.testing.assert_close(bn.running_mean.double(), 0.9 * rm0.double() + 0.1 * mean, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(bn.running_var.double(), 0.9 * rv0.double() + 0.1 * xd.var(0, unbiased=True),
                               rtol=1e-5, atol=1e-6)
    assert bn.num_batches_tracked.item() == 1
    r = torch.randn(rows, C, device="cuda", generator=g).to(dtype)
    r4 = r.view(1, rows, 1, C).permute(0, 3, 1, 2)
    for res, rst in ((None, None), (r4, None), (r4, st)):
        y = x4.clone(memory_format=torch.channels_last)
        _bn_apply_(y, st, residual=res, rst=rst)
        ref = xd * st[0].double() + st[1].double()
        if res is not None:
            ref = ref + (r.double() * st[0].double() + st[1].double() if rst is not None else r.double())
        ref = ref.clamp_min(0)
        got = y.permute(0, 2, 3, 1).reshape(rows, C).double()
        tol = 1e-5 if dtype == torch.float32 else 1e-2
        torch.testing.assert_close(got, ref, rtol=tol, atol=tol)


@pytest.mark.gpu
def test_c5_train_mode_bn_4096_tiles(monkeypatch):
    """Config C5's encoder in train mode at its own size (4096 tiles, fp32; the reference's frozen
    encoder under Lightning's model.train(), code/models/model_interface.py:237-247,303-309): the
    bag runs in 8 pieces of 512 tiles (every library tensor < 2^31 elements) while every BatchNorm
    normalises with the whole bag's statistics.
      * each BatchNorm's scale / shift and running mean / variance against an fp64 restatement of
        the batch statistics of that BatchNorm's actual input (all 4096 tiles, computed here from
        the pieces in fp64): scale = gamma / sqrt(var + eps), shift = beta - mean * scale, running
        statistics with momentum 0.1 and the unbiased variance;
      * the features of 4 tiles spread over the bag against the fp64 oracle forward of those tiles
        normalised with the same whole-bag statistics (oracle/encoder_ref.py, stats_in)."""
    import torch.nn as nn
    from oracle.encoder_ref import BN_EPS, features
    from transmil_deepgraft_amd import encoder as E
    torch.backends.cudnn.allow_tf32 = False
    enc = _encoder(torch.float32)
    sd0 = {k: v.clone() for k, v in enc.state_dict().items()}
    enc = enc.cuda().train()
    assert E.train_pieces(C5_TILES, enc.chunk, elem_bytes=4) == 512
    names = {id(m): n for n, m in enc.named_modules() if isinstance(m, nn.BatchNorm2d)}
    rec = {}
    orig = E._bn_train_stats

    def spy(ys, bn, ws):
        assert all(y.numel() * y.element_size() <= E.LIB_MAX_BYTES for y in ys)
        C = ys[0].shape[1]
        n = sum(y.numel() // C for y in ys)
        mean = sum(y.double().sum(dim=(0, 2, 3)) for y in ys) / n
        var = sum(((y.double() - mean.view(1, C, 1, 1)) ** 2).sum(dim=(0, 2, 3)) for y in ys) / n
        rm0, rv0 = bn.running_mean.double().clone(), bn.running_var.double().clone()
        st = orig(ys, bn, ws)
        rec[names[id(bn)]] = dict(mean=mean, var=var, st=st.double().clone(), rm0=rm0, rv0=rv0,
                                  rm1=bn.running_mean.double().clone(), rv1=bn.running_var.double().clone(), n=n,
                                  g=bn.weight.double(), b=bn.bias.double())
        return st

    monkeypatch.setattr(E, "_bn_train_stats", spy)
    g = torch.Generator(device="cuda").manual_seed(5)
    tiles = torch.randn(C5_TILES, 3, 224, 224, device="cuda", generator=g)
    with torch.no_grad():
        feats = enc(tiles)
    torch.cuda.synchronize()
    assert len(rec) == 53 and torch.isfinite(feats).all()
    worst = {}
    for name, r in rec.items():
        assert r["n"] > 1 and r["n"] % C5_TILES == 0
        scale = r["g"] / torch.sqrt(r["var"] + BN_EPS)
        shift = r["b"] - r["mean"] * scale
        rm = 0.9 * r["rm0"] + 0.1 * r["mean"]
        rv = 0.9 * r["rv0"] + 0.1 * r["var"] * r["n"] / (r["n"] - 1)
        errs = [((r["st"][0] - scale).abs().max() / scale.abs().max()).item(),
                ((r["st"][1] - shift).abs().max() / shift.abs().max().clamp_min(1e-6)).item(),
                ((r["rm1"] - rm).abs().max() / rm.abs().max().clamp_min(1e-6)).item(),
                ((r["rv1"] - rv).abs().max() / rv.abs().max()).item()]
        worst[name] = max(errs)
    bad = {k: v for k, v in worst.items() if v > 1e-4}
    assert not bad, bad
    idx = torch.tensor([0, 1365, 2731, 4095])
    stats = {name: (r["mean"], r["var"]) for name, r in rec.items()}
    ref = features(tiles[idx.cuda()].cpu(), sd0, train=True, stats_in=stats)
    got = feats[idx.cuda()].double().cpu()
    err = ((got - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    assert err < 2e-3, err


@pytest.mark.gpu
@pytest.mark.parametrize("n,h", [(3, 112), (2, 15)])
def test_stem_bias_relu_maxpool_equals_bias_act_then_pool(n, h):
    """tm_bias_relu_maxpool against tm_bias_act + max_pool2d (the two-pass eval stem tail),
    channels-last bf16, odd and even sizes: bitwise."""
    import torch.nn.functional as F
    from transmil_deepgraft_amd import encoder as E
    g = torch.Generator(device="cpu").manual_seed(n * 100 + h)
    y = (torch.randn(n, 64, h, h + 1, generator=g) * 2).to(torch.bfloat16).to("cuda")
    y = y.contiguous(memory_format=torch.channels_last)
    b = torch.randn(64, generator=g).to(torch.bfloat16).to("cuda")
    ref = F.max_pool2d(E._bias_act_(y.clone(), b), 3, 2, 1)
    out = E._stem_pool_(y, b)
    torch.cuda.synchronize()
    assert out.shape == ref.shape and out.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(out, ref)


@pytest.mark.gpu
def test_stem_bn_relu_maxpool_equals_bn_apply_then_pool():
    """tm_bn_relu_maxpool (train-mode stem: batch-statistics BN, some negative scales) against
    tm_bn_apply + max_pool2d: bitwise."""
    import torch.nn.functional as F
    from transmil_deepgraft_amd import encoder as E
    g = torch.Generator(device="cpu").manual_seed(5)
    y = (torch.randn(2, 64, 30, 29, generator=g) * 2).to(torch.bfloat16).to("cuda")
    y = y.contiguous(memory_format=torch.channels_last)
    scale = torch.randn(64, generator=g).to("cuda")
    shift = torch.randn(64, generator=g).to("cuda")
    ref = F.max_pool2d(E._bn_apply_(y.clone(), (scale, shift)), 3, 2, 1)
    out = E._stem_pool_bn_(y, (scale, shift))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(2, 224, 224), (3, 61, 47), (1, 9, 16)])
def test_stem_conv_pool_against_torch_fp32(n, h, w):
    """tm_stem_conv_pool (the whole eval stem in one pass: conv 7x7/2 + folded bias + ReLU +
    max-pool 3x3/2) against the fp32 torch ops on the same bf16 inputs, within one bf16 rounding of
    the output; NCHW and channels-last inputs give the same bits; ragged sizes cover the partial
    8 x 8 pooled blocks and the padding at every edge."""
    import torch.nn.functional as F
    from transmil_deepgraft_amd import encoder as E
    g = torch.Generator(device="cpu").manual_seed(n * 1000 + h + w)
    x = torch.randn(n, 3, h, w, generator=g).to(torch.bfloat16).to("cuda")
    wt = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(torch.bfloat16).to("cuda")
    b = (torch.randn(64, generator=g) * 0.1).to(torch.bfloat16).to("cuda")
    ref = F.max_pool2d(F.relu(F.conv2d(x.float(), wt.float(), b.float(), stride=2, padding=3)), 3, 2, 1)
    wp = E._pack_stem(wt)
    out = E._stem_conv_pool(x, wp, b)
    out_cl = E._stem_conv_pool(x.contiguous(memory_format=torch.channels_last), wp, b)
    torch.cuda.synchronize()
    assert out.shape == ref.shape and out.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(out, out_cl)
    err = (out.float() - ref).abs()
    assert (err <= ref.abs() * 2 ** -8 + 1e-5).all(), err.max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(5, 64, 72), (2, 224, 224), (3, 33, 17)])
def test_stem_train_bn_passes_against_torch(n, h, w):
    """Train-mode stem (tm_stem_bn_stats + tm_stem_conv_pool_bn, the conv recomputed instead of
    stored): batch statistics of the bf16-rounded conv output against fp64 torch over every pixel of
    every tile (scale / shift / running statistics), and the pooled output against the fp32 torch
    ops with those statistics."""
    import torch.nn as nn
    import torch.nn.functional as F
    from transmil_deepgraft_amd import encoder as E
    g = torch.Generator(device="cpu").manual_seed(n * 7 + h + w)
    x = torch.randn(n, 3, h, w, generator=g).to(torch.bfloat16).to("cuda")
    wt = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(torch.bfloat16).to("cuda")
    bn = nn.BatchNorm2d(64, momentum=0.1).cuda()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(64, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(64, generator=g) * 0.1)
        bn.running_mean.copy_(torch.randn(64, generator=g) * 0.1)
    rm0, rv0 = bn.running_mean.clone().double(), bn.running_var.clone().double()
    wp = E._pack_stem(wt)
    st = E._stem_bn_stats(x, wp, bn)
    out = E._stem_conv_pool_bn(x, wp, st)
    torch.cuda.synchronize()
    conv = F.conv2d(x.double(), wt.double(), stride=2, padding=3).to(torch.bfloat16).double()
    mean = conv.mean(dim=(0, 2, 3))
    var = conv.var(dim=(0, 2, 3), unbiased=False)
    cnt = conv.numel() // 64
    sc = bn.weight.double() / torch.sqrt(var + bn.eps)
    sf = bn.bias.double() - mean * sc
    torch.testing.assert_close(st[0].double(), sc, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(st[1].double(), sf, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn.running_mean.double(), 0.9 * rm0 + 0.1 * mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var.double(), 0.9 * rv0 + 0.1 * var * cnt / (cnt - 1), rtol=1e-5,
                               atol=1e-6)
    ref = F.max_pool2d(F.relu(conv.float() * st[0].view(1, 64, 1, 1) + st[1].view(1, 64, 1, 1)), 3, 2, 1)
    assert out.shape == ref.shape and out.is_contiguous(memory_format=torch.channels_last)
    err = (out.float() - ref).abs()
    # one bf16 rounding of the output, plus a one-ulp tie flip of bf16(conv) where the summation
    # order differs (scaled by |scale|)
    tol = ref.abs() * 2 ** -8 + st[0].abs().view(1, 64, 1, 1) * conv.float().abs().amax() * 2 ** -8 + 1e-5
    assert (err <= tol).all(), err.max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_subsample_equals_strided_copy(dtype):
    """tm_subsample2d (the stride-2 downsample input) against x[:, :, ::2, ::2]: bitwise, odd size."""
    from transmil_deepgraft_amd import encoder as E
    x = torch.randn(3, 64, 15, 14, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    out = E._subsample(x, 2)
    torch.cuda.synchronize()
    assert out.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(out, x[:, :, ::2, ::2])
