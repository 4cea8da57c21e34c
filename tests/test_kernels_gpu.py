"""Kernel-level numerics on the MI355X, each HIP entry point against a plain
PyTorch fp64 reference of the same op (through the C ABI)."""
import ctypes as C
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lib():
    from transmil_deepgraft_amd import _lib
    return _lib


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


# ----------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("a_trans,b_kn", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("K", [168, 320])
def test_gemm_layouts(dtype, a_trans, b_kn, K):
    """K = 168: register-staged loop; K = 320 (bf16): the global_load_lds ring."""
    from transmil_deepgraft_amd.engine import gemm
    from transmil_deepgraft_amd._lib import BF16, F32
    code = BF16 if dtype == torch.bfloat16 else F32
    M, N = 296, 264   # not tile multiples, but 16-B rows when stored transposed
    g = torch.Generator(device="cpu").manual_seed(1)
    A = torch.randn(M, K, generator=g).to(dtype)
    B = torch.randn(K, N, generator=g).to(dtype)
    ref = A.double() @ B.double()
    As = (A.t().contiguous() if a_trans else A).to(DEV)
    Bs = (B.contiguous() if b_kn else B.t().contiguous()).to(DEV)
    out = torch.empty(M, N, dtype=torch.float32, device=DEV)
    gemm(As, Bs, out, M, N, K, lda=M if a_trans else K, ldb=N if b_kn else K, ldc=N, a_trans=a_trans,
         b_kn=b_kn, dtype=code, c_dtype=F32)
    torch.cuda.synchronize()
    assert _rel(out.cpu(), ref) < 1e-5


@pytest.mark.parametrize("a_trans,b_kn", [(0, 0), (0, 1), (1, 1)])
def test_gemm_persistent_many_tiles(a_trans, b_kn):
    """More tiles than workgroups (every workgroup walks several tiles, the DMA ring runs across
    tile boundaries) in the QKV / dX layouts and the split-K weight gradient (6 splits x 48 tiles)."""
    from transmil_deepgraft_amd.engine import gemm, weight_grad, Pool
    from transmil_deepgraft_amd._lib import BF16, F32
    g = torch.Generator(device="cpu").manual_seed(3)
    if a_trans:     # dW[M, N] = sum_k dY[k, m] X[k, n]
        M, N, K = 1536, 512, 4224
        dY = torch.randn(K, M, generator=g).to(torch.bfloat16)
        X = torch.randn(K, N, generator=g).to(torch.bfloat16)
        ref = dY.double().t() @ X.double()
        out = torch.empty(M, N, device=DEV)
        weight_grad(dY.to(DEV), X.to(DEV), out, M, N, K, ldy=M, ldx=N, dtype=BF16, work_pool=Pool(DEV),
                    slab_bf16=False)
    else:
        M, N, K = 4136, 1536, 512
        A = torch.randn(M, K, generator=g).to(torch.bfloat16)
        B = torch.randn(K, N, generator=g).to(torch.bfloat16)
        ref = A.double() @ B.double()
        Bs = (B.contiguous() if b_kn else B.t().contiguous()).to(DEV)
        out = torch.empty(M, N, dtype=torch.float32, device=DEV)
        gemm(A.to(DEV), Bs, out, M, N, K, lda=K, ldb=N if b_kn else K, ldc=N, b_kn=b_kn, dtype=BF16, c_dtype=F32)
    torch.cuda.synchronize()
    assert _rel(out.cpu(), ref) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogue_bias_gelu_rowmap_dup(dtype):
    from transmil_deepgraft_amd.engine import gemm
    from transmil_deepgraft_amd._lib import BF16, F32
    code = BF16 if dtype == torch.bfloat16 else F32
    Bg, Nn, F, D = 2, 37, 64, 128
    G = 7
    add, S = G * G - Nn, G * G + 1
    g = torch.Generator().manual_seed(2)
    x = torch.randn(Bg * Nn, F, generator=g).to(dtype)
    w = torch.randn(D, F, generator=g).to(dtype) * 0.2
    b = torch.randn(D, generator=g)
    pre_ref = x.double() @ w.double().t() + b.double()
    y_ref = torch.nn.functional.gelu(pre_ref)
    H = torch.full((Bg * S, D), 7.0, device=DEV)
    pre = torch.empty(Bg * Nn, D, device=DEV)
    gemm(x.to(DEV), w.to(DEV), H, Bg * Nn, D, F, lda=F, ldb=F, ldc=D, dtype=code, c_dtype=F32, bias=b.to(DEV),
         gelu=True, pre=pre, ld_pre=D, rowmap=(Nn, 0, S, 1, add, 1 + Nn))
    torch.cuda.synchronize()
    Hc = H.cpu().view(Bg, S, D)
    yr = y_ref.view(Bg, Nn, D)
    assert (Hc[:, 0] == 7.0).all()
    assert _rel(Hc[:, 1:1 + Nn], yr) < 1e-5
    assert _rel(Hc[:, 1 + Nn:], yr[:, :add]) < 1e-5
    assert _rel(pre.cpu(), pre_ref) < 1e-5


def test_gemm_dropout_residual_and_splitk():
    from transmil_deepgraft_amd.engine import gemm, weight_grad, Pool
    from transmil_deepgraft_amd._lib import F32
    M, N, K = 512, 256, 128
    g = torch.Generator().manual_seed(3)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g)
    R = torch.randn(M, N, generator=g)
    out = torch.empty(M, N, device=DEV)
    gemm(A.to(DEV), W.to(DEV), out, M, N, K, lda=K, ldb=K, ldc=N, dtype=F32, c_dtype=F32, drop_p=0.7, seed=123,
         resid=R.to(DEV))
    torch.cuda.synchronize()
    o = out.cpu() - R
    full = (A.double() @ W.double().t()) / 0.3
    kept = o.abs() > 0
    frac = kept.double().mean().item()
    assert abs(frac - 0.3) < 0.02
    assert _rel(o[kept], full[kept]) < 1e-5
    # split-K weight gradient: out[m,n] = sum_k dY[k,m] X[k,n]
    dY = torch.randn(4000, 96, generator=g)
    X = torch.randn(4000, 160, generator=g)
    res = torch.empty(96, 160, device=DEV)
    weight_grad(dY.to(DEV), X.to(DEV), res, 96, 160, 4000, ldy=96, ldx=160, dtype=F32, work_pool=Pool(DEV))
    torch.cuda.synchronize()
    assert _rel(res.cpu(), dY.double().t() @ X.double()) < 1e-5


@pytest.mark.parametrize("slab_bf16", [False, True])
@pytest.mark.parametrize("M,N,K", [(192, 136, 33 * 256), (512, 512, 8448), (520, 512, 8192), (1536, 512, 8448)])
def test_gemm_ring_splitk_weight_grad_bf16(M, N, K, slab_bf16):
    """bf16 split-K weight gradient through the global_load_lds ring, with the bias gradient
    (column sums of dY) summed by the same launch (tm_gemm_args.colsum); M = 520: a ragged last
    column tile of the A image (clamped chunks must not leak into the sums).  fp32 slabs: within
    1e-5 of fp64; bf16 slabs (the bf16 step's form): each split's partial rounded once to bf16, half
    an ulp = 2^-9 of a partial whose size approaches the result's (5-16 partials of random-sign
    sums), so within 5e-3 of the result's max (2.2e-3 measured at 1536 x 512, K = 8448)."""
    from transmil_deepgraft_amd.engine import weight_grad, Pool, flush_reductions
    from transmil_deepgraft_amd._lib import BF16
    g = torch.Generator().manual_seed(5)
    dY = torch.randn(K, M, generator=g).bfloat16()
    X = torch.randn(K, N, generator=g).bfloat16()
    res = torch.empty(M, N, device=DEV)
    bias = torch.full((M,), float("nan"), device=DEV)
    weight_grad(dY.to(DEV), X.to(DEV), res, M, N, K, ldy=M, ldx=N, dtype=BF16, work_pool=Pool(DEV), bias_out=bias,
                slab_bf16=slab_bf16)
    flush_reductions()
    torch.cuda.synchronize()
    assert _rel(res.cpu(), dY.double().t() @ X.double()) < (5e-3 if slab_bf16 else 1e-5)
    assert _rel(bias.cpu(), dY.double().sum(0)) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_qkv_scatter(dtype):
    from transmil_deepgraft_amd.engine import gemm
    from transmil_deepgraft_amd._lib import BF16, F32
    code = BF16 if dtype == torch.bfloat16 else F32
    Bg, n, D, nh = 2, 256, 512, 8
    g = torch.Generator().manual_seed(4)
    x = torch.randn(Bg * n, D, generator=g).to(dtype)
    w = (torch.randn(3 * D, D, generator=g) * 0.05).to(dtype)
    out = torch.empty(3, Bg * nh, n, 64, dtype=dtype, device=DEV)
    gemm(x.to(DEV), w.to(DEV), out, Bg * n, 3 * D, D, lda=D, ldb=D, ldc=0, dtype=code, qkv=(Bg, nh, 64, n, 0.125))
    torch.cuda.synchronize()
    ref = (x.double() @ w.double().t()).view(Bg, n, 3, nh, 64).permute(2, 0, 3, 1, 4).reshape(3, Bg * nh, n, 64)
    ref[0] *= 0.125
    tol = 1e-5 if dtype == torch.float32 else 8e-3
    assert _rel(out.cpu(), ref) < tol


@pytest.mark.parametrize("Bg,n", [(1, 8448), (2, 2304)])
def test_gemm_qkv_scatter_big_tile(Bg, n):
    """to_qkv at the step's sizes takes the 256 x 256 big-tile kernel (M >= 2048, N = 1536): the
    head-major scatter + q scale against fp64, every output element written (two 128-row epilogue
    passes per tile; n = 8448: 33 row tiles, the last one full; 2 x 2304: tiles straddle bags)."""
    from transmil_deepgraft_amd.engine import gemm
    from transmil_deepgraft_amd._lib import BF16
    D, nh = 512, 8
    g = torch.Generator().manual_seed(14)
    x = (torch.randn(Bg * n, D, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(3 * D, D, generator=g) * 0.05).to(torch.bfloat16)
    out = torch.full((3, Bg * nh, n, 64), float("nan"), dtype=torch.bfloat16, device=DEV)
    gemm(x.to(DEV), w.to(DEV), out, Bg * n, 3 * D, D, lda=D, ldb=D, ldc=0, dtype=BF16, qkv=(Bg, nh, 64, n, 0.125))
    torch.cuda.synchronize()
    ref = (x.double() @ w.double().t()).view(Bg, n, 3, nh, 64).permute(2, 0, 3, 1, 4).reshape(3, Bg * nh, n, 64)
    ref[0] *= 0.125
    got = out.cpu()
    assert torch.isfinite(got).all()
    assert _rel(got, ref) < 8e-3


@pytest.mark.parametrize("N,K,b_kn,mode", [(512, 1536, 1, "plain"), (512, 512, 1, "plain"),
                                          (512, 512, 0, "to_out"), (1536, 512, 0, "qkv")])
def test_gemm_160_row_tiles_at_bench_rows(N, K, b_kn, mode):
    """The step's bf16 GEMMs at M = n' = 8448 rows (33 x 256), which run on 160-row tiles (53 row
    tiles: 212 / 636 tiles instead of 264 / 792): dxn / dmerged (B [K, N]), to_out (bias, dropout,
    residual, the front-pad row map), QKV (head-major scatter, q x 1/8) against fp64."""
    from transmil_deepgraft_amd.engine import gemm
    from transmil_deepgraft_amd._lib import BF16, F32
    M = 8448
    g = torch.Generator().manual_seed(N + K + b_kn)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(K, N, generator=g) if b_kn else torch.randn(N, K, generator=g)) * 0.05
    W = W.to(torch.bfloat16)
    Wt = W.double() if b_kn else W.double().t()
    full = A.double() @ Wt
    if mode == "plain":
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        gemm(A.to(DEV), W.to(DEV), out, M, N, K, lda=K, ldb=N if b_kn else K, ldc=N, b_kn=b_kn, dtype=BF16)
        torch.cuda.synchronize()
        assert _rel(out.cpu(), full) < 8e-3
    elif mode == "to_out":
        # rows of the padded layout [n' = 8448] -> residual rows (pad 166 dropped): S = 8282
        pad, S = 166, 8282
        bias = torch.randn(N, generator=g)
        R = torch.randn(S, N, generator=g)
        out = torch.full((S, N), float("nan"), device=DEV)
        gemm(A.to(DEV), W.to(DEV), out, M, N, K, lda=K, ldb=K, ldc=N, dtype=BF16, c_dtype=F32, bias=bias.to(DEV),
             drop_p=0.7, seed=99, resid=R.to(DEV), rowmap=(M, pad, S, 0, 0, 0))
        torch.cuda.synchronize()
        o = out.cpu().double() - R.double()
        ref = (full[pad:] + bias.double()) / 0.3
        kept = o.abs() > 0
        assert abs(kept.double().mean().item() - 0.3) < 0.01
        assert _rel(o[kept], ref[kept]) < 8e-3
    else:
        Bg, nh = 1, 8
        out = torch.empty(3, nh, M, 64, dtype=torch.bfloat16, device=DEV)
        gemm(A.to(DEV), W.to(DEV), out, M, N, K, lda=K, ldb=K, ldc=0, dtype=BF16, qkv=(Bg, nh, 64, M, 0.125))
        torch.cuda.synchronize()
        ref = full.view(M, 3, nh, 64).permute(1, 2, 0, 3).clone()
        ref[0] *= 0.125
        assert _rel(out.cpu(), ref) < 8e-3


# ----------------------------------------------------------------------------- LayerNorm
def test_layernorm_fwd_bwd():
    from transmil_deepgraft_amd import ops
    ln = torch.nn.LayerNorm(512).to(DEV)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    x = torch.randn(3, 77, 512, device=DEV, requires_grad=True)
    y = ops.layer_norm(ln, x)
    gy = torch.randn_like(y)
    y.backward(gy)
    x2 = x.detach().double().requires_grad_()
    w2 = ln.weight.detach().double().requires_grad_()
    b2 = ln.bias.detach().double().requires_grad_()
    y2 = torch.nn.functional.layer_norm(x2, (512,), w2, b2, 1e-5)
    y2.backward(gy.double())
    assert _rel(y, y2) < 1e-5
    assert _rel(x.grad, x2.grad) < 1e-4
    assert _rel(ln.weight.grad, w2.grad) < 1e-4
    assert _rel(ln.bias.grad, b2.grad) < 1e-4


# ----------------------------------------------------------------------------- PPEG
@pytest.mark.parametrize("G,D,B", [(1, 64, 2), (5, 64, 2), (32, 64, 2), (13, 128, 3), (91, 512, 1)])
def test_ppeg_fwd_bwd(G, D, B):
    """The persistent PPEG walker (tile teams per 64-channel chunk, fused weight gradient) against the
    fp64 oracle PPEG (code/models/TransMIL.py:60-75); G = 91, D = 512 is the bench shape."""
    from oracle.transmil_ref import PPEG as RefPPEG
    from transmil_deepgraft_amd.models.TransMIL import PPEG
    torch.manual_seed(G)
    ref = RefPPEG(D).double()
    ours = PPEG(D).to(DEV)
    ours.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    x = torch.randn(B, 1 + G * G, D, dtype=torch.float64)
    y_ref = ref(x.clone().requires_grad_(), G, G)
    xr = x.clone().requires_grad_()
    y_ref = ref(xr, G, G)
    gy = torch.randn_like(y_ref)
    y_ref.backward(gy)
    xo = x.float().to(DEV).requires_grad_()
    y = ours(xo, G, G)
    y.backward(gy.float().to(DEV))
    assert _rel(y.cpu(), y_ref) < 1e-5
    assert _rel(xo.grad.cpu(), xr.grad) < 1e-5
    for (n1, p1), (n2, p2) in zip(ours.named_parameters(), ref.named_parameters()):
        assert _rel(p1.grad.cpu(), p2.grad) < 1e-4, n1


# ----------------------------------------------------------------------------- bmm
@pytest.mark.parametrize("prec,tol", [(0, 2e-6), (1, 3e-5)])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("K", [64, 256])
def test_bmm_batched_epilogue(prec, tol, ta, tb, K):
    """C = alpha*op(A) op(B) + diag*I + e1*E1 + e2*E2, fp32 in/out; prec 1 = bf16x3 split."""
    from transmil_deepgraft_amd.engine import bmm, bmm_job
    nb, M, N = 3, 256, 64 if K == 256 else 256
    g = torch.Generator().manual_seed(K + 4 * ta + 2 * tb + prec)
    A = torch.randn(nb, M, K, generator=g, dtype=torch.float64)
    B = torch.randn(nb, K, N, generator=g, dtype=torch.float64)
    E1 = torch.randn(nb, M, N, generator=g, dtype=torch.float64)
    E2 = torch.randn(nb, M, N, generator=g, dtype=torch.float64)
    ref = 0.7 * A @ B + 0.5 * E1 - 2.0 * E2
    ref += 3.0 * torch.eye(M, N, dtype=torch.float64)
    Ad = (A.transpose(1, 2) if ta else A).contiguous().float().to(DEV)
    Bd = (B.transpose(1, 2) if tb else B).contiguous().float().to(DEV)
    out = torch.empty(nb, M, N, device=DEV)
    bmm([bmm_job(Ad, ta, Bd, tb, out, M, N, K, alpha=0.7, diag=3.0, E1=E1.float().to(DEV), e1=0.5,
                 E2=E2.float().to(DEV), e2=-2.0)], nb, prec)
    torch.cuda.synchronize()
    assert _rel(out.cpu(), ref) < tol


# ----------------------------------------------------------------------------- pinv
def test_pinv_bf16x3_close_to_exact():
    """The bench mode's bf16x3 products keep the 6 Newton-Schulz steps within 1e-4."""
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd.engine import _p, _stream
    nbh = 8
    g = torch.Generator().manual_seed(8)
    X = torch.softmax(torch.randn(nbh, 256, 256, generator=g) * 0.3, dim=-1).to(DEV)
    zs = []
    for prec in (0, 1):
        saved = torch.empty(_lib.query("tm_pinv_saved_floats", nbh, 6), device=DEV)
        _lib.call("tm_pinv_fwd", _p(X), nbh, 6, prec, _p(saved), _stream())
        zs.append(saved[6 * nbh * 65536:7 * nbh * 65536].clone())
    torch.cuda.synchronize()
    assert _rel(zs[1].cpu(), zs[0].cpu()) < 1e-4


def test_pinv_fwd_bwd_fp32_exact_path():
    """Z = pinv(softmax(s)); compare Z and dL/ds.  dL/dA2 itself is not compared: the
    max(rowsum) term of Z0's scale adds a row-constant gradient that torch gives to
    one arg-max row but that fp32 rounding spreads over exact ties; the softmax
    backward annihilates row constants, so dL/ds is tie-independent."""
    from oracle.nystrom_ref import moore_penrose_iter_pinv
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd.engine import _p, _stream
    nbh = 8
    g = torch.Generator().manual_seed(7)
    s64 = (torch.randn(nbh, 256, 256, generator=g, dtype=torch.float64) * 0.3).requires_grad_()
    a64 = torch.softmax(s64, dim=-1)
    a = a64.detach()
    z_ref = moore_penrose_iter_pinv(a64, 6)
    gz = torch.randn(nbh, 256, 256, generator=g, dtype=torch.float64) * 1e-3
    z_ref.backward(gz)
    X = a.float().to(DEV)
    saved = torch.empty(_lib.query("tm_pinv_saved_floats", nbh, 6), device=DEV)
    _lib.call("tm_pinv_fwd", _p(X), nbh, 6, 0, _p(saved), _stream())
    z = saved[6 * nbh * 65536:7 * nbh * 65536].view(nbh, 256, 256)
    dz = gz.float().to(DEV).contiguous()
    work = torch.empty(_lib.query("tm_pinv_bwd_workspace_floats", nbh), device=DEV)
    dX = torch.empty(nbh, 256, 256, device=DEV)
    _lib.call("tm_pinv_bwd", _p(X), nbh, 6, 0, _p(saved), _p(dz), _p(work), _p(dX), _stream())
    ds = torch.empty_like(dX)
    _lib.call("tm_softmax_bwd_rows256", _p(X), _p(dX), _p(ds), nbh * 256, _stream())
    torch.cuda.synchronize()
    assert _rel(z.cpu(), z_ref.detach()) < 2e-4
    assert _rel(ds.cpu(), s64.grad) < 2e-3


@pytest.mark.parametrize("nbh", [2, 12, 32])
@pytest.mark.parametrize("prec", [0, 1])
def test_pinv_odd_head_counts(nbh, prec):
    """nbh = 2 / 12 / 32 (B*heads other than 8): Z_6 and dL/ds against fp64 autograd through the
    restatement; B*heads is the bmm batch, and blockIdx % nbatch picks the head."""
    from oracle.nystrom_ref import moore_penrose_iter_pinv
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd.engine import _p, _stream
    g = torch.Generator().manual_seed(11 + nbh)
    s64 = (torch.randn(nbh, 256, 256, generator=g, dtype=torch.float64) * 0.3).requires_grad_()
    a64 = torch.softmax(s64, dim=-1)
    z_ref = moore_penrose_iter_pinv(a64, 6)
    gz = torch.randn(nbh, 256, 256, generator=g, dtype=torch.float64) * 1e-3
    z_ref.backward(gz)
    X = a64.detach().float().to(DEV).contiguous()
    saved = torch.full((_lib.query("tm_pinv_saved_floats", nbh, 6),), float("nan"), device=DEV)
    _lib.call("tm_pinv_fwd", _p(X), nbh, 6, prec, _p(saved), _stream())
    z = saved[6 * nbh * 65536:7 * nbh * 65536].view(nbh, 256, 256)
    work = torch.full((_lib.query("tm_pinv_bwd_workspace_floats", nbh),), float("nan"), device=DEV)
    dz = gz.float().to(DEV).contiguous()
    dX = torch.full((nbh, 256, 256), float("nan"), device=DEV)
    _lib.call("tm_pinv_bwd", _p(X), nbh, 6, prec, _p(saved), _p(dz), _p(work), _p(dX), _stream())
    ds = torch.empty_like(dX)
    _lib.call("tm_softmax_bwd_rows256", _p(X), _p(dX), _p(ds), nbh * 256, _stream())
    torch.cuda.synchronize()
    assert _rel(z.cpu(), z_ref.detach()) < (2e-4 if prec == 0 else 5e-4)
    assert _rel(ds.cpu(), s64.grad) < 4e-3



# ----------------------------------------------------------------------------- NystromAttention
@pytest.mark.parametrize("S", [2, 101, 257, 1025, 2000])
def test_nystrom_attention_fp32_vs_oracle(S):
    from oracle.nystrom_ref import NystromAttention as Ref
    from transmil_deepgraft_amd.nystrom_attention import NystromAttention
    torch.manual_seed(S)
    ref = Ref(dim=512, dim_head=64, heads=8, num_landmarks=256, pinv_iterations=6, residual=True).double().eval()
    with torch.no_grad():
        ref.res_conv.weight.mul_(3.0)
    ours = NystromAttention(dim=512, dim_head=64, heads=8, num_landmarks=256, pinv_iterations=6,
                            residual=True).to(DEV).eval()
    ours.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    ours.compute_dtype = torch.float32
    x = torch.randn(2, S, 512, dtype=torch.float64)
    xr = x.clone().requires_grad_()
    out_ref = ref(xr)
    gy = torch.randn_like(out_ref)
    out_ref.backward(gy)
    xo = x.float().to(DEV).requires_grad_()
    out = ours(xo)
    out.backward(gy.float().to(DEV))
    assert _rel(out.cpu(), out_ref) < 1e-4
    assert _rel(xo.grad.cpu(), xr.grad) < 1e-3
    for (n1, p1), (n2, p2) in zip(ours.named_parameters(), ref.named_parameters()):
        assert _rel(p1.grad.cpu(), p2.grad) < 1e-3, n1


def test_nystrom_attention_bf16_close():
    from oracle.nystrom_ref import NystromAttention as Ref
    from transmil_deepgraft_amd.nystrom_attention import NystromAttention
    torch.manual_seed(11)
    ref = Ref(dim=512).double().eval()
    ours = NystromAttention(dim=512).to(DEV).eval()
    ours.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    x = torch.randn(1, 1500, 512, dtype=torch.float64)
    with torch.no_grad():
        out_ref = ref(x)
        out = ours(x.float().to(DEV))
    assert _rel(out.cpu(), out_ref) < 3e-2


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 1e-2)])
def test_return_attn_matrix(dtype, tol):
    """The attention map of the same forward (its compute dtype's factors) against the oracle."""
    from oracle.nystrom_ref import NystromAttention as Ref
    from transmil_deepgraft_amd.nystrom_attention import NystromAttention
    torch.manual_seed(12)
    ref = Ref(dim=512).double().eval()
    ours = NystromAttention(dim=512).to(DEV).eval()
    ours.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    ours.compute_dtype = dtype
    x = torch.randn(1, 300, 512, dtype=torch.float64)
    with torch.no_grad():
        _, attn_ref = ref(x, return_attn=True)
        _, attn = ours(x.float().to(DEV), return_attn=True)
    assert attn.shape == attn_ref.shape
    assert _rel(attn.cpu(), attn_ref) < tol


# ----------------------------------------------------------------------------- A1 forward (bf16 kernels)
def _a1_ref(q, v, kl, y, wconv, nh):
    """fp64 restatement: merged[bag][t][head*64 + d] = softmax(q kl^T) y + conv33(v); lse."""
    nbh, n, dh = q.shape
    s = q.double() @ kl.double().transpose(1, 2)
    lse = torch.logsumexp(s, -1)
    o = torch.softmax(s, -1) @ y.double()
    vp = torch.nn.functional.pad(v.double(), (0, 0, 16, 16))
    w = wconv.double().view(-1, 33)
    for tau in range(33):
        o += w[torch.arange(nbh) % nh, tau].view(nbh, 1, 1) * vp[:, tau:tau + n]
    merged = o.view(nbh // nh, nh, n, dh).permute(0, 2, 1, 3).reshape(nbh // nh, n, nh * dh)
    return merged, lse


@pytest.mark.parametrize("nbh,n", [(8, 256), (8, 1280), (32, 512), (8, 8448), (8, 33280)])
def test_a1_fwd_bf16_kernels(nbh, n):
    """The per-CU chunk-walking bf16 A1 kernel (MFMA conv, LDS-DMA windows) against fp64."""
    L = _lib()
    from transmil_deepgraft_amd._lib import BF16
    from transmil_deepgraft_amd.engine import _p, _stream
    g = torch.Generator(device="cpu").manual_seed(n + nbh)
    nh = 8
    q = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16)
    v = torch.randn(nbh, n, 64, generator=g).to(torch.bfloat16)
    kl = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(torch.bfloat16)
    y = torch.randn(nbh, 256, 64, generator=g).to(torch.bfloat16)
    wconv = torch.randn(nh, 33, generator=g) * 0.1
    ref_m, ref_l = _a1_ref(q, v, kl, y, wconv, nh)
    merged = torch.full((nbh // nh, n, nh * 64), float("nan"), dtype=torch.bfloat16, device=DEV)
    lse = torch.full((nbh, n), float("nan"), device=DEV)
    qd, vd, kd, yd, wd = (t.to(DEV).contiguous() for t in (q, v, kl, y, wconv))
    L.call("tm_nys_a1_fwd", BF16, _p(qd), _p(vd), _p(kd), _p(yd), _p(wd), nbh, nh, n, _p(merged), _p(lse),
           _stream())
    torch.cuda.synchronize()
    assert torch.isfinite(merged.float()).all() and torch.isfinite(lse).all()
    assert _rel(merged.cpu(), ref_m) < 2e-2
    assert (lse.cpu().double() - ref_l).abs().max().item() < 1e-4


# ----------------------------------------------------------------------------- conv33 backward
def _conv_bwd_ref(dO, O, v, wconv, nh):
    """fp64: dv = conv33^T(dO), c_tau(t) = dO[t].v[t + tau - 16], D1 = dO.O - sum_tau w c_tau,
    dw[head][tau] = sum over bags and rows of c_tau."""
    nbags, n, _ = dO.shape
    nbh = nbags * nh
    g = dO.double().view(nbags, n, nh, 64).permute(0, 2, 1, 3).reshape(nbh, n, 64)
    o = O.double().view(nbags, n, nh, 64).permute(0, 2, 1, 3).reshape(nbh, n, 64)
    vv = v.double()
    w = wconv.double().view(nh, 33)[torch.arange(nbh) % nh]          # [nbh, 33]
    gp = torch.nn.functional.pad(g, (0, 0, 16, 16))
    vp = torch.nn.functional.pad(vv, (0, 0, 16, 16))
    dv = torch.zeros_like(vv)
    c = torch.zeros(nbh, n, 33, dtype=torch.float64)
    for tau in range(33):
        dv += w[:, tau].view(nbh, 1, 1) * gp[:, 32 - tau:32 - tau + n]
        c[:, :, tau] = (g * vp[:, tau:tau + n]).sum(-1)
    d1 = (g * o).sum(-1) - (c * w.view(nbh, 1, 33)).sum(-1)
    dw = c.sum(1).view(nbags, nh, 33).sum(0)
    return dv, d1, dw


@pytest.mark.gpu
@pytest.mark.parametrize("nbags,n", [(1, 100), (1, 8448), (2, 1000), (4, 300)])
def test_conv_bwd_bf16_mfma(nbags, n):
    """The MFMA conv33 backward (bf16 mode) against fp64; dv is written bf16 (the fused A3 backward
    reads it once), d1 and the weight gradient fp32."""
    L = _lib()
    from transmil_deepgraft_amd._lib import BF16
    from transmil_deepgraft_amd.engine import _p, _stream
    nh = 8
    nbh = nbags * nh
    g = torch.Generator(device="cpu").manual_seed(n * 7 + nbags)
    dO = (torch.randn(nbags, n, nh * 64, generator=g) * 0.5).to(torch.bfloat16)
    O = torch.randn(nbags, n, nh * 64, generator=g).to(torch.bfloat16)
    v = torch.randn(nbh, n, 64, generator=g).to(torch.bfloat16)
    wconv = torch.randn(nh, 33, generator=g) * 0.1
    ref_dv, ref_d1, ref_dw = _conv_bwd_ref(dO, O, v, wconv, nh)
    dv = torch.full((nbh, n, 64), float("nan"), device=DEV, dtype=torch.bfloat16)   # dv in the step's dtype
    d1 = torch.full((nbh, n), float("nan"), device=DEV)
    dw = torch.full((nh * 33,), float("nan"), device=DEV)
    work = torch.empty(L.query("tm_nys_conv_bwd_workspace", nbags, nh, n) // 4 + 16, device=DEV)
    dOd, Od, vd, wd = (t.to(DEV).contiguous() for t in (dO, O, v, wconv))
    L.call("tm_nys_conv_bwd", BF16, _p(dOd), _p(Od), _p(vd), _p(wd), nbh, nh, n, _p(dv), _p(d1), _p(work),
           _p(dw), None, _stream())
    torch.cuda.synchronize()
    assert torch.isfinite(dv).all() and torch.isfinite(d1).all() and torch.isfinite(dw).all()
    assert _rel(dv.cpu(), ref_dv) < 4e-3          # fp32 sums, one bf16 rounding (half an ulp: 2^-9)
    assert _rel(dv.cpu(), ref_dv.to(torch.bfloat16)) < 4e-3
    assert (d1.cpu().double() - ref_d1).abs().max().item() < 1e-3 * ref_d1.abs().max().item()
    assert _rel(dw.cpu().view(nh, 33), ref_dw) < 1e-5


# ----------------------------------------------------------------------------- A3 attention backward
def _a3_bwd_ref(ql, dw, k, v):
    """fp64: A = softmax(ql k^T) over the keys; dS = A (dw v^T - rowsum(dw o A v));
    dk = dS^T ql, dv = A^T dw, dql = dS k (the backward of W = A v, SURVEY App. A eq. 3/9)."""
    ql, dw, k, v = (t.double() for t in (ql, dw, k, v))
    s = ql @ k.transpose(1, 2)
    lse = torch.logsumexp(s, -1)
    a = torch.exp(s - lse[..., None])
    w = a @ v
    d = (dw * w).sum(-1)
    ds = a * (dw @ v.transpose(1, 2) - d[..., None])
    return lse, d, ds.transpose(1, 2) @ ql, a.transpose(1, 2) @ dw, ds @ k


@pytest.mark.parametrize("nbh,n", [(8, 256), (8, 1280), (8, 8448), (16, 8448), (8, 33280), (24, 2048)])
def test_a3_fwd_bf16(nbh, n):
    """W = softmax(q~ k^T) v and lse3 (SURVEY App. A eq. 5-8, the A3 factor): the bf16 kernel (all
    256 landmark queries per workgroup against an even share of the keys, online softmax across
    chunks, fixed-order combine of the partials) against fp64 on the same bf16-rounded operands."""
    L = _lib()
    from transmil_deepgraft_amd._lib import BF16
    from transmil_deepgraft_amd.engine import _p, _stream
    g = torch.Generator(device="cpu").manual_seed(n + 7 * nbh)
    ql = torch.randn(nbh, 256, 64, generator=g) * 0.4
    k = (torch.randn(nbh, n, 64, generator=g) * 0.4).to(torch.bfloat16)
    v = torch.randn(nbh, n, 64, generator=g).to(torch.bfloat16)
    s = ql.to(torch.bfloat16).double() @ k.double().transpose(1, 2)
    ref_lse = torch.logsumexp(s, -1)
    ref_w = torch.softmax(s, -1) @ v.double()
    w = torch.full((nbh, 256, 64), float("nan"), device=DEV)
    lse = torch.full((nbh, 256), float("nan"), device=DEV)
    work = torch.empty(L.query("tm_nys_a3_workspace", nbh, n) // 4 + 16, device=DEV)
    qd, kd, vd = ql.to(DEV).contiguous(), k.to(DEV).contiguous(), v.to(DEV).contiguous()
    L.call("tm_nys_a3_fwd", BF16, _p(qd), _p(kd), _p(vd), nbh, n, _p(work), _p(w), _p(lse), _stream())
    torch.cuda.synchronize()
    assert torch.isfinite(w).all() and torch.isfinite(lse).all()
    assert _rel(w.cpu(), ref_w) < 1e-2
    assert (lse.cpu().double() - ref_lse).abs().max().item() < 1e-3


@pytest.mark.parametrize("nbh,n", [(8, 256), (2, 1280), (8, 1280), (8, 8448), (16, 8448)])
def test_a3_bwd_bf16_even_split(nbh, n):
    """The bf16 A3 backward (key units split evenly over the workgroups of a head: the 9-wave
    form at 8 heads x 8448 keys, short workgroups elsewhere) against fp64."""
    L = _lib()
    from transmil_deepgraft_amd._lib import BF16
    from transmil_deepgraft_amd.engine import _p, _stream
    g = torch.Generator(device="cpu").manual_seed(n * 3 + nbh)
    ql = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(torch.bfloat16)
    dw = (torch.randn(nbh, 256, 64, generator=g) * 0.1).to(torch.bfloat16)
    k = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16)
    v = torch.randn(nbh, n, 64, generator=g).to(torch.bfloat16)
    lse, d, ref_dk, ref_dv, ref_dql = _a3_bwd_ref(ql, dw, k, v)
    dk = torch.full((nbh, n, 64), float("nan"), device=DEV)
    dv = torch.zeros(nbh, n, 64, device=DEV)           # accumulated into (+=)
    dql = torch.full((nbh, 256, 64), float("nan"), device=DEV)
    work = torch.empty(L.query("tm_nys_a3_bwd_workspace", nbh, n) // 4 + 16, device=DEV)
    qd, wd, kd, vd = (t.to(DEV).contiguous() for t in (ql, dw, k, v))
    # D as the [2][nbh][256] partials over the two 32-column halves (tm_bmm_job.Rd of dW = Z^T dY)
    wv = torch.softmax(ql.double() @ k.double().transpose(1, 2), -1) @ v.double()
    dparts = torch.stack([(dw.double() * wv)[..., :32].sum(-1), (dw.double() * wv)[..., 32:].sum(-1)])
    assert torch.allclose(dparts.sum(0), d)
    lsed, dd = lse.float().to(DEV).contiguous(), dparts.float().to(DEV).contiguous()
    L.call("tm_nys_a3_bwd", BF16, _p(qd), _p(wd), _p(kd), _p(vd), _p(lsed), _p(dd), nbh, 8, n,
           _p(dk), _p(dv), _p(work), _p(dql), 0, None, _stream())
    torch.cuda.synchronize()
    assert torch.isfinite(dk).all() and torch.isfinite(dv).all() and torch.isfinite(dql).all()
    assert _rel(dk.cpu(), ref_dk) < 2e-2
    assert _rel(dv.cpu(), ref_dv) < 2e-2
    assert _rel(dql.cpu(), ref_dql) < 2e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nbh,n", [(8, 256), (3, 1280), (8, 8448), (2, 33280)])
def test_landmarks_segment_means(dtype, nbh, n):
    """q~, k~ = means of l = n / 256 consecutive rows (App. A eq. 2) and their dtype copies."""
    L = _lib()
    from transmil_deepgraft_amd._lib import BF16, F32
    from transmil_deepgraft_amd.engine import _p, _stream
    g = torch.Generator(device="cpu").manual_seed(n + nbh)
    q = torch.randn(nbh, n, 64, generator=g).to(dtype)
    k = torch.randn(nbh, n, 64, generator=g).to(dtype)
    l = n // 256
    ref_q = q.double().view(nbh, 256, l, 64).mean(2)
    ref_k = k.double().view(nbh, 256, l, 64).mean(2)
    ql, kl = (torch.full((nbh, 256, 64), float("nan"), device=DEV) for _ in range(2))
    qt, kt = (torch.empty(nbh, 256, 64, dtype=dtype, device=DEV) for _ in range(2))
    qd, kd = q.to(DEV).contiguous(), k.to(DEV).contiguous()
    L.call("tm_nys_landmarks", BF16 if dtype == torch.bfloat16 else F32, _p(qd), _p(kd), nbh, n, _p(ql), _p(kl),
           _p(qt), _p(kt), _stream())
    torch.cuda.synchronize()
    assert (ql.cpu().double() - ref_q).abs().max().item() < 1e-5
    assert (kl.cpu().double() - ref_k).abs().max().item() < 1e-5
    assert torch.equal(qt.cpu(), ql.cpu().to(dtype)) and torch.equal(kt.cpu(), kl.cpu().to(dtype))


def test_bmm_rowdot_partials():
    """tm_bmm_job.Rd: per 32-column tile the partial row dots of C with Rw (D = rowsum(dW o W) of
    the A3 backward as 2 partials), beside C itself, in both precisions."""
    from transmil_deepgraft_amd import engine as E
    g = torch.Generator(device="cpu").manual_seed(5)
    nbh = 8
    z = torch.randn(nbh, 256, 256, generator=g).to(DEV) * 0.1
    dy = torch.randn(nbh, 256, 64, generator=g).to(DEV)
    w = torch.randn(nbh, 256, 64, generator=g).to(DEV)
    ref = z.double().transpose(1, 2) @ dy.double()
    for prec in (0, 1):
        dw = torch.empty(nbh, 256, 64, device=DEV)
        rd = torch.full((2, nbh, 256), float("nan"), device=DEV)
        dw_t = torch.empty(nbh, 256, 64, dtype=torch.bfloat16, device=DEV)
        j = E.bmm_job(z, 1, dy, 0, dw, 256, 64, 256, Ct=dw_t, ct_mode=1)
        j.Rd, j.Rw = rd.data_ptr(), w.data_ptr()
        E.bmm([j], nbh, prec)
        torch.cuda.synchronize()
        assert _rel(dw.cpu(), ref.cpu()) < (1e-6 if prec == 0 else 1e-5)
        assert torch.equal(dw_t, dw.to(torch.bfloat16))
        prod = dw.double() * w.double()
        exp = torch.stack([prod[..., :32].sum(-1), prod[..., 32:].sum(-1)])
        assert torch.allclose(rd.double(), exp, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("rows,cols,ld,acc", [(8448, 512, 512, 0), (1000, 1024, 1536, 1), (300, 520, 520, 0),
                                              (77, 512, 512, 1)])
def test_colsum_bf16_matches_fp64(rows, cols, ld, acc):
    """tm_colsum (the bias gradients' deterministic two-level column sum) against an fp64 sum of the
    same bf16 values, with and without accumulate, ragged row chunks and a row stride > cols."""
    from transmil_deepgraft_amd import _lib
    from transmil_deepgraft_amd._lib import BF16
    from transmil_deepgraft_amd.engine import _p, _stream
    g = torch.Generator().manual_seed(rows + cols)
    X = torch.randn(rows, ld, generator=g).to(torch.bfloat16).to("cuda")
    out = torch.randn(cols, generator=g).to("cuda")
    base = out.clone()
    work = torch.empty(_lib.query("tm_colsum_workspace", rows, cols, 64) // 4 + 4, device="cuda")
    _lib.call("tm_colsum", _p(X), BF16, rows, cols, ld, 64, _p(work), _p(out), acc, None, _stream())
    torch.cuda.synchronize()
    ref = X[:, :cols].double().sum(0).cpu() + (base.double().cpu() if acc else 0)
    assert torch.allclose(out.double().cpu(), ref, rtol=1e-5, atol=2e-3)   # fp32 sums of ~8 K terms of size ~1


# ----------------------------------------------------------------------------- _fc1 GELU backward
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,N", [(1, 8192), (2, 300)])
def test_fc1_gelu_bwd_against_fp64(dtype, B, N):
    """tm_fc1_gelu_bwd: dpre[b, i] = (dH[b, 1 + i] + [i < add] dH[b, 1 + N + i]) * GELU'(pre[b, i]) and
    dcls = sum_b dH[b, 0], against fp64 on the same (T-rounded) pre-activation: fp32 within 1e-6,
    the bf16 result (one rounding) within 4e-3 of the max."""
    from transmil_deepgraft_amd._lib import BF16, F32
    from transmil_deepgraft_amd.engine import _p, _stream
    L = _lib()
    D = 512
    G = math.ceil(math.sqrt(N))
    add, S = G * G - N, G * G + 1
    g = torch.Generator(device="cpu").manual_seed(N + B)
    dH = torch.randn(B, S, D, generator=g)
    pre = (torch.randn(B, N, D, generator=g) * 2.0).to(dtype)
    dpre = torch.full((B, N, D), float("nan"), dtype=dtype, device=DEV)
    dcls = torch.full((D,), float("nan"), device=DEV)
    dHd, pred = dH.to(DEV).contiguous(), pre.to(DEV).contiguous()
    L.call("tm_fc1_gelu_bwd", BF16 if dtype == torch.bfloat16 else F32, _p(dHd), _p(pred), B, N, S, add, D,
           _p(dpre), _p(dcls), _stream())
    torch.cuda.synchronize()
    x = pre.double()
    gd = 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)
    up = dH[:, 1:1 + N].double().clone()
    up[:, :add] += dH[:, 1 + N:1 + N + add].double()
    ref = up * gd
    assert _rel(dpre.cpu(), ref) < (1e-6 if dtype == torch.float32 else 4e-3)
    assert _rel(dcls.cpu(), dH[:, 0].double().sum(0)) < 1e-6


# ----------------------------------------------------------------------------- assemble_q_slab
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("dq_row", [-1, 300])
@pytest.mark.parametrize("B,n", [(2, 768), (1, 8448), (1, 33280)])   # l = 3, 33 (C2), 130 (C3)
def test_assemble_q_slab_reduces_the_a3_partials(dtype, dq_row, B, n):
    """tm_nys_assemble_q_slab: q part of dqkv = scale * (dq + (dql + sum_p slab[p])[t / l] / l)
    against fp64 (the slab's bf16 partials summed in fp32), the other two thirds of dqkv untouched
    (the fused A3 backward wrote them)."""
    from transmil_deepgraft_amd._lib import BF16, F32
    from transmil_deepgraft_amd.engine import _p, _stream
    lib = _lib()
    nh, slabs, scale = 8, 33, 0.125
    nbh, l = B * nh, n // 256
    g = torch.Generator(device=DEV).manual_seed(11)
    dq = torch.randn(nbh, n, 64, device=DEV, generator=g)
    dql = torch.randn(nbh, 256, 64, device=DEV, generator=g)
    slab = torch.randn(slabs, nbh, 256, 64, device=DEV, generator=g).to(torch.bfloat16)   # as the fused A3 backward leaves it
    dqkv = torch.full((B, n, 3 * nh * 64), 7.0, device=DEV).to(dtype)
    lib.call("tm_nys_assemble_q_slab", BF16 if dtype == torch.bfloat16 else F32, _p(dq), dq_row, _p(dql), _p(slab),
             slabs, B, nh, n, C.c_float(scale), _p(dqkv), _stream())
    torch.cuda.synchronize()
    dqd = dq.double()
    if dq_row >= 0:
        keep = torch.zeros_like(dqd)
        keep[:, dq_row] = dqd[:, dq_row]
        dqd = keep
    lm = (dql.double() + slab.double().sum(0)) / l                       # [nbh, 256, 64]
    ref = scale * (dqd + lm.repeat_interleave(l, dim=1))                  # [nbh, n, 64]
    ref = ref.view(B, nh, n, 64).permute(0, 2, 1, 3).reshape(B, n, nh * 64)
    got = dqkv[:, :, :nh * 64].double()
    tol = 1e-5 if dtype == torch.float32 else 8e-3
    assert _rel(got, ref) < tol
    assert (dqkv[:, :, nh * 64:] == 7).all()


# ----------------------------------------------------------------------------- class-row q operands
@pytest.mark.parametrize("B,n,nslabs", [(1, 8448, 32), (2, 1024, 5), (1, 256, 0), (1, 33024, 70)])
def test_cls_q_rows_against_torch(B, n, nslabs):
    """tm_cls_q_rows: Aq rows = (dql + sum of the slabs) / l per landmark, the class row's dq; Xs
    rows = the segment sums of the bf16 LayerNorm output, the class row; zero rows past 257."""
    L = _lib()
    from transmil_deepgraft_amd.engine import _p, _stream, QROWS
    nh, D, NL = 8, 512, 256
    nbh, l, r = B * nh, n // 256, n // 3
    g = torch.Generator(device="cpu").manual_seed(n + nslabs)
    dql = torch.randn(nbh, NL, 64, generator=g).to(DEV)
    slab = torch.randn(max(nslabs, 1), nbh, NL, 64, generator=g).to(torch.bfloat16).to(DEV)   # bf16 partials
    dq = torch.randn(nbh, n, 64, generator=g).to(DEV)
    xn = torch.randn(B, n, D, generator=g).to(torch.bfloat16).to(DEV)
    Aq = torch.full((B, QROWS, D), float("nan"), device=DEV)
    Xs = torch.full((B, QROWS, D), float("nan"), device=DEV)
    L.call("tm_cls_q_rows", _p(dql), _p(slab), nslabs, _p(dq), _p(xn), B, nh, n, r, _p(Aq), _p(Xs), _stream())
    torch.cuda.synchronize()
    tot = (dql.double() + slab[:nslabs].double().sum(0)) / l                     # [nbh][256][64]
    ea = torch.zeros(B, QROWS, D, dtype=torch.float64)
    ex = torch.zeros(B, QROWS, D, dtype=torch.float64)
    for b in range(B):
        ea[b, :NL] = tot[b * nh:(b + 1) * nh].permute(1, 0, 2).reshape(NL, D).cpu()
        ea[b, NL] = dq[b * nh:(b + 1) * nh, r].reshape(D).double().cpu()
        ex[b, :NL] = xn[b].double().view(NL, l, D).sum(1).cpu()
        ex[b, NL] = xn[b, r].double().cpu()
    assert _rel(Aq.cpu(), ea) < 1e-6 and _rel(Xs.cpu(), ex) < 1e-6
    assert (Aq[:, NL + 1:] == 0).all() and (Xs[:, NL + 1:] == 0).all()


@pytest.mark.parametrize("deferred", [False, True])
@pytest.mark.parametrize("nbags,n", [(1, 8448), (2, 1024)])
def test_a1_bwd_bf16_landmark_and_y_grads_vs_fp64(nbags, n, deferred):
    """The bf16 A1 backward's key-side sums against fp64: dk~ = dS^T q and dY = P^T dO with
    P = exp(q k~^T - lse), dS = P o (dO Y^T - D).  Its per-workgroup partials are bf16 slabs
    (rounded once each, summed in fp32 in index order by the flush); checked through the immediate
    reduce and through a caller-owned queue flushed afterwards (the engine's deferred form), which
    must give the same bits."""
    L = _lib()
    import ctypes as C_
    from transmil_deepgraft_amd.engine import _p, _stream
    nh, nbh = 8, 8 * nbags
    g = torch.Generator(device="cpu").manual_seed(29 + n)
    q = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16)
    kl = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(torch.bfloat16)
    y = torch.randn(nbh, 256, 64, generator=g).to(torch.bfloat16)
    dm = (torch.randn(nbags, n, nh * 64, generator=g) * 0.1).to(torch.bfloat16)
    lse = torch.logsumexp(q.float() @ kl.float().transpose(1, 2), -1)
    d1 = torch.randn(nbh, n, generator=g) * 0.05
    qd, kd, yd, dmd, lsed, d1d = (t.to(DEV).contiguous() for t in (q, kl, y, dm, lse, d1))
    ws = L.query("tm_nys_a1_bwd_workspace", nbh, n, 256) // 4
    work = torch.empty(ws, device=DEV)
    dkl = torch.full((nbh, 256, 64), 3.0, device=DEV)
    dy = torch.full((nbh, 256, 64), 3.0, device=DEV)
    dq = torch.empty(nbh, n, 64, device=DEV)
    rq = C_.c_void_p(L.lib().tm_reduce_queue_create()) if deferred else None
    try:
        L.call("tm_nys_a1_bwd", 1, _p(qd), _p(dmd), _p(kd), _p(yd), _p(lsed), _p(d1d), nbh, nh, n, 256,
               _p(dq), _p(work), _p(dkl), _p(dy), 0, rq, _stream())
        if deferred:
            assert L.lib().tm_reduce_queue_pending(rq) == 2
            L.call("tm_reduce_flush", rq, _stream())
        torch.cuda.synchronize()
    finally:
        if deferred:
            L.lib().tm_reduce_queue_destroy(rq)
    # fp64 reference per head
    dO = dm.double().view(nbags, n, nh, 64).permute(0, 2, 1, 3).reshape(nbh, n, 64)
    qf, kf, yf = q.double(), kl.double(), y.double()
    P = torch.exp(qf @ kf.transpose(1, 2) - lse.double()[..., None])
    dS = P * (dO @ yf.transpose(1, 2) - d1.double()[..., None])
    ek = dS.transpose(1, 2) @ qf
    ey = P.transpose(1, 2) @ dO
    ak, ay = dkl.cpu(), dy.cpu()
    rk, ry = _rel(ak, ek), _rel(ay, ey)
    # bf16 partials (2^-9 each) over fp32 sums of bf16 products: well inside 4e-3 of the max
    assert rk < 4e-3 and ry < 4e-3, (rk, ry)
    test_a1_bwd_bf16_landmark_and_y_grads_vs_fp64.last = getattr(test_a1_bwd_bf16_landmark_and_y_grads_vs_fp64,
                                                                 "last", {})
    key = (nbags, n)
    prev = test_a1_bwd_bf16_landmark_and_y_grads_vs_fp64.last.get(key)
    if prev is not None:                       # the other reduce path: identical bits
        assert torch.equal(prev[0], ak) and torch.equal(prev[1], ay)
    test_a1_bwd_bf16_landmark_and_y_grads_vs_fp64.last[key] = (ak, ay)


@pytest.mark.parametrize("nbags,n", [(1, 1024), (2, 512)])
def test_a1_bwd_dqkv_bf16_path_equals_the_fp32_dq_path(nbags, n):
    """The bf16 layer-1 path (tm_nys_a1_bwd_dqkv: bf16(scale dq) straight into dqkv, then
    tm_nys_assemble_q_slab_inplace adds the landmark term and rounds again) against the fp32 dq path
    (tm_nys_a1_bwd + tm_nys_assemble_q_slab, one rounding): dk~ and dY bitwise equal, the q columns
    within one bf16 ulp of the single-rounding result (the extra rounding), the k / v columns of dqkv
    untouched (the double rounding had only end-to-end gradient tolerances)."""
    L = _lib()
    from transmil_deepgraft_amd._lib import BF16
    from transmil_deepgraft_amd.engine import _p, _stream
    nh, nbh, scale, slabs = 8, 8 * nbags, 0.125, 3
    g = torch.Generator(device="cpu").manual_seed(11 + n)
    q = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16)
    kl = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(torch.bfloat16)
    y = torch.randn(nbh, 256, 64, generator=g).to(torch.bfloat16)
    dm = (torch.randn(nbags, n, nh * 64, generator=g) * 0.1).to(torch.bfloat16)
    lse = torch.logsumexp(q.float() @ kl.float().transpose(1, 2), -1)          # a consistent softmax
    d1 = torch.randn(nbh, n, generator=g) * 0.05
    dql = torch.randn(nbh, 256, 64, generator=g) * 0.1
    slab = (torch.randn(slabs, nbh, 256, 64, generator=g) * 0.1).to(torch.bfloat16)
    qd, kd, yd, dmd, lsed, d1d, dqld, slabd = (t.to(DEV).contiguous() for t in (q, kl, y, dm, lse, d1, dql, slab))
    ws = L.query("tm_nys_a1_bwd_workspace", nbh, n, 256) // 4
    sentinel = 7.0
    out = {}
    for path in ("dqkv", "fp32"):
        dqkv = torch.full((nbags, n, 3 * nh * 64), sentinel, dtype=torch.bfloat16, device=DEV)
        work = torch.empty(ws, device=DEV)
        dkl = torch.empty(nbh, 256, 64, device=DEV)
        dy = torch.empty(nbh, 256, 64, device=DEV)
        if path == "dqkv":
            L.call("tm_nys_a1_bwd_dqkv", _p(qd), _p(dmd), _p(kd), _p(yd), _p(lsed), _p(d1d), nbh, nh, n, _p(dqkv),
                   C.c_float(scale), _p(work), _p(dkl), _p(dy), None, _stream())
            L.call("tm_nys_assemble_q_slab_inplace", _p(dqld), _p(slabd), slabs, nbags, nh, n, C.c_float(scale),
                   _p(dqkv), _stream())
        else:
            dq = torch.empty(nbh, n, 64, device=DEV)
            L.call("tm_nys_a1_bwd", BF16, _p(qd), _p(dmd), _p(kd), _p(yd), _p(lsed), _p(d1d), nbh, nh, n, 256,
                   _p(dq), _p(work), _p(dkl), _p(dy), 0, None, _stream())
            L.call("tm_nys_assemble_q_slab", BF16, _p(dq), -1, _p(dqld), _p(slabd), slabs, nbags, nh, n,
                   C.c_float(scale), _p(dqkv), _stream())
            # scale * dq in dqkv's q-column layout: the value the bf16 path rounds first
            sdq = (scale * dq).view(nbags, nh, n, 64).permute(0, 2, 1, 3).reshape(nbags, n, nh * 64).cpu()
        torch.cuda.synchronize()
        out[path] = (dqkv.cpu().float(), dkl.cpu(), dy.cpu())
    a, b = out["dqkv"], out["fp32"]
    assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    qa, qb = a[0][..., :nh * 64], b[0][..., :nh * 64]
    assert torch.isfinite(qb).all() and qb.abs().max() > 0
    # the bf16 path rounds scale*dq to bf16 (half an ulp of that term) before the landmark term is
    # added and the sum rounded (half an ulp of the result, as the fp32 path's single rounding):
    # |a - b| <= ulp(scale dq) / 2 + ulp(b), ulp(x) = 2^(floor(log2 |x|) - 7)
    def ulp(x):
        return torch.exp2(torch.floor(torch.log2(x.abs().clamp_min(1e-30))) - 7)
    bound = 0.5 * ulp(sdq) + ulp(qb)
    assert ((qa - qb).abs() <= bound * 1.0001 + 1e-30).all(), ((qa - qb).abs() - bound).max()
    assert (a[0][..., nh * 64:] == sentinel).all()
