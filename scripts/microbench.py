"""Per-kernel timing of the HIP entry points with HIP events (one process, interleaved rounds).

    python scripts/microbench.py [--n 8192] [--reps 50]

Each case is run `reps` times between two events on the current stream; the
median of 5 rounds is printed.  Used to A/B kernel variants on the GPU box: it runs on the
diagnostic build (`make -C transmil_deepgraft_amd/csrc diag`), whose tm_debug_* switches select
the variants; the product library has none.
"""
import argparse
import ctypes as C
import math
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("TRANSMIL_HIP_LIB", os.path.join(ROOT, "transmil_deepgraft_amd", "libtransmil_hip_diag.so"))

from transmil_deepgraft_amd import _lib  # noqa: E402
from transmil_deepgraft_amd import engine as E  # noqa: E402
from transmil_deepgraft_amd._lib import BF16, F32  # noqa: E402


def timeit(fn, reps, graph=True):
    """GPU time per call: `reps` calls captured in one hipGraph and replayed, so the
    Python/launch cost of a call does not hide short kernels (eager if graph=False)."""
    fn()
    torch.cuda.synchronize()
    g = None
    if graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fn()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
    out = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        if g is not None:
            g.replay()
        else:
            for _ in range(reps):
                fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / reps * 1e3)
    return statistics.median(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default="")
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="a1_fwd in-kernel s_memtime stamps")
    ap.add_argument("--gemm-ab", action="store_true", help="also time the GEMMs on the register-staged loop")
    ap.add_argument("--split-stamps", action="store_true", help="per-wave s_memtime stamps of the split pinv chain")
    args = ap.parse_args()
    dev = "cuda"
    N = args.n
    G = math.ceil(math.sqrt(N))
    S = G * G + 1
    n = (S + 255) // 256 * 256
    nbh = 8
    bf = torch.bfloat16
    res = {}

    tag = [""]

    def case(name, fn, flops=None, byts=None):
        name = tag[0] + name
        if args.only and args.only not in name:
            return
        us = timeit(fn, args.reps, graph=not args.eager)
        extra = ""
        if flops:
            extra += f" {flops / us / 1e6:8.1f} TF/s"
        if byts:
            extra += f" {byts / us / 1e3:8.1f} GB/s"
        res[name] = us
        print(f"{name:40s} {us:9.2f} us{extra}", flush=True)

    st = E._stream
    if not args.only or args.only == "xcc":
        for nb, th in ((512, 512), (64, 256), (1024, 256)):
            xm = torch.zeros(nb, dtype=torch.int32, device=dev)
            _lib.call("tm_debug_xcc_map", E._p(xm), nb, th, st())
            torch.cuda.synchronize()
            v = xm.cpu().tolist()
            same = sum(1 for b in range(8, nb) if v[b] == v[b - 8]) / max(nb - 8, 1)
            print(f"xcc map {nb}x{th}: first 24 {v[:24]}  frac(b, b+8 same XCD)={same:.3f}", flush=True)
    # ---------------- bmm (pinv building block) ----------------
    X = torch.softmax(torch.randn(nbh, 256, 256, device=dev), -1)
    Z = torch.randn(nbh, 256, 256, device=dev) * 1e-2
    P = torch.empty_like(Z)
    W = torch.randn(nbh, 256, 64, device=dev)
    Y = torch.empty(nbh, 256, 64, device=dev)
    f = 2 * nbh * 256 ** 3
    Y2 = torch.randn(nbh, 256, 256, device=dev)
    Z2 = torch.empty_like(Z)
    case("bmm NN 256^3 x8", lambda: E.bmm([E.bmm_job(X, 0, Z, 0, P, 256, 256, 256)], nbh), f)
    case("bmm NT 256^3 x8", lambda: E.bmm([E.bmm_job(X, 0, Z, 1, P, 256, 256, 256)], nbh), f)
    case("bmm TN 256^3 x8", lambda: E.bmm([E.bmm_job(X, 1, Z, 0, P, 256, 256, 256)], nbh), f)
    case("bmm 2-job 256^3 x8", lambda: E.bmm([E.bmm_job(X, 0, Z, 0, P, 256, 256, 256),
                                              E.bmm_job(Z, 1, X, 0, Y.new_empty(nbh, 256, 256), 256, 256, 256)], nbh), 2 * f)
    case("bmm NN 256^3 x8 [bf16x3]", lambda: E.bmm([E.bmm_job(X, 0, Z, 0, P, 256, 256, 256)], nbh, 1), f)
    case("bmm NT bf16x3", lambda: E.bmm([E.bmm_job(X, 0, Z, 1, P, 256, 256, 256)], nbh, 1), f)
    case("bmm TN bf16x3", lambda: E.bmm([E.bmm_job(X, 1, Z, 0, P, 256, 256, 256)], nbh, 1), f)
    case("bmm Y=ZW bf16x3", lambda: E.bmm([E.bmm_job(Z, 0, W, 0, Y, 256, 64, 256)], nbh, 1), f // 4)
    case("bmm dependent pair bf16x3 (per bmm)", lambda: (E.bmm([E.bmm_job(X, 0, Z, 0, P, 256, 256, 256)], nbh, 1),
                                                        E.bmm([E.bmm_job(X, 0, P, 0, Z2, 256, 256, 256)], nbh, 1)), 2 * f)
    case("bmm NN+E1 bf16x3", lambda: E.bmm([E.bmm_job(X, 0, Z, 0, P, 256, 256, 256, E1=Y2, e1=1.0)], nbh, 1), f)
    case("bmm 2-job 256^3 x8 [bf16x3]", lambda: E.bmm([E.bmm_job(X, 0, Z, 0, P, 256, 256, 256),
                                              E.bmm_job(Z, 1, X, 0, Y.new_empty(nbh, 256, 256), 256, 256, 256)], nbh, 1), 2 * f)
    case("bmm Y=ZW 256x64x256 x8", lambda: E.bmm([E.bmm_job(Z, 0, W, 0, Y, 256, 64, 256)], nbh), f // 4)
    case("torch bmm fp32 256^3 x8", lambda: torch.bmm(X, Z, out=P), f)
    saved = torch.empty(_lib.query("tm_pinv_saved_floats", nbh, 6), device=dev)
    pwork = torch.empty(_lib.query("tm_pinv_bwd_workspace_floats", nbh), device=dev)
    pdz = torch.randn(nbh, 256, 256, device=dev) * 1e-3
    pdX = torch.empty(nbh, 256, 256, device=dev)
    case("pinv_fwd fp32", lambda: _lib.call("tm_pinv_fwd", E._p(X), nbh, 6, 0, E._p(saved), st()), 24 * f)
    case("pinv_fwd bf16x3 (fp32 storage)", lambda: _lib.call("tm_pinv_fwd", E._p(X), nbh, 6, 1, E._p(saved), st()),
         24 * f)
    case("pinv_bwd bf16x3 (fp32 storage)", lambda: _lib.call("tm_pinv_bwd", E._p(X), nbh, 6, 1, E._p(saved),
                                                              E._p(pdz), E._p(pwork), E._p(pdX), st()), 28 * f)
    # split-operand chain (pinv_split.hip): 14 launches forward, 4 per iteration + 2 backward
    Xs = torch.empty(2 * nbh * 65536, dtype=torch.bfloat16, device=dev)
    _lib.call("tm_split_f32", E._p(X), E._p(Xs), nbh * 65536, st())
    ssaved = torch.empty(_lib.query("tm_pinv_split_saved_floats", nbh, 6), device=dev)
    swork = torch.empty(_lib.query("tm_pinv_bwd_split_workspace_floats", nbh), device=dev)
    sout = torch.empty(nbh, 256, 256, device=dev)
    sdz = torch.empty(2 * nbh * 65536, dtype=torch.bfloat16, device=dev)
    _lib.call("tm_split_f32", E._p(pdz), E._p(sdz), nbh * 65536, st())
    for v, nm in ((0, "per-level launches"), (8, "persistent team"), (9, "team, plain DMA (probe)")):
        _lib.lib().tm_debug_set_split_variant(v)
        case(f"pinv_fwd split [{nm}]", lambda: _lib.call("tm_pinv_fwd_split", E._p(X), E._p(Xs), nbh, 6,
                                                           E._p(ssaved), st()), 24 * f)

        def bwd():
            swork[:2 * nbh * 65536 // 2].view(torch.bfloat16).copy_(sdz)
            _lib.call("tm_pinv_bwd_split", E._p(X), E._p(Xs), nbh, 6, E._p(ssaved), E._p(swork), 1, E._p(sout), st())
        case(f"pinv_bwd split [{nm}]", bwd, 48 * f)
    _lib.lib().tm_debug_set_split_variant(0)
    if args.split_stamps:
        import numpy as np
        # workgroups per launch: L1 (S + abs sums), A_0, B_0, (A_k, B_k) k=1..4, A_5, B_5, F
        t16 = 16 * nbh
        wgs = [2 * t16, t16, 2 * t16] + [2 * t16] * 8 + [2 * t16, t16, t16]
        nl = len(wgs)
        buf = torch.zeros(sum(wgs) * 4 * 8, dtype=torch.int64, device=dev)
        for rep in range(3):  # the third run is measured (warm caches)
            buf.zero_()
            _lib.lib().tm_debug_set_split_stamps(C.c_void_p(buf.data_ptr()))
            _lib.call("tm_pinv_fwd_split", E._p(X), E._p(Xs), nbh, 6, E._p(ssaved), st())
            _lib.lib().tm_debug_set_split_stamps(None)
            torch.cuda.synchronize()
        a = buf.cpu().numpy()
        off = 0
        prev_end = None
        names = ["setup", "wait c0", "chunk0", "chunks1+", "epilogue"]
        print("split pinv_fwd stamps: per launch, medians over waves (shader cycles); realtime in us")
        for li in range(nl):
            nwg = wgs[li]
            seg = a[off:off + nwg * 32].reshape(nwg, 4, 8)
            off += nwg * 32
            seg = seg[seg[:, 0, 7] > 0]  # product workgroups (abs-sum ones do not stamp)
            rt0, rt1 = seg[:, :, 0].min(), seg[:, :, 7].max()
            d = np.diff(seg[:, :, 1:7].astype(np.int64), axis=2)
            med = [int(np.median(d[:, :, i])) for i in range(5)]
            mx = [int(np.max(d[:, :, i])) for i in range(5)]
            gap = (rt0 - prev_end) / 100.0 if prev_end is not None else float("nan")
            startspread = (seg[:, :, 0].max() - rt0) / 100.0
            print(f"  launch {li:2d} ({nwg} wg): span {(rt1 - rt0) / 100.0:6.2f} us  gap {gap:6.2f} us  start spread "
                  f"{startspread:5.2f} us  " + "  ".join(f"{n} {m}/{x}" for n, m, x in zip(names, med, mx)))
            prev_end = rt1
    _lib.call("tm_split_f32", E._p(pdz), E._p(swork), nbh * 65536, st())
    case("pinv_bwd split (+softmax bwd)", lambda: _lib.call("tm_pinv_bwd_split", E._p(X), E._p(Xs), nbh, 6,
                                                            E._p(ssaved), E._p(swork), 1, E._p(sout), st()), 32 * f)
    for gv in ((0, 1, 2, 4, 7) if args.gemm_ab else (0,)):
        _lib.lib().tm_debug_set_variant(2, gv)
        tag[0] = {0: "", 1: "[2 LDS buf] ", 2: "[4-stage ring] ", 4: "[persistent ring] ", 7: "[big tile] "}[gv]
        # ---------------- GEMMs ----------------
        pool = E.Pool(dev)
        xn = torch.randn(n, 512, device=dev).to(bf)
        wqkv = (torch.randn(1536, 512, device=dev) * 0.05).to(bf)
        qkv = torch.empty(3, nbh, n, 64, device=dev, dtype=bf)
        case("gemm qkv (NT, scatter)", lambda: E.gemm(xn, wqkv, qkv, n, 1536, 512, lda=512, ldb=512, ldc=0, dtype=BF16,
                                                      qkv=(1, 8, 64, n, 0.125)), 2 * n * 1536 * 512)
        slabq = torch.empty(n, 1536, device=dev)

        def plain_gemm(K_):
            g = _lib.GemmArgs()
            g.M, g.N, g.K = n, 1536, K_
            g.lda, g.ldb, g.ldc = 512, 512, 1536
            g.ab_dtype, g.c_dtype = BF16, F32
            g.splits, g.k_per_split = 1, 512
            g.mode = _lib.EPI_SPLITK
            g.alpha = 1.0
            _lib.call("tm_gemm", E._p(xn), E._p(wqkv), E._p(slabq), C.byref(g), st())
        case("gemm qkv shape, plain fp32 store", lambda: plain_gemm(512), 2 * n * 1536 * 512)
        case("gemm qkv shape, K=64 plain store", lambda: plain_gemm(64), 2 * n * 1536 * 64)
        outb = torch.empty(n, 1536, device=dev, dtype=bf)
        case("torch.matmul bf16 (hipBLASLt) qkv", lambda: torch.matmul(xn, wqkv.t(), out=outb), 2 * n * 1536 * 512)
        H = torch.randn(S, 512, device=dev)
        Ho = torch.empty_like(H)
        wo = (torch.randn(512, 512, device=dev) * 0.05).to(bf)
        bo = torch.randn(512, device=dev)
        case("gemm to_out (NT, drop+resid)", lambda: E.gemm(xn, wo, Ho, n, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16,
                                                            c_dtype=F32, bias=bo, drop_p=0.7, seed=3, resid=H,
                                                            rowmap=(n, n - S, S, 0, 0, 0)), 2 * n * 512 * 512)
        case("gemm to_out shape, bias only", lambda: E.gemm(xn, wo, Ho, n, 512, 512, lda=512, ldb=512, ldc=512,
                                                            dtype=BF16, c_dtype=F32, bias=bo), 2 * n * 512 * 512)
        case("torch.matmul bf16 to_out shape", lambda: torch.matmul(xn, wo.t(), out=outb[:, :512]), 2 * n * 512 * 512)
        dq = torch.randn(n, 1536, device=dev).to(bf)
        dx = torch.empty(n, 512, device=dev, dtype=bf)
        case("gemm dxn (B k-strided)", lambda: E.gemm(dq, wqkv, dx, n, 512, 1536, lda=1536, ldb=512, ldc=512, b_kn=1,
                                                      dtype=BF16), 2 * n * 1536 * 512)
        dW = torch.empty(1536, 512, device=dev)
        case("wgrad dWqkv (split-K + reduce)", lambda: E.weight_grad(dq, xn, dW, 1536, 512, n, ldy=1536, ldx=512,
                                                                     dtype=BF16, work_pool=pool), 2 * n * 1536 * 512)
        slab = torch.randn(8, 1536 * 512, device=dev)
        case("splitk_reduce 8 x 786K", lambda: _lib.call("tm_splitk_reduce", E._p(slab), E._p(dW), 8, 1536 * 512,
                                                         C.c_float(1.0), 0, None, st()), byts=9 * 1536 * 512 * 4)
        slab2 = torch.randn(33, 512, device=dev)
        ob = torch.empty(512, device=dev)
        nf = torch.empty(n * 1536, device=dev)
    case("torch fill 52 MB fp32", lambda: nf.fill_(1.0), byts=n * 1536 * 4)
    case("torch copy 52 MB fp32", lambda: slabq.view(-1).copy_(nf), byts=2 * n * 1536 * 4)
    case("splitk_reduce 33 x 512", lambda: _lib.call("tm_splitk_reduce", E._p(slab2), E._p(ob), 33, 512,
                                                         C.c_float(1.0), 0, None, st()))
    _lib.lib().tm_debug_set_variant(2, 0)
    tag[0] = ""

    # ---------------- NystromAttention core ----------------
    q = (torch.randn(nbh, n, 64, device=dev) * 0.3).to(bf)
    k = (torch.randn(nbh, n, 64, device=dev) * 0.3).to(bf)
    v = torch.randn(nbh, n, 64, device=dev).to(bf)
    ql = torch.randn(nbh, 256, 64, device=dev) * 0.3
    kl = torch.randn(nbh, 256, 64, device=dev) * 0.3
    ql_t, kl_t = ql.to(bf), kl.to(bf)
    qkv3 = torch.stack([q, k, v])
    case("landmarks", lambda: _lib.call("tm_nys_landmarks", BF16, E._p(q), E._p(k), nbh, n, E._p(ql), E._p(kl),
                                        E._p(ql_t), E._p(kl_t), st()), byts=2 * nbh * n * 64 * 2)
    a3w = torch.empty(_lib.query("tm_nys_a3_workspace", nbh, n) // 4, device=dev)
    w_ = torch.empty(nbh, 256, 64, device=dev)
    lse3 = torch.empty(nbh, 256, device=dev)
    case("a3_fwd (+combine)", lambda: _lib.call("tm_nys_a3_fwd", BF16, E._p(ql), E._p(k), E._p(v), nbh, n, E._p(a3w),
                                                E._p(w_), E._p(lse3), st()), 4 * nbh * 256 * n * 64)
    y_t = torch.randn(nbh, 256, 64, device=dev).to(bf)
    wconv = torch.randn(8, 33, device=dev) * 0.1
    merged = torch.empty(1, n, 512, device=dev, dtype=bf)
    lse1 = torch.empty(nbh, n, device=dev)
    case("a1_fwd", lambda: _lib.call("tm_nys_a1_fwd", BF16, E._p(q), E._p(v), E._p(kl_t), E._p(y_t), E._p(wconv),
                                     nbh, 8, n, E._p(merged), E._p(lse1), st()),
         4 * nbh * n * 256 * 64, 3 * n * 512 * 2)
    for var, nm in ((11, "no conv"), (12, "no attention"), (13, "prologue only"),
                    (14, "legacy 128-query kernel")):
        _lib.lib().tm_debug_set_variant(1, var)
        case(f"a1_fwd [{nm}]", lambda: _lib.call("tm_nys_a1_fwd", BF16, E._p(q), E._p(v), E._p(kl_t), E._p(y_t),
                                                E._p(wconv), nbh, 8, n, E._p(merged), E._p(lse1), st()))
    if args.stamps:
        _lib.lib().tm_debug_set_variant(1, 19)
        _lib.call("tm_nys_a1_fwd", BF16, E._p(q), E._p(v), E._p(kl_t), E._p(y_t), E._p(wconv), nbh, 8, n,
                  E._p(merged), E._p(lse1), st())
        torch.cuda.synchronize()
        import numpy as np
        buf = (C.c_ulonglong * (256 * 64))()
        _lib.call("tm_debug_a1_stamps", buf, 256 * 64)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(256, 8, 8).astype(np.int64)[:, :4]
        t0 = a[:, :, 0].min()
        print("a1_fwd stamps (cycles from first start): slot medians / maxima over waves")
        names = ["start", "prologue", "attn1", "window", "conv1", "stores1", "end"]
        for slot in range(7):
            rel = a[:, :, slot] - a[:, :, 0]   # per wave, from its own start (XCD clocks differ)
            ok = a[:, :, slot] > 0
            vals = rel[ok]
            if vals.size:
                print(f"  {slot} {names[slot]:9s} median {int(np.median(vals)):7d} max {int(vals.max()):7d}")
        d = a[:, :, 6] - a[:, :, 0]
        print(f"  wave lifetime median {int(np.median(d))} max {int(d.max())}; "
              f"last end - first start {int(a[:, :, 6].max() - t0)}")
    _lib.lib().tm_debug_set_variant(1, 0)
    dmerged = torch.randn(1, n, 512, device=dev).to(bf)
    dv = torch.empty(nbh, n, 64, device=dev)
    d1 = torch.empty(nbh, n, device=dev)
    cw = torch.empty(_lib.query("tm_nys_conv_bwd_workspace", 1, 8, n) // 4, device=dev)
    dwc = torch.empty(8, 33, device=dev)
    case("conv_bwd", lambda: _lib.call("tm_nys_conv_bwd", BF16, E._p(dmerged), E._p(merged), E._p(v), E._p(wconv),
                                       nbh, 8, n, E._p(dv), E._p(d1), E._p(cw), E._p(dwc), None, st()),
         byts=4 * n * 512 * 2)
    dqf = torch.empty(nbh, n, 64, device=dev)
    a1w = torch.empty(_lib.query("tm_nys_a1_bwd_workspace", nbh, n, 256) // 4, device=dev)
    dkl = torch.empty(nbh, 256, 64, device=dev)
    dy = torch.empty(nbh, 256, 64, device=dev)
    lse1.uniform_(3, 4)
    case("a1_bwd (+2 reduces)", lambda: _lib.call("tm_nys_a1_bwd", BF16, E._p(q), E._p(dmerged), E._p(kl_t),
                                                  E._p(y_t), E._p(lse1), E._p(d1), nbh, 8, n, 256, E._p(dqf),
                                                  E._p(a1w), E._p(dkl), E._p(dy), 0, None, st()), 10 * nbh * n * 256 * 64)
    a3bw = torch.empty(_lib.query("tm_nys_a3_bwd_workspace", nbh, n) // 4, device=dev)
    d3 = torch.randn(2, nbh, 256, device=dev)   # [2][nbh][256] partials
    dw_t = torch.randn(nbh, 256, 64, device=dev).to(bf)
    dk = torch.empty(nbh, n, 64, device=dev)
    dql = torch.zeros(nbh, 256, 64, device=dev)
    lse3.uniform_(8, 9)
    case("a3_bwd (+reduce)", lambda: _lib.call("tm_nys_a3_bwd", BF16, E._p(ql_t), E._p(dw_t), E._p(k), E._p(v),
                                               E._p(lse3), E._p(d3), nbh, 8, n, E._p(dk), E._p(dv), E._p(a3bw),
                                               E._p(dql), 1, None, st()), 10 * nbh * n * 256 * 64)
    zz = torch.randn(nbh, 256, 256, device=dev) * 1e-2
    arow = torch.empty(nbh, n, device=dev)
    case("attn_row (return_attn row)", lambda: _lib.call("tm_nys_attn_row", BF16, E._p(q), E._p(k), E._p(ql), E._p(kl),
                                                         E._p(zz), E._p(lse3), nbh, n, 167, E._p(arow), st()),
         2 * nbh * n * 256 * 64)
    if args.only == "overlap":
        # pinv backward chain beside the A3 backward on a second stream (fork / join in one graph)
        saved8 = torch.empty(_lib.query("tm_pinv_saved_floats", nbh, 6), device=dev)
        X8 = torch.softmax(torch.randn(nbh, 256, 256, device=dev), -1)
        _lib.call("tm_pinv_fwd", E._p(X8), nbh, 6, 1, E._p(saved8), st())
        pw = torch.empty(_lib.query("tm_pinv_bwd_workspace_floats", nbh), device=dev)
        dz8 = torch.randn(nbh, 256, 256, device=dev) * 1e-3
        dX8 = torch.empty(nbh, 256, 256, device=dev)
        side = torch.cuda.Stream()

        def chain():
            _lib.call("tm_pinv_bwd", E._p(X8), nbh, 6, 1, E._p(saved8), E._p(dz8), E._p(pw), E._p(dX8), st())

        def a3():
            _lib.call("tm_nys_a3_bwd", BF16, E._p(ql_t), E._p(dw_t), E._p(k), E._p(v), E._p(lse3), E._p(d3), nbh, 8,
                      n, E._p(dk), E._p(dv), E._p(a3bw), E._p(dql), 1, None, st())

        def both():
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                a3()
            chain()
            torch.cuda.current_stream().wait_stream(side)

        args.only = ""
        case("overlap: pinv_bwd alone", chain)
        case("overlap: a3_bwd alone", a3)
        case("overlap: serial", lambda: (chain(), a3()))
        case("overlap: a3_bwd on a side stream", both)
        return
    # ---------------- PPEG ----------------
    x = torch.randn(1, S, 512, device=dev)
    wf = torch.randn(512 * 49, device=dev) * 0.1
    bfo = torch.randn(512, device=dev)
    yp = torch.empty_like(x)
    case("ppeg_fwd", lambda: _lib.call("tm_ppeg_fwd", E._p(x), 1, G, 512, E._p(wf), E._p(bfo), E._p(yp), st()),
         byts=2 * S * 512 * 4)


if __name__ == "__main__":
    main()
